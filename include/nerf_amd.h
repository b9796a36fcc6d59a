/*
 * nerf_amd.h -- C ABI of the MI355X (gfx950) NeRF render-and-train hot path.
 *
 * Library: nerf-replication_amd/nerf_amd/libnerf_amd.so (hipcc --offload-arch=gfx950).
 *
 * Conventions (every entry point):
 *   - plain device pointers + sizes + an explicit hipStream_t; no torch types;
 *   - returns int status: 0 ok, -22 bad argument, <= -1000 a HIP launch error
 *     (-1000 - hipError_t); nerf_last_error() gives a thread-local message;
 *   - no allocation and no host synchronisation inside (graph-capturable); the caller
 *     owns every buffer (sizes from the *_bytes() helpers);
 *   - re-entrant; no mutable global state.
 *
 * Each entry point replaces an ATen op sequence of echo636/nerf-replication; the
 * reference interface it stands in for is cited per function (paths relative to the
 * reference repository).  Float arithmetic that fixes sample positions and indices is
 * done with separately rounded IEEE ops, so those match the reference bit for bit on
 * identical inputs.
 */
#ifndef NERF_AMD_H
#define NERF_AMD_H

#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NERF_DTYPE_F32 0
#define NERF_DTYPE_BF16 1
#define NERF_DTYPE_BF16X3 2 /* fp32 operands split into bf16 hi + lo: three bf16 MFMAs per product */
#define NERF_DTYPE_BF16X3F 3 /* the bf16x3 forward (outputs bit-identical to bf16x3) + the bf16 backward */
#define NERF_DTYPE_BF16X6 4  /* inference forward only: operands split into three bf16, six products */

#define NERF_MLP_STORE 1   /* keep activations + ReLU masks for backward */
#define NERF_MLP_DENSITY 2 /* sigma only (grid bake) */

const char* nerf_last_error(void);
int nerf_abi_version(void);

/* ---- (a1/a2) rays ---------------------------------------------------------------------
 * Replaces Dataset.get_rays (src/datasets/nerf/blender.py:13-32) and the train-batch ray
 * gather (blender.py:124-131).  Pixel id = img*H*W + j*W + i.  pix == NULL draws ids
 * uniformly from a Philox stream (seed, offset).  images [n_img,H,W,3] (optional) gives
 * the ground-truth rgb gather. */
int nerf_raygen(const float* c2w, int n_img, int H, int W, float focal, const int64_t* pix, int64_t R,
                uint64_t seed, uint64_t offset, const float* images, float* rays, float* rgb, int64_t* pix_out,
                hipStream_t stream);

/* ---- (a3) stratified depths --------------------------------------------------------------
 * Replaces Renderer.render :165-187 (linspace, perturb, pts = o + d z, viewdirs = d/|d|).
 * t_lin = torch.linspace(0,1,S) computed on the host CPU; near/far are device scalars.
 * t_rand == NULL with perturb draws the jitter from Philox (seed, offset). */
int nerf_sample_stratified(const float* rays, int64_t R, int S, const float* t_lin, const float* near,
                           const float* far, int perturb, const float* t_rand, uint64_t seed, uint64_t offset,
                           float* z, float* pts, float* viewdirs, hipStream_t stream);

/* ---- (a8) searchsorted(right=True), wave-level, one row per wave (nb <= 64) --------------
 * Replaces torch.searchsorted in Renderer.sample_pdf (volume_renderer.py:117). */
int nerf_searchsorted(const float* cdf, const float* u, int64_t R, int nb, int n, int32_t* inds,
                      hipStream_t stream);

/* ---- (a8/a9) importance sampling + merge --------------------------------------------------
 * Replaces Renderer.sample_pdf (volume_renderer.py:82-134) on z_mid / weights[...,1:-1] and
 * the sort(cat(z, z_samples)) + pts_f of render() (:205-221).  det uses u_lin =
 * torch.linspace(0,1,Ni) (host CPU table).  Optional outputs: samples (u order), the CDF and
 * the searchsorted indices. */
int nerf_sample_pdf(const float* z, const float* weights, int64_t R, int Sc, int Ni, int det, const float* u_lin,
                    const float* u, uint64_t seed, uint64_t offset, const float* rays, float* z_fine,
                    float* pts_fine, float* samples, float* cdf_out, int32_t* inds_out, hipStream_t stream);

/* Same algorithm with the reference's own signature: bins [R,nb] (z mids) and pdf weights
 * [R,nb-1] -> samples [R,Ni] in u order (volume_renderer.py:82-134). */
int nerf_sample_pdf_bins(const float* bins, const float* weights, int64_t R, int nb, int Ni, int det,
                         const float* u_lin, const float* u, uint64_t seed, uint64_t offset, float* samples,
                         float* cdf_out, int32_t* inds_out, hipStream_t stream);

/* ---- (a7) alpha compositing -----------------------------------------------------------------
 * Replaces Renderer.raw2outputs (volume_renderer.py:20-80) and its autograd backward.
 * dirs: ray directions with row stride dir_stride floats (6 when passing rays [R,6]). */
int nerf_composite_fwd(const float* raw, const float* z, const float* dirs, int dir_stride, int64_t R, int S,
                       int white_bkgd, float* rgb, float* depth, float* acc, float* weights, hipStream_t stream);
int nerf_composite_bwd(const float* raw, const float* z, const float* dirs, int dir_stride, int64_t R, int S,
                       int white_bkgd, const float* g_rgb, const float* g_depth, const float* g_acc, float* g_raw,
                       hipStream_t stream);
/* The coarse pass's compositing and the importance sampling + merge that reads its weights, in one
 * launch (volume_renderer.py:197-221; the weights handed over in registers): the outputs of
 * nerf_composite_fwd (S = Sc <= 64; weights nullable) and of nerf_sample_pdf (z_fine, pts_fine),
 * bit-identical to the two separate launches. */
int nerf_composite_pdf(const float* raw, const float* z, const float* dirs, int dir_stride, int64_t R, int Sc,
                       int white_bkgd, float* rgb, float* depth, float* acc, float* weights, int Ni, int det,
                       const float* u_lin, const float* u, uint64_t seed, uint64_t offset, const float* rays,
                       float* z_fine, float* pts_fine, hipStream_t stream);
/* (ABI 4) nerf_composite_pdf at det (u = u_lin, the linspace of volume_renderer.py:96-99) that also flags
 * "fragile" rays: fragile[r] = 1 when an importance sample's bin (searchsorted) could change if every CDF entry c
 * moved by up to rel_tol * min(c, 1 - c) + abs_tol, or the den of its interval is within den_tol of the
 * den < 1e-5 switch (volume_renderer.py:120-126; den_tol 0: not flagged), or (z_tol > 0) those CDF moves
 * could move a sample within its bin by more than z_tol -- the rays whose fine samples a slightly different
 * coarse MLP could move.  The render of the split-bf16 tiers evaluates its coarse net in the tier's own arithmetic and
 * re-evaluates only these rays at fp32 (Renderer.render). */
int nerf_composite_pdf_fragile(const float* raw, const float* z, const float* dirs, int dir_stride, int64_t R, int Sc,
                               int white_bkgd, float* rgb, float* depth, float* acc, int Ni, const float* u_lin,
                               const float* rays, float* z_fine, float* pts_fine, float rel_tol, float abs_tol,
                               float den_tol, float z_tol, int32_t* fragile, hipStream_t stream);

/* ---- (a10) loss: MSE(rgb_map_c, gt) + MSE(rgb_map_f, gt) (src/train/trainers/nerf.py:21-29) -----
 * n = 3 R values.  fwd: out[3] = (loss_c, loss_f, loss_c + loss_f), one workgroup, fp64 sums in a
 * fixed order (run-to-run identical); f nullable.  The losses are the correctly rounded means, so
 * they can differ in the last bits from nn.MSELoss's fp32 CPU reduction: they are logged only --
 * the backward needs no forward value, and its gradients equal torch's bit for bit.  bwd: gc = (2/n) (c - gt) (g_lc + g_total), gf = (2/n) (f - gt) (g_lf +
 * g_total) with device-scalar output grads (null = 0), ATen's rounding order. */
int nerf_mse2_fwd(const float* c, const float* f, const float* gt, int64_t n, float* out, hipStream_t stream);
int nerf_mse2_bwd(const float* c, const float* f, const float* gt, int64_t n, const float* g_lc, const float* g_lf,
                  const float* g_total, float* gc, float* gf, hipStream_t stream);

/* ---- (a4-a6) fused PE + NeRF MLP ------------------------------------------------------------
 * Replaces Network.forward / NeRF.forward (src/models/nerf/network.py:49-74, 171-192) with
 * the frequency encoders (src/models/encoding/freq.py:7-32), and their autograd backward.
 * params: host array of 24 device pointers in state_dict order of one NeRF
 * (pts_linears.0..7.{weight,bias}, views_linears.0, feature_linear, alpha_linear,
 * rgb_linear), fp32 nn.Linear layout.  nerf_mlp_pack re-packs them (call after every
 * optimizer step); dir 0 = forward, 1 = backward (W^T).
 * fwd: raw [M,4] = (rgb logits, sigma pre-activation) for pts [M,3]; view direction of
 * sample m is viewdirs[dir_index ? dir_index[m] : m / samples_per_dir].
 * bwd: accumulates into grad[nerf_mlp_net_params()] (flat, state_dict order).
 * act / masks / dz are opaque workspaces of nerf_mlp_{act,mask,dz}_bytes(M) bytes written by the
 * training forward (flags & NERF_MLP_STORE) and the dX chain; their layouts are internal.
 * dtype: 0 = fp32 (fp32 MFMA, the reference's precision), 1 = bf16 (operands rounded to bf16),
 * 2 = bf16x3 (operands split into bf16 hi + lo, three bf16 MFMAs per product, fp32 accumulation),
 * 3 = bf16x3f: the bf16x3 forward (its outputs are bf16x3's, bit for bit) whose training stores are
 * the bf16 (hi) halves, and the bf16 backward (dX chain, dW).  Every function maps 3 to its part:
 * packed_bytes / pack dir 0 and fwd -> bf16x3, pack dir 1 / act / dz bytes / bwd -> bf16.
 * 4 = bf16x6, an inference forward only (x = hi + mid + lo, products hh hm mh hl lh mm, fp32 accumulation:
 * at least as accurate as fp32): packed_bytes / pack dir 0 and nerf_mlp_fwd with flags 0; everything else
 * rejects it.  Any other dtype: the size helpers return -1, every launching function -22 (nerf_last_error
 * names the dtype). */
int64_t nerf_mlp_net_params(void);
int64_t nerf_mlp_param_offset(int i);
int64_t nerf_mlp_packed_bytes(int dtype, int dir);
int64_t nerf_mlp_padded_samples(int64_t M);
int64_t nerf_mlp_act_bytes(int dtype, int64_t M);
int64_t nerf_mlp_dz_bytes(int dtype, int64_t M);
int64_t nerf_mlp_mask_bytes(int64_t M);
int64_t nerf_mlp_dw_items(int dtype, int64_t M);  /* workgroups of the dW launch */
int nerf_mlp_pack(const float* const* params, int dtype, void* packed_fwd, void* packed_bwd, hipStream_t stream);
int nerf_mlp_fwd(const void* packed_fwd, int dtype, const float* pts, const float* viewdirs, int samples_per_dir,
                 const int32_t* dir_index, int64_t M, int flags, float* raw, void* act, uint16_t* masks,
                 hipStream_t stream);
/* Inference forward whose sample count lives on the device: M = min(*M_dev, M_cap) is read by the
 * kernel (a persistent grid loops over the sample blocks), so a producer kernel's count -- the grid
 * march's gather -- sizes the launch without a host round trip.  raw: [M_cap,4]. */
int nerf_mlp_fwd_count(const void* packed_fwd, int dtype, const float* pts, const float* viewdirs, int samples_per_dir,
                       const int32_t* dir_index, const int32_t* M_dev, int64_t M_cap, float* raw, hipStream_t stream);
int nerf_mlp_bwd(const void* packed_bwd, int dtype, const float* d_raw, int64_t M, const void* act,
                 const uint16_t* masks, void* dz, float* grad, hipStream_t stream);
/* the two halves of nerf_mlp_bwd (dX chain kernel, dW/db GEMM kernel) as separate calls */
int nerf_mlp_bwd_dx(const void* packed_bwd, int dtype, const float* d_raw, int64_t M, const uint16_t* masks, void* dz,
                    hipStream_t stream);
/* nerf_mlp_bwd_dw (= the _ws form with workspace NULL) adds the work items' partial sums with fp32
 * atomics: NOT bit-reproducible run to run (the sum order varies).  The production path (ops.py,
 * DETERMINISTIC_DW) uses nerf_mlp_bwd_dw_ws with a workspace. */
int nerf_mlp_bwd_dw(int dtype, int64_t M, const void* act, const void* dz, float* grad, hipStream_t stream);
/* dW/db with a workspace of nerf_mlp_dw_workspace_bytes(dtype, M): each work item writes its partial
 * sums to its own slice and a second kernel adds them per parameter in a fixed order, so the gradient
 * is bit-reproducible run to run (workspace == NULL: fp32 atomics, as nerf_mlp_bwd_dw). */
int64_t nerf_mlp_dw_workspace_bytes(int dtype, int64_t M);
int nerf_mlp_bwd_dw_ws(int dtype, int64_t M, const void* act, const void* dz, float* grad, void* workspace,
                       hipStream_t stream);

/* ---- (a14) evaluator metrics (src/evaluators/nerf.py:23-45) --------------------------------------
 * pred / gt fp32 [H,W,3] on the device -> out (device, 4 doubles): PSNR of the float images,
 * SSIM of uint8(pred*255) vs uint8(gt*255) (7x7 uniform window, K1 0.01, K2 0.03, sample
 * covariance, data_range = max - min of the uint8 prediction, 3-pixel crop, mean over channels),
 * the sum of squared errors and the data range.  workspace: nerf_metrics_workspace_bytes(H, W). */
int64_t nerf_metrics_workspace_bytes(int H, int W);
int nerf_image_metrics(const float* pred, const float* gt, int H, int W, void* workspace, double* out,
                       hipStream_t stream);

/* ---- (a11) occupancy lookup ------------------------------------------------------------------
 * Replaces Renderer.world_to_grid_indices (volume_renderer.py:261-265) + the grid gather of
 * render_accelerated (:307-312).  bbox_host = {min xyz, max xyz} on the host. */
int nerf_grid_index(const float* pts, int64_t M, const float* bbox_host, int res, const uint8_t* grid,
                    int64_t* idx_out, uint8_t* occ_out, hipStream_t stream);

/* ---- (a13) grid bake (occupancy_grid.py:15-80) --------------------------------------------------
 * Points at the voxel corners (dedup = 1: the (res+1)^3 shared lattice, exact when
 * bmin + L * voxel is exact in fp32, as for the lego bbox; dedup = 0: res^3 x 8 corners as
 * the reference enumerates them), then the density-only MLP, then
 * occupied = any_corner(relu(sigma) > threshold). */
int64_t nerf_bake_num_points(int res, int dedup);
int nerf_bake_points(int res, const float* bbox_host, int dedup, float* pts, hipStream_t stream);
int nerf_bake_reduce(const float* raw, int res, int dedup, float threshold, uint8_t* grid, hipStream_t stream);
/* The same for the voxel slab x in [x0, x1) only (one slab per rank, the bool
 * grid all-gathered afterwards); grid is the slab [x1-x0][res][res]. */
int64_t nerf_bake_num_points_slab(int res, int dedup, int x0, int x1);
int nerf_bake_points_slab(int res, const float* bbox_host, int dedup, int x0, int x1, float* pts, hipStream_t stream);
int nerf_bake_reduce_slab(const float* raw, int res, int dedup, int x0, int x1, float threshold, uint8_t* grid,
                          hipStream_t stream);

/* ---- (a12) grid-accelerated march (render_accelerated, volume_renderer.py:268-357) --------------
 * Round structure: init; repeat { zero counters[0..1]; gather (<= K occupied steps per alive ray,
 * compacted points; a ray whose T < t_split gathers at most k_low; cap = room for points,
 * K <= cap <= INT32_MAX; a ray that finds no room keeps its position for the next round, and
 * every position below min(counters[0], cap) still holds a valid point; evaluated (nullable,
 * uint64) += that count); fine MLP on the points (nerf_mlp_fwd_count with M_dev = counters: no
 * host sync); composite (stops at T < t_thresh; consumed (nullable, uint64) += the points
 * composited, i.e. the reference's MLP queries -- points gathered past a ray's termination are
 * dropped) } until counters[1] (rays alive entering a round) is 0; finish (white background). */
int nerf_march_init(float* T, float* rgb, float* depth, float* acc, int32_t* next_step, uint8_t* alive,
                    uint8_t* exhausted, int64_t N, hipStream_t stream);
/* macro occupancy of 8^3 cell blocks (nullable input of the gather: an empty block is crossed in
 * one skip; exact, like the cell-level skip) */
int64_t nerf_march_macro_bytes(int res);
int nerf_march_macro(const uint8_t* grid, int res, uint8_t* macro, hipStream_t stream);
/* start_step_scratch: null = one pass (the counting walk records its points as runs of occupied
 * steps and writes them after the reservation; the default), or an [N] int32 workspace = the
 * two-pass form (a second walk writes the points).  Same outputs.  One pass needs n_steps < 65536. */
int nerf_march_gather(const float* rays, int64_t N, const float* t_table, int n_steps, const uint8_t* grid, int res,
                      const uint8_t* macro, const float* bbox_host, int K, int k_low, float t_split, float* T,
                      float* rgb, float* depth,
                      float* acc, int32_t* next_step, uint8_t* alive, uint8_t* exhausted, int32_t* counters,
                      unsigned long long* evaluated, int32_t* start_step_scratch, int32_t* out_ray, int32_t* out_step,
                      float* out_pts, int32_t* ray_off, int32_t* ray_cnt, int64_t cap, hipStream_t stream);
int nerf_march_composite(const float* raw, const float* rays, int64_t N, const float* t_table, const int32_t* ray_off,
                         const int32_t* ray_cnt, const int32_t* out_step, float* T, float* rgb, float* depth,
                         float* acc, int32_t* next_step, uint8_t* alive, uint8_t* exhausted, float step_size,
                         float t_thresh, unsigned long long* consumed, hipStream_t stream);
int nerf_march_finish(float* rgb, const float* acc, int64_t N, int white, hipStream_t stream);

/* ---- (a10) clip_grad_value_ + Adam (src/train/trainers/trainer.py:61-62, optimizer.py:8-28) ---- */
int nerf_adam_step(float* param, float* grad, float* exp_avg, float* exp_avg_sq, int64_t n, double lr, double beta1,
                   double beta2, double eps, int64_t step, double clip_value, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* NERF_AMD_H */
