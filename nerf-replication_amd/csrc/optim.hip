// Fused clip_grad_value_ + Adam step over flat parameter / gradient / moment buffers.
//
// Reference: src/train/trainers/trainer.py:61-62 (torch.nn.utils.clip_grad_value_(40),
// optimizer.step()) with src/train/optimizer.py:8-28 (torch.optim.Adam, one param group
// per tensor, lr 5e-4, betas (0.9, 0.999), eps 1e-8, weight_decay 0).  The reference runs
// ~48 x 10 small ATen kernels per step; here one launch updates all 1,191,688 values.
#include "common.h"

namespace nerf {

struct AdamArgs {
  float* p;
  float* g;
  float* m;
  float* v;
  int64_t n;
  float lr_over_bc1;     // lr / (1 - beta1^t)
  float inv_bc2_sqrt;    // 1 / sqrt(1 - beta2^t)  (used as division by sqrt(bc2))
  float bc2_sqrt;
  float beta1, beta2, eps, clip;
};

__global__ void adam_kernel(AdamArgs a) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n) return;
  float g = a.g[i];
  if (a.clip > 0.f) {
    g = fminf(fmaxf(g, -a.clip), a.clip);
    a.g[i] = g;
  }
  float m = a.m[i], v = a.v[i];
  m = fadd(m, fmul(1.f - a.beta1, fsub(g, m)));        // exp_avg.lerp_(grad, 1 - beta1)
  v = fadd(fmul(v, a.beta2), fmul(1.f - a.beta2, fmul(g, g)));  // mul_(b2).addcmul_(g, g, 1 - b2)
  const float denom = fadd(fdiv(sqrtf(v), a.bc2_sqrt), a.eps);
  a.p[i] = fadd(a.p[i], fmul(-a.lr_over_bc1, fdiv(m, denom)));
  a.m[i] = m;
  a.v[i] = v;
}

// ------------------------------------------------------------------------------------
// MSE(c, gt) + MSE(f, gt) (src/train/trainers/nerf.py:21-29: nn.MSELoss, mean reduction) in one
// launch, and its backward in one: the reference's loss is ~7 small ATen kernels per step.
// Forward: one workgroup, every thread a strided slice, sums in fp64, combined in a fixed order
// (bit-reproducible; torch's fp32 reduction order differs in the last bits).  Backward: the
// ATen formula, grad = (2 / n) * (x - gt) * grad_out, rounded in that order.
// ------------------------------------------------------------------------------------
struct Mse2Args {
  const float* c;
  const float* f;   // or null (coarse only)
  const float* gt;
  int64_t n;
  float* out;       // [3]: loss_c, loss_f, loss_c + loss_f
  // backward
  const float* g_lc;     // grad of loss_c (device scalar) or null
  const float* g_lf;     // or null
  const float* g_total;  // or null
  float* gc;        // [n]
  float* gf;        // [n] or null
};

__global__ void __launch_bounds__(1024) mse2_fwd_kernel(Mse2Args a) {
  __shared__ double red[2][16];
  double sc = 0.0, sf = 0.0;
  for (int64_t i = threadIdx.x; i < a.n; i += 1024) {
    const float g = a.gt[i];
    const float dc = fsub(a.c[i], g);
    sc += (double)fmul(dc, dc);
    if (a.f) {
      const float df = fsub(a.f[i], g);
      sf += (double)fmul(df, df);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    sc += __shfl_xor(sc, o, 64);
    sf += __shfl_xor(sf, o, 64);
  }
  const int w = threadIdx.x >> 6;
  if (lane_id() == 0) {
    red[0][w] = sc;
    red[1][w] = sf;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double tc = 0.0, tf = 0.0;
    for (int k = 0; k < 16; ++k) {
      tc += red[0][k];
      tf += red[1][k];
    }
    const float lc = (float)(tc / (double)a.n), lf = (float)(tf / (double)a.n);
    a.out[0] = lc;
    a.out[1] = lf;
    a.out[2] = a.f ? fadd(lc, lf) : lc;
  }
}

__global__ void mse2_bwd_kernel(Mse2Args a) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n) return;
  const float gt = a.gt[i];
  const float norm = (float)(2.0 / (double)a.n);
  const float gtot = a.g_total ? *a.g_total : 0.f;
  const float goc = a.g_lc ? fadd(*a.g_lc, gtot) : gtot;
  a.gc[i] = fmul(fmul(norm, fsub(a.c[i], gt)), goc);
  if (a.gf) {
    const float gof = a.g_lf ? fadd(*a.g_lf, gtot) : gtot;
    a.gf[i] = fmul(fmul(norm, fsub(a.f[i], gt)), gof);
  }
}

}  // namespace nerf

using namespace nerf;

extern "C" {

// step = the Adam step count after increment (1 for the first update)
int nerf_adam_step(float* param, float* grad, float* exp_avg, float* exp_avg_sq, int64_t n, double lr, double beta1,
                   double beta2, double eps, int64_t step, double clip_value, hipStream_t stream) {
  NERF_REQUIRE(n >= 0 && step >= 1, "nerf_adam_step: bad arguments");
  if (n == 0) return 0;
  NERF_REQUIRE(param && grad && exp_avg && exp_avg_sq, "nerf_adam_step: null pointer");
  const double bc1 = 1.0 - std::pow(beta1, (double)step);
  const double bc2 = 1.0 - std::pow(beta2, (double)step);
  AdamArgs a{param, grad, exp_avg, exp_avg_sq, n, (float)(lr / bc1), (float)(1.0 / std::sqrt(bc2)),
             (float)std::sqrt(bc2), (float)beta1, (float)beta2, (float)eps, (float)clip_value};
  hipLaunchKernelGGL(adam_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, a);
  return check_launch("nerf_adam_step");
}

// out[3] = (MSE(c, gt), MSE(f, gt), their sum) over n values; f may be null (then out[1] = 0)
int nerf_mse2_fwd(const float* c, const float* f, const float* gt, int64_t n, float* out, hipStream_t stream) {
  NERF_REQUIRE(n > 0, "nerf_mse2_fwd: n must be > 0");
  NERF_REQUIRE(c && gt && out, "nerf_mse2_fwd: null pointer");
  Mse2Args a{c, f, gt, n, out, nullptr, nullptr, nullptr, nullptr, nullptr};
  hipLaunchKernelGGL(mse2_fwd_kernel, dim3(1), dim3(1024), 0, stream, a);
  return check_launch("nerf_mse2_fwd");
}

// gc = (2/n) (c - gt) (g_lc + g_total), gf likewise (null grads count as 0; device scalars)
int nerf_mse2_bwd(const float* c, const float* f, const float* gt, int64_t n, const float* g_lc, const float* g_lf,
                  const float* g_total, float* gc, float* gf, hipStream_t stream) {
  NERF_REQUIRE(n > 0, "nerf_mse2_bwd: n must be > 0");
  NERF_REQUIRE(c && gt && gc && (!gf || f), "nerf_mse2_bwd: null pointer");
  Mse2Args a{c, f, gt, n, nullptr, g_lc, g_lf, g_total, gc, gf};
  hipLaunchKernelGGL(mse2_bwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, a);
  return check_launch("nerf_mse2_bwd");
}

}  // extern "C"
