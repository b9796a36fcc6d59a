"""Drop-in ``renderer_module`` (reference: src/models/nerf/renderer/volume_renderer.py:8-357).

Same class, methods and output keys; every step is a gfx950 kernel:

  render               stratified sampling (nerf_sample_stratified) -> fused coarse MLP ->
                       compositing (nerf_composite_fwd/bwd, autograd) -> importance sampling
                       + merge (nerf_sample_pdf) -> fused fine MLP -> compositing
  render_accelerated   occupancy-grid march with early termination (nerf_march_*): rounds of
                       gather -> MLP -> composite sized on the device, one host check for live
                       rays every 4 rounds (the reference syncs once per t step)
  raw2outputs / sample_pdf / world_to_grid_indices   the reference's helper signatures

Randomness (perturb > 0) comes from counter-based Philox streams inside the kernels,
seeded from torch.initial_seed() and advanced per call (distribution-equivalent to the
reference's torch.rand, not the same numbers).
"""
import os
import time

import torch

from nerf_amd import ops
from src.config import cfg


# fragile-ray tolerances of the (opt-in) selective coarse pass: a CDF entry c may move by FRAGILE_REL_TOL *
# min(c, 1 - c) + FRAGILE_ABS_TOL between the split-bf16 and the fp32 coarse net; FRAGILE_Z_TOL > 0 also flags a
# sample those moves could shift within its bin by more than it (tools/cdf_sensitivity.py, tools/selective_sweep.py,
# holding the frame's bounds needed fp32 on 34-100 % of the rays)
FRAGILE_REL_TOL = 1e-4
FRAGILE_ABS_TOL = 1.2e-7
FRAGILE_DEN_TOL = 0.0
FRAGILE_Z_TOL = 0.0


class Renderer:
    def __init__(self, net):
        self.net = net
        self.fragile_rays = 0  # rays the selective coarse pass re-evaluated at fp32 (running count)
        self.occupancy_grid = None
        self.scene_bbox = None
        self.resolution = None
        self.grid_resolution = None
        self.voxel_size = None
        self._calls = 0
        rank = int(os.environ.get("RANK", "0"))
        self._seed = (torch.initial_seed() * 1000003 + rank * 7919) & ((1 << 63) - 1)

    # ------------------------------------------------------------------ helpers
    def _next_offsets(self):
        self._calls += 1
        return self._calls * 4, self._calls * 4 + 1

    def raw2outputs(self, raw, z_vals, rays_d, raw_noise_std=0, white_bkgd=False):
        """volume_renderer.py:20-80 -> rgb_map [R,3], depth_map [R], acc_map [R], weights [R,S]."""
        if raw_noise_std > 0.0:
            noise = torch.randn(raw.shape[:-1], device=raw.device) * raw_noise_std
            raw = torch.cat([raw[..., :3], (raw[..., 3] + noise)[..., None]], -1)
        return ops.composite(raw, z_vals, rays_d, bool(white_bkgd))

    def sample_pdf(self, bins, weights, N_samples, det=False):
        """volume_renderer.py:82-134 (bins [R,nb], weights [R,nb-1]) -> samples [R,N]."""
        off, _ = self._next_offsets()
        return ops.sample_pdf_bins(bins, weights, N_samples, det, seed=self._seed, offset=off)

    # ------------------------------------------------------------------ hierarchical render
    def _selective(self, grad, perturb):
        """The selective coarse pass (round 6, opt-in): an inference render (no autograd graph, perturb 0:
        u = linspace) of a split-bf16 tier with task_arg.coarse_inference_dtype "selective"."""
        return (not grad and not perturb and self.net.mlp_dtype in ("bf16x3", "bf16x3f")
                and (cfg.task_arg.get("coarse_inference_dtype", "fp32") or "") == "selective")

    def _chunk(self, grad):
        ta = cfg.task_arg
        return int(ta.chunk_size) if grad else int(ta.get("render_chunk", ta.chunk_size))

    def _stratified_key(self, rays_flat, n, near, far):
        ta = cfg.task_arg
        return (rays_flat.data_ptr(), n, id(near), id(far), int(ta.N_samples), float(ta.perturb) > 0.0)

    def prepare(self, batch):
        """Enqueue the first training chunk's stratified sampling of a batch ahead of its
        render (volume_renderer.py:160-187 reads no parameter): the trainer issues it before
        waiting for the previous step's gradient all-reduce, so it runs during the reduction.
        render() then uses it (same Philox offsets as it would have drawn itself)."""
        rays = batch["rays"]
        rays_flat = rays.reshape(-1, 6) if rays.ndim == 3 else rays
        n = min(self._chunk(True), rays_flat.shape[0])
        ta = cfg.task_arg
        o1, o2 = self._next_offsets()
        z, pts, vd = ops.sample_stratified(rays_flat[:n], batch["near"], batch["far"], int(ta.N_samples),
                                           float(ta.perturb) > 0.0, seed=self._seed, offset=o1)
        batch["_stratified0"] = (self._stratified_key(rays_flat, n, batch["near"], batch["far"]), o2, z, pts, vd)
        return batch

    def render(self, batch):
        start = time.time()
        ta = cfg.task_arg
        rays = batch["rays"]
        rays_flat = rays.reshape(-1, 6) if rays.ndim == 3 else rays
        near, far = batch["near"], batch["far"]
        grad = torch.is_grad_enabled() and any(p.requires_grad for p in self.net.parameters())
        chunk = self._chunk(grad)
        perturb = float(ta.perturb) > 0.0
        white = bool(ta.white_bkgd)
        n_s, n_i = int(ta.N_samples), int(ta.N_importance)
        outs = {}
        pre = batch.pop("_stratified0", None) if isinstance(batch, dict) else None
        for i in range(0, rays_flat.shape[0], chunk):
            rc = rays_flat[i:i + chunk]
            rd = rc[:, 3:6]
            if i == 0 and pre is not None and pre[0] == self._stratified_key(rays_flat, rc.shape[0], near, far):
                _, o2, z, pts, vd = pre  # prepared ahead (prepare)
            else:
                o1, o2 = self._next_offsets()
                z, pts, vd = ops.sample_stratified(rc, near, far, n_s, perturb, seed=self._seed, offset=o1)
            fused = n_i > 0 and float(ta.raw_noise_std) == 0.0 and n_s <= 64 and ta.get("fuse_composite_pdf", True)
            if fused and self._selective(grad, perturb):
                # (round 6) the split-bf16 tiers' coarse pass in their own arithmetic; the fragile rays -- those
                # whose importance samples a CDF perturbation of the coarse net's error could move across a bin
                # (nerf_composite_pdf_fragile) -- re-evaluated at fp32, so that every ray's fine samples are the
                # fp32 coarse net's (Network.mlp_dtype_for)
                raw_c = self.net(pts, vd, "coarse", dtype=self.net.mlp_dtype)
                rgb_c, dep_c, acc_c, pdf, frag = ops.composite_sample_pdf_fragile(
                    raw_c, z, rc, white, n_i, float(ta.get("fragile_rel_tol", FRAGILE_REL_TOL)),
                    float(ta.get("fragile_abs_tol", FRAGILE_ABS_TOL)), float(ta.get("fragile_den_tol", FRAGILE_DEN_TOL)),
                    float(ta.get("fragile_z_tol", FRAGILE_Z_TOL)))
                idx = frag.nonzero().squeeze(1)
                self.fragile_rays += int(idx.numel())
                if idx.numel():
                    raw_x = self.net(pts[idx], vd[idx], "coarse", dtype="fp32")
                    r2, d2, a2, p2 = ops.composite_sample_pdf(raw_x, z[idx], rc[idx], white, n_i, det=True)
                    rgb_c[idx], dep_c[idx], acc_c[idx] = r2, d2, a2
                    pdf["z_fine"][idx], pdf["pts_fine"][idx] = p2["z_fine"], p2["pts_fine"]
            elif fused:  # raw2outputs + sample_pdf + merge in one launch (ops.composite_sample_pdf)
                raw_c = self.net(pts, vd, "coarse")
                rgb_c, dep_c, acc_c, pdf = ops.composite_sample_pdf(raw_c, z, rc, white, n_i, det=not perturb,
                                                                    seed=self._seed, offset=o2)
            else:
                raw_c = self.net(pts, vd, "coarse")
                rgb_c, dep_c, acc_c, w_c = self.raw2outputs(raw_c, z, rd, ta.raw_noise_std, white)
            ret = {"rgb_map_c": rgb_c, "depth_map_c": dep_c, "acc_map_c": acc_c}
            if n_i > 0:
                if not fused:
                    pdf = ops.sample_pdf(z, w_c, n_i, det=not perturb, seed=self._seed, offset=o2, rays=rc)
                raw_f = self.net(pdf["pts_fine"], vd, "fine")
                rgb_f, dep_f, acc_f, _ = self.raw2outputs(raw_f, pdf["z_fine"], rd, ta.raw_noise_std, white)
                ret.update(rgb_map_f=rgb_f, depth_map_f=dep_f, acc_map_f=acc_f)
            for k, v in ret.items():
                outs.setdefault(k, []).append(v)
        all_ret = {k: (v[0] if len(v) == 1 else torch.cat(v, 0)) for k, v in outs.items()}
        if ta.get("verbose_render", False):
            print(f"Render time: {time.time() - start:.4f} seconds")
        return all_ret

    # ------------------------------------------------------------------ occupancy grid
    def load_occupancy_grid(self, grid_path, device=None):
        """volume_renderer.py:249-259; a missing file leaves the renderer in slow mode."""
        if not os.path.exists(grid_path):
            print(f"Occupancy grid file not found: {grid_path}, run in slow mode.")
            return
        print(f"Loading occupancy grid from {grid_path}...")
        grid = torch.load(grid_path, map_location="cpu", weights_only=True)
        self.set_occupancy_grid(grid, device)
        print("Occupancy grid loaded and ready for accelerated rendering.")

    def set_occupancy_grid(self, grid, device=None):
        device = device or torch.device("cuda", torch.cuda.current_device())
        if grid.dtype != torch.bool or grid.dim() != 3:
            raise ValueError("occupancy grid must be a 3-D bool tensor")
        self.occupancy_grid = grid.to(device)
        self.grid_resolution = torch.tensor(self.occupancy_grid.shape, device=device)
        self.resolution = int(grid.shape[0])
        self.scene_bbox = torch.tensor(cfg.train_dataset.scene_bbox, device=device, dtype=torch.float32)
        self.voxel_size = (self.scene_bbox[1] - self.scene_bbox[0]) / self.grid_resolution

    def _bbox_tuple(self):
        b = cfg.train_dataset.scene_bbox
        return (tuple(float(v) for v in b[0]), tuple(float(v) for v in b[1]))

    def world_to_grid_indices(self, points):
        """volume_renderer.py:261-265 -> int64 [M,3]."""
        idx, _ = ops.grid_index(points, None, int(self.grid_resolution[0]), self._bbox_tuple())
        return idx

    def render_accelerated(self, batch):
        """volume_renderer.py:268-357: march the fine net through the occupancy grid."""
        if self.occupancy_grid is None:
            print("Occupancy grid not loaded, running in slow mode.")
            return self.render(batch)
        ta = cfg.task_arg
        rays = batch["rays"]
        rays_flat = rays.reshape(-1, 6) if rays.ndim == 3 else rays
        near = float(batch["near"].reshape(-1)[0]) if torch.is_tensor(batch["near"]) else float(batch["near"])
        far = float(batch["far"].reshape(-1)[0]) if torch.is_tensor(batch["far"]) else float(batch["far"])
        starter = torch.cuda.Event(enable_timing=True)
        ender = torch.cuda.Event(enable_timing=True)
        starter.record()
        out = ops.march(self.net.model_fine.packer(), rays_flat, near, far, self.occupancy_grid,
                        step_size=float(ta.render_step_size), t_thresh=float(ta.transmittance_threshold),
                        bbox=self._bbox_tuple(), white_bkgd=bool(ta.white_bkgd), dtype=self.net.mlp_dtype)
        ender.record()
        torch.cuda.synchronize()
        render_time_s = starter.elapsed_time(ender) / 1000.0
        print(f"Accelerated Render time: {render_time_s:.4f} seconds")
        return {"rgb_map_f": out["rgb_map_f"], "depth_map_f": out["depth_map_f"], "acc_map_f": out["acc_map_f"],
                "render_time": render_time_s, "n_queried": out["n_queried"], "n_evaluated": out["n_evaluated"],
                "rounds": out["rounds"]}
