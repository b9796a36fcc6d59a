"""Torch-facing wrappers of the gfx950 kernels (device memory and streams come from torch;
the arithmetic is in libnerf_amd.so).  Every function raises on CPU tensors.

Reference interfaces mirrored (echo636/nerf-replication):
  raygen               src/datasets/nerf/blender.py:13-32, 124-131
  sample_stratified    src/models/nerf/renderer/volume_renderer.py:165-187
  sample_pdf           volume_renderer.py:82-134 (+ merge :205-221)
  composite            volume_renderer.py:20-80 (autograd Function)
  mlp                  src/models/nerf/network.py:171-192 (autograd Function)
  grid_index           volume_renderer.py:261-265
  march                volume_renderer.py:268-357
  bake                 occupancy_grid.py:15-80
  adam_step            src/train/trainers/trainer.py:61-62
"""
from __future__ import annotations

import contextlib
import ctypes as _ctypes
import functools
import os
from typing import List, Optional, Sequence

import torch

from ._lib import check, lib, ptr, stream_of

F32, BF16, BF16X3, BF16X3F, BF16X6 = 0, 1, 2, 3, 4
# bf16x3: fp32 operands split into bf16 hi + lo, products hi*hi + hi*lo + lo*hi on the bf16
# MFMA with fp32 accumulation (csrc/mlp.hip PBF3): fp32-class results at bf16-MFMA cost x3.
# bf16x3f: the bf16x3 forward (outputs identical to bf16x3's) with the bf16 backward (its
# training stores are the bf16 hi halves): bf16x3 outputs, bf16 gradients
# bf16x6: an inference forward only -- operands split exactly into three bf16, six products (at least
# as accurate as fp32): the coarse net of a bf16x3 / bf16x3f render (Network.mlp_dtype_for)
DTYPES = {"fp32": F32, "float32": F32, "f32": F32, "bf16": BF16, "bfloat16": BF16, "bf16x3": BF16X3,
          "bf16x3f": BF16X3F, "bf16x6": BF16X6}
DTYPE_NAMES = {F32: "fp32", BF16: "bf16", BF16X3: "bf16x3", BF16X3F: "bf16x3f", BF16X6: "bf16x6"}


def pack_code(dtype: int, direction: int) -> int:
    """The packed-weight layout a (dtype, direction) uses: bf16x3f packs its forward as
    bf16x3 and its backward (W^T) as bf16, so it shares those caches."""
    if dtype == BF16X3F:
        return BF16X3 if direction == 0 else BF16
    return dtype

SCENE_BBOX = ((-1.5, -1.5, -1.5), (1.5, 1.5, 1.5))


def dtype_code(d) -> int:
    if isinstance(d, int):
        return d
    if d not in DTYPES:
        raise ValueError(f"unsupported MLP dtype {d!r} (fp32, bf16, bf16x3, bf16x3f or the inference-only bf16x6)")
    return DTYPES[d]


def _f32c(t: torch.Tensor, name: str) -> torch.Tensor:
    if t.dtype != torch.float32:
        raise TypeError(f"{name} must be float32, got {t.dtype}")
    return t.contiguous()


@functools.lru_cache(maxsize=None)
def _cpu_table(kind: str, a: float, b: float, n_or_step) -> torch.Tensor:
    """Host CPU tables (torch.linspace / torch.arange evaluated on the CPU, as the reference)."""
    if kind == "linspace":
        return torch.linspace(a, b, steps=int(n_or_step))
    return torch.arange(a, b, n_or_step)


_dev_tables = {}


def device_table(kind: str, a: float, b: float, n_or_step, device) -> torch.Tensor:
    key = (kind, a, b, n_or_step, str(device))
    t = _dev_tables.get(key)
    if t is None:
        t = _cpu_table(kind, a, b, n_or_step).to(device)
        _dev_tables[key] = t
    return t


_dev_scalars = {}


def device_scalar(x: float, device) -> torch.Tensor:
    """A cached 1-element fp32 device tensor.  Building one per call (torch.tensor(...,
    device=)) is a pageable host-to-device copy, which blocks the host until the GPU queue
    has drained: at every training step that idles the GPU for the whole Python launch
    sequence."""
    key = (float(x), str(torch.device(device)))
    t = _dev_scalars.get(key)
    if t is None:
        t = torch.tensor([float(x)], dtype=torch.float32, device=device)
        _dev_scalars[key] = t
    return t


def _scalar_dev(x, device) -> torch.Tensor:
    if isinstance(x, torch.Tensor):
        return x.reshape(-1)[:1].to(device=device, dtype=torch.float32).contiguous()
    return device_scalar(x, device)


# --------------------------------------------------------------------------------------
# optional per-kernel timing with HIP events on the launching stream (bench.py roofline)
# --------------------------------------------------------------------------------------
class _KernelTimes:
    """MLP kernels are timed whenever ``enabled``; the HBM-bound sampling / compositing kernels
    (units = algorithmic bytes) only when ``detail`` is also set, so that a
    headline timing run carries no extra events on those short launches."""

    def __init__(self):
        self.enabled = False
        self.detail = False
        self.pending = []  # (name, units, start_event, end_event)

    def reset(self):
        self.pending = []

    def summary(self):
        """{name: (launches, total_ms, total_units)} -- synchronises on the recorded events."""
        out = {}
        for name, units, a, b in self.pending:
            n, ms, u = out.get(name, (0, 0.0, 0))
            out[name] = (n + 1, ms + a.elapsed_time(b), u + units)
        return out


KERNEL_TIMES = _KernelTimes()


class kernel_timer:
    def __init__(self, name, units, detail=False):
        self.name, self.units = name, units
        self.on = KERNEL_TIMES.enabled and (KERNEL_TIMES.detail or not detail)

    def __enter__(self):
        if self.on:
            self.a = torch.cuda.Event(enable_timing=True)
            self.b = torch.cuda.Event(enable_timing=True)
            self.a.record(torch.cuda.current_stream())
        return self

    def __exit__(self, *exc):
        if self.on:
            self.b.record(torch.cuda.current_stream())
            KERNEL_TIMES.pending.append((self.name, self.units, self.a, self.b))
        return False


# --------------------------------------------------------------------------------------
# rays
# --------------------------------------------------------------------------------------
def raygen(c2w: torch.Tensor, H: int, W: int, focal: float, pix: Optional[torch.Tensor] = None, n_rays: int = 0,
           seed: int = 0, offset: int = 0, images: Optional[torch.Tensor] = None, want_pix: bool = False):
    """Pinhole rays for flat pixel ids (img*H*W + j*W + i) -> rays [R,6] (+ rgb [R,3])."""
    c2w = _f32c(c2w.reshape(-1, 4, 4) if c2w.shape[-2:] == (4, 4) else c2w, "c2w")
    if c2w.shape[-2:] != (4, 4):
        raise ValueError("c2w must be [..., 4, 4]")
    dev = c2w.device
    R = int(pix.numel()) if pix is not None else int(n_rays)
    if pix is not None:
        pix = pix.to(device=dev, dtype=torch.int64).contiguous()
    rays = torch.empty(R, 6, device=dev, dtype=torch.float32)
    rgb = torch.empty(R, 3, device=dev, dtype=torch.float32) if images is not None else None
    pout = torch.empty(R, device=dev, dtype=torch.int64) if want_pix else None
    if images is not None:
        images = _f32c(images, "images")
    # bytes per ray: pixel id read (given) or written (want_pix), 24 B rays, 12 B rgb gather + 12 B write
    nbytes = R * (24 + (8 if pix is not None else 0) + (8 if want_pix else 0) + (24 if images is not None else 0))
    with kernel_timer("raygen", nbytes, detail=True):
        check(lib().nerf_raygen(ptr(c2w), c2w.shape[0], H, W, float(focal), ptr(pix), R, seed, offset, ptr(images),
                                ptr(rays), ptr(rgb), ptr(pout), stream_of(c2w)), "nerf_raygen")
    return rays, rgb, pout


def sample_stratified(rays: torch.Tensor, near, far, n_samples: int, perturb: bool,
                      t_rand: Optional[torch.Tensor] = None, seed: int = 0, offset: int = 0,
                      want_pts: bool = True):
    """-> z [R,S], pts [R,S,3] (or None), viewdirs [R,3]."""
    rays = _f32c(rays.reshape(-1, 6), "rays")
    dev, R = rays.device, rays.shape[0]
    t_lin = device_table("linspace", 0.0, 1.0, n_samples, dev)
    z = torch.empty(R, n_samples, device=dev, dtype=torch.float32)
    pts = torch.empty(R, n_samples, 3, device=dev, dtype=torch.float32) if want_pts else None
    vd = torch.empty(R, 3, device=dev, dtype=torch.float32)
    if t_rand is not None:
        t_rand = _f32c(t_rand, "t_rand")
    near_t, far_t = _scalar_dev(near, dev), _scalar_dev(far, dev)  # keep alive across the launch
    # bytes per ray: 24 B ray read, 4 B z (+12 B pts, +4 B injected uniform) per sample, 12 B viewdir
    nbytes = R * (24 + 12 + n_samples * (4 + (12 if want_pts else 0) + (4 if t_rand is not None else 0)))
    with kernel_timer("sample_stratified", nbytes, detail=True):
        check(lib().nerf_sample_stratified(ptr(rays), R, n_samples, ptr(t_lin), ptr(near_t), ptr(far_t),
                                           int(bool(perturb)), ptr(t_rand), seed, offset, ptr(z), ptr(pts), ptr(vd),
                                           stream_of(rays)), "nerf_sample_stratified")
    return z, pts, vd


def searchsorted(cdf: torch.Tensor, u: torch.Tensor) -> torch.Tensor:
    """torch.searchsorted(cdf, u, right=True) for rows of <= 64 sorted entries (int32)."""
    cdf, u = _f32c(cdf, "cdf"), _f32c(u, "u")
    R, nb = cdf.shape
    out = torch.empty(u.shape, device=cdf.device, dtype=torch.int32)
    check(lib().nerf_searchsorted(ptr(cdf), ptr(u), R, nb, u.shape[1], ptr(out), stream_of(cdf)), "nerf_searchsorted")
    return out


def sample_pdf(z: torch.Tensor, weights: torch.Tensor, n_importance: int, det: bool,
               u: Optional[torch.Tensor] = None, seed: int = 0, offset: int = 0,
               rays: Optional[torch.Tensor] = None, debug: bool = False):
    """Importance sampling on the coarse weights + merge with z.

    Returns dict(z_fine [R,Sc+Ni] sorted, pts_fine [R,Sc+Ni,3] if rays given, and with
    ``debug`` samples [R,Ni], cdf [R,Sc-1], inds [R,Ni] int32).
    """
    z, weights = _f32c(z, "z"), _f32c(weights.detach(), "weights")
    R, Sc = z.shape
    dev = z.device
    S = Sc + n_importance
    out = {"z_fine": torch.empty(R, S, device=dev, dtype=torch.float32)}
    if rays is not None:
        rays = _f32c(rays.reshape(-1, 6), "rays")
        out["pts_fine"] = torch.empty(R, S, 3, device=dev, dtype=torch.float32)
    if debug:
        out["samples"] = torch.empty(R, n_importance, device=dev, dtype=torch.float32)
        out["cdf"] = torch.empty(R, Sc - 1, device=dev, dtype=torch.float32)
        out["inds"] = torch.empty(R, n_importance, device=dev, dtype=torch.int32)
    u_lin = device_table("linspace", 0.0, 1.0, n_importance, dev) if det else None
    if u is not None:
        u = _f32c(u, "u")
    # bytes per ray: z + weights read (8 B per coarse sample), injected u, ray; merged z (+ pts) written
    nbytes = R * (8 * Sc + (4 * n_importance if u is not None else 0) + (24 if rays is not None else 0)
                  + S * (4 + (12 if rays is not None else 0)) + (12 * n_importance + 4 * (Sc - 1) if debug else 0))
    with kernel_timer("sample_pdf", nbytes, detail=True):
        check(lib().nerf_sample_pdf(ptr(z), ptr(weights), R, Sc, n_importance, int(bool(det)), ptr(u_lin), ptr(u),
                                    seed, offset, ptr(rays), ptr(out["z_fine"]), ptr(out.get("pts_fine")),
                                    ptr(out.get("samples")), ptr(out.get("cdf")), ptr(out.get("inds")), stream_of(z)),
              "nerf_sample_pdf")
    return out


def sample_pdf_bins(bins: torch.Tensor, weights: torch.Tensor, n_samples: int, det: bool,
                    u: Optional[torch.Tensor] = None, seed: int = 0, offset: int = 0, debug: bool = False):
    """Reference-signature sample_pdf: bins [R,nb], weights [R,nb-1] -> samples [R,N] (u order)."""
    bins, weights = _f32c(bins, "bins"), _f32c(weights.detach(), "weights")
    R, nb = bins.shape
    dev = bins.device
    samples = torch.empty(R, n_samples, device=dev, dtype=torch.float32)
    cdf = torch.empty(R, nb, device=dev, dtype=torch.float32) if debug else None
    inds = torch.empty(R, n_samples, device=dev, dtype=torch.int32) if debug else None
    u_lin = device_table("linspace", 0.0, 1.0, n_samples, dev) if det else None
    if u is not None:
        u = _f32c(u, "u")
    check(lib().nerf_sample_pdf_bins(ptr(bins), ptr(weights), R, nb, n_samples, int(bool(det)), ptr(u_lin), ptr(u),
                                     seed, offset, ptr(samples), ptr(cdf), ptr(inds), stream_of(bins)),
          "nerf_sample_pdf_bins")
    return (samples, cdf, inds) if debug else samples


# --------------------------------------------------------------------------------------
# compositing (autograd)
# --------------------------------------------------------------------------------------
def _dirs_view(rays_d: torch.Tensor):
    """(tensor owning memory, pointer, row stride) for [R,3] direction rows, allowing the
    [R,6]-ray slice view rays[:, 3:6] without a copy."""
    if rays_d.dim() == 2 and rays_d.shape[1] == 3 and rays_d.stride(1) == 1 and rays_d.dtype == torch.float32:
        return rays_d, rays_d.data_ptr(), rays_d.stride(0)
    c = _f32c(rays_d.reshape(-1, 3), "rays_d")
    return c, c.data_ptr(), 3


class _Composite(torch.autograd.Function):
    @staticmethod
    def forward(ctx, raw, z, rays_d, white):
        raw, z = _f32c(raw, "raw"), _f32c(z, "z")
        R, S = z.shape
        keep, dptr, dstride = _dirs_view(rays_d)
        dev = raw.device
        rgb = torch.empty(R, 3, device=dev, dtype=torch.float32)
        depth = torch.empty(R, device=dev, dtype=torch.float32)
        acc = torch.empty(R, device=dev, dtype=torch.float32)
        w = torch.empty(R, S, device=dev, dtype=torch.float32)
        # bytes per ray: raw 16 B + z 4 B read and weight 4 B written per sample; dir 12 B; rgb/depth/acc 20 B
        with kernel_timer("composite_fwd", R * (24 * S + 32), detail=True):
            check(lib().nerf_composite_fwd(ptr(raw), ptr(z), dptr, dstride, R, S, int(bool(white)), ptr(rgb),
                                           ptr(depth), ptr(acc), ptr(w), stream_of(raw)), "nerf_composite_fwd")
        ctx.set_materialize_grads(False)  # unused outputs (depth, acc) arrive as None, not zero-filled
        ctx.save_for_backward(raw, z, keep)
        ctx.dptr, ctx.dstride, ctx.white = dptr, dstride, int(bool(white))
        ctx.mark_non_differentiable(w)
        return rgb, depth, acc, w

    @staticmethod
    def backward(ctx, g_rgb, g_depth, g_acc, g_w):
        if g_rgb is None and g_depth is None and g_acc is None:
            return None, None, None, None
        raw, z, _keep = ctx.saved_tensors
        R, S = z.shape
        if g_rgb is None:
            g_rgb = torch.zeros(R, 3, device=raw.device, dtype=torch.float32)
        g_rgb = g_rgb.contiguous()
        g_depth = None if g_depth is None else g_depth.contiguous()
        g_acc = None if g_acc is None else g_acc.contiguous()
        g_raw = torch.empty_like(raw)
        # bytes per ray: raw 16 B + z 4 B read and d_raw 16 B written per sample; dir 12 B; output grads
        nbytes = R * (36 * S + 24 + (4 if g_depth is not None else 0) + (4 if g_acc is not None else 0))
        with kernel_timer("composite_bwd", nbytes, detail=True):
            check(lib().nerf_composite_bwd(ptr(raw), ptr(z), ctx.dptr, ctx.dstride, R, S, ctx.white, ptr(g_rgb),
                                           ptr(g_depth), ptr(g_acc), ptr(g_raw), stream_of(raw)), "nerf_composite_bwd")
        return g_raw, None, None, None


def composite(raw: torch.Tensor, z: torch.Tensor, rays_d: torch.Tensor, white_bkgd: bool = True):
    """raw2outputs: -> rgb [R,3], depth [R], acc [R], weights [R,S] (weights carry no grad)."""
    return _Composite.apply(raw.reshape(z.shape[0], z.shape[1], 4), z, rays_d, white_bkgd)


class _CompositePdf(torch.autograd.Function):
    """The coarse compositing (differentiable in raw, as _Composite) fused with the importance
    sampling + merge that reads its weights (no gradient: the reference detaches the samples,
    volume_renderer.py:216)."""

    @staticmethod
    def forward(ctx, raw, z, rays_d, white, n_importance, det, seed, offset, rays):
        raw, z = _f32c(raw, "raw"), _f32c(z, "z")
        R, Sc = z.shape
        keep, dptr, dstride = _dirs_view(rays_d)
        dev = raw.device
        rgb = torch.empty(R, 3, device=dev, dtype=torch.float32)
        depth = torch.empty(R, device=dev, dtype=torch.float32)
        acc = torch.empty(R, device=dev, dtype=torch.float32)
        S = Sc + n_importance
        z_fine = torch.empty(R, S, device=dev, dtype=torch.float32)
        pts_fine = torch.empty(R, S, 3, device=dev, dtype=torch.float32)
        rays = _f32c(rays.reshape(-1, 6), "rays")
        u_lin = device_table("linspace", 0.0, 1.0, n_importance, dev) if det else None
        # bytes per ray: raw 16 B + z 4 B per coarse sample, dir + ray; merged z + pts written
        nbytes = R * (20 * Sc + 12 + 24 + 16 * S + 20)
        with kernel_timer("composite_pdf", nbytes, detail=True):
            check(lib().nerf_composite_pdf(ptr(raw), ptr(z), dptr, dstride, R, Sc, int(bool(white)), ptr(rgb),
                                           ptr(depth), ptr(acc), None, int(n_importance), int(bool(det)), ptr(u_lin),
                                           None, seed, offset, ptr(rays), ptr(z_fine), ptr(pts_fine),
                                           stream_of(raw)), "nerf_composite_pdf")
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(raw, z, keep)
        ctx.dptr, ctx.dstride, ctx.white = dptr, dstride, int(bool(white))
        ctx.mark_non_differentiable(z_fine, pts_fine)
        return rgb, depth, acc, z_fine, pts_fine

    @staticmethod
    def backward(ctx, g_rgb, g_depth, g_acc, g_zf, g_pf):
        return _Composite.backward(ctx, g_rgb, g_depth, g_acc, None)[:1] + (None,) * 8


def composite_sample_pdf(raw: torch.Tensor, z: torch.Tensor, rays: torch.Tensor, white_bkgd: bool, n_importance: int,
                         det: bool, seed: int = 0, offset: int = 0):
    """composite (rgb, depth, acc of the coarse pass) + sample_pdf (merged z_fine, pts_fine) in one
    launch: bit-identical to composite() then sample_pdf(z, weights, ..., rays=rays)."""
    rays = rays.reshape(-1, 6)
    rgb, depth, acc, z_fine, pts_fine = _CompositePdf.apply(raw.reshape(z.shape[0], z.shape[1], 4), z, rays[:, 3:6],
                                                            white_bkgd, n_importance, det, seed, offset, rays)
    return rgb, depth, acc, {"z_fine": z_fine, "pts_fine": pts_fine}


@torch.no_grad()
def composite_sample_pdf_fragile(raw: torch.Tensor, z: torch.Tensor, rays: torch.Tensor, white_bkgd: bool,
                                 n_importance: int, rel_tol: float, abs_tol: float, den_tol: float = 0.0,
                                 z_tol: float = 0.0):
    """composite_sample_pdf at det (u = linspace), inference only, that also returns the per-ray fragile flag
    (int32 [R]): 1 when an importance sample's bin could change if every CDF entry c moved by up to
    rel_tol * min(c, 1 - c) + abs_tol, or the den of its interval is within den_tol of the den < 1e-5 switch, or
    (z_tol > 0) those moves could shift a sample within its bin by more than z_tol (nerf_composite_pdf_fragile)."""
    raw, z = _f32c(raw.reshape(z.shape[0], z.shape[1], 4), "raw"), _f32c(z, "z")
    rays = _f32c(rays.reshape(-1, 6), "rays")
    R, Sc = z.shape
    dev = raw.device
    keep, dptr, dstride = _dirs_view(rays[:, 3:6])
    rgb = torch.empty(R, 3, device=dev, dtype=torch.float32)
    depth = torch.empty(R, device=dev, dtype=torch.float32)
    acc = torch.empty(R, device=dev, dtype=torch.float32)
    S = Sc + n_importance
    z_fine = torch.empty(R, S, device=dev, dtype=torch.float32)
    pts_fine = torch.empty(R, S, 3, device=dev, dtype=torch.float32)
    fragile = torch.empty(R, device=dev, dtype=torch.int32)
    u_lin = device_table("linspace", 0.0, 1.0, n_importance, dev)
    nbytes = R * (20 * Sc + 12 + 24 + 16 * S + 24)
    with kernel_timer("composite_pdf", nbytes, detail=True):
        check(lib().nerf_composite_pdf_fragile(ptr(raw), ptr(z), dptr, dstride, R, Sc, int(bool(white_bkgd)), ptr(rgb),
                                               ptr(depth), ptr(acc), int(n_importance), ptr(u_lin), ptr(rays),
                                               ptr(z_fine), ptr(pts_fine), float(rel_tol), float(abs_tol),
                                               float(den_tol), float(z_tol), ptr(fragile), stream_of(raw)),
              "nerf_composite_pdf_fragile")
    del keep
    return rgb, depth, acc, {"z_fine": z_fine, "pts_fine": pts_fine}, fragile


class _Mse2(torch.autograd.Function):
    @staticmethod
    def forward(ctx, c, f, gt):
        c, gt = _f32c(c, "rgb_c"), _f32c(gt, "gt")
        f = _f32c(f, "rgb_f") if f is not None else None
        out = torch.empty(3, device=c.device, dtype=torch.float32)
        check(lib().nerf_mse2_fwd(ptr(c), ptr(f), ptr(gt), c.numel(), ptr(out), stream_of(c)), "nerf_mse2_fwd")
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(c, f, gt)
        ctx.has_f = f is not None
        return out[0], out[1], out[2]

    @staticmethod
    def backward(ctx, g_lc, g_lf, g_total):
        c, f, gt = ctx.saved_tensors
        gc = torch.empty_like(c)
        gf = torch.empty_like(f) if ctx.has_f else None
        g = [None if t is None else t.reshape(1).to(torch.float32).contiguous() for t in (g_lc, g_lf, g_total)]
        check(lib().nerf_mse2_bwd(ptr(c), ptr(f), ptr(gt), c.numel(), ptr(g[0]), ptr(g[1]), ptr(g[2]), ptr(gc),
                                  ptr(gf), stream_of(c)), "nerf_mse2_bwd")
        return gc, gf, None


def mse_pair(rgb_c: torch.Tensor, rgb_f: Optional[torch.Tensor], gt: torch.Tensor):
    """(MSE(rgb_c, gt), MSE(rgb_f, gt), their sum) -- nn.MSELoss twice and an add
    (src/train/trainers/nerf.py:21-29) -- in one forward and one backward launch."""
    gt = gt.reshape(rgb_c.shape)
    return _Mse2.apply(rgb_c, rgb_f, gt)


# --------------------------------------------------------------------------------------
# MLP (autograd)
# --------------------------------------------------------------------------------------
NET_PARAM_NAMES = (
    [f"pts_linears.{i}.{k}" for i in range(8) for k in ("weight", "bias")]
    + [f"{n}.{k}" for n in ("views_linears.0", "feature_linear", "alpha_linear", "rgb_linear")
       for k in ("weight", "bias")]
)


_PARAM_GENERATION = [0]
_DIRECT_GRAD = [0]
# dW partial sums reduced in a fixed order (bit-reproducible gradients) instead of fp32 atomics
DETERMINISTIC_DW = True
# samples per backward chunk, by backward precision (a multiple of 256; absent = one launch).
# None by default: in the whole training step (tools/step_ab.py, interleaved) 262,144-sample
# chunks were slower for bf16 (4.57 vs 4.53 ms/step) and bf16x3f (6.53 vs 6.49), although the
# backward alone was faster chunked (tools/mlp_bench.py --chunks)
BWD_CHUNK = {}


# inside direct_grad(), with NERF_DW_STREAM=1: the dW launches run on a second stream (per
# device), each after its chunk's dX, so the next dX -- the same net's next chunk, or the other
# net's backward -- overlaps the dW's dZ stream; direct_grad's exit joins it.  Bit-identical;
# off by default: in the whole step (tools/step_ab.py) bf16 4.53 -> 4.44 ms but bf16x3f 6.49 ->
# 6.53 -- the overlap is only the dW's work-item tail (a dX workgroup needs a whole CU's LDS)
DW_STREAM = os.environ.get("NERF_DW_STREAM", "0") == "1"
_DW_STREAMS = {}
_DW_PENDING = []  # (device, event recorded on its dW stream after the last enqueued dW)


def dw_stream(dev: torch.device) -> torch.cuda.Stream:
    st = _DW_STREAMS.get(dev.index)
    if st is None:
        st = _DW_STREAMS[dev.index] = torch.cuda.Stream(device=dev)
    return st


def dw_join() -> None:
    """The current stream waits for every dW enqueued on the dW streams (a no-op when none is)."""
    while _DW_PENDING:
        dev, ev = _DW_PENDING.pop()
        torch.cuda.current_stream(dev).wait_event(ev)


class direct_grad:
    """Context for a plain ``loss.backward()`` of a training step whose parameters' ``.grad``
    are views of one flat buffer (FusedAdam): inside it the dW kernel adds straight into
    ``.grad`` (no zero-filled temporary, no 24 autograd accumulations) and autograd receives
    None for the parameters.  Outside it (``torch.autograd.grad``, hooks, a non-flat
    optimizer) the MLP backward returns ordinary gradients to autograd.  On exit the compute
    stream waits for the dW stream (DW_STREAM): every later use of ``.grad`` sees it whole."""

    def __enter__(self):
        _DIRECT_GRAD[0] += 1
        return self

    def __exit__(self, *exc):
        _DIRECT_GRAD[0] -= 1
        dw_join()
        return False


def params_updated() -> None:
    """Invalidate every packed-weight cache: call after parameters were written by a kernel
    torch does not see (the fused Adam step bypasses torch's version counters)."""
    _PARAM_GENERATION[0] += 1


class PackedMLP:
    """Re-packs one NeRF's 24 fp32 parameters into the kernels' lane-linear layout,
    lazily, whenever a parameter changed (version counter / storage)."""

    def __init__(self, params: Sequence[torch.Tensor]):
        if len(params) != 24:
            raise ValueError("expected the 24 parameters of one NeRF in state_dict order")
        self.params = list(params)
        self._cache = {}
        # called as grad_ready(flat_grad_view) once this net's gradient is complete in a
        # backward pass (the data-parallel trainer starts its all-reduce bucket there)
        self.grad_ready = None
        # training forwards of this net whose backward has not run yet: a render split into
        # chunks (volume_renderer.py:62-67) calls the MLP once per chunk, and the net's
        # gradient is complete only after the LAST of those backwards
        self.pending = 0

    def forward_started(self) -> None:
        self.pending += 1

    def backward_done(self, flat: Optional[torch.Tensor]) -> bool:
        """One training forward's backward has been enqueued; fires grad_ready(flat) when it
        was the last pending one.  Returns True when it fired."""
        self.pending = max(0, self.pending - 1)
        if self.pending == 0 and self.grad_ready is not None:
            self.grad_ready(flat)
            return True
        return False

    def flat_grad(self) -> Optional[torch.Tensor]:
        """The 24 .grad tensors as one flat fp32 view, when they are laid out back to back in
        state_dict order (FusedAdam's flat buffer); else None."""
        gs = [p.grad for p in self.params]
        if any(g is None for g in gs):
            return None
        g0 = gs[0]
        if g0.dtype != torch.float32 or not g0.is_cuda:
            return None
        base, st = g0.data_ptr(), g0.untyped_storage().data_ptr()
        off = 0
        for g in gs:
            if (g.dtype != torch.float32 or not g.is_contiguous() or g.untyped_storage().data_ptr() != st
                    or g.data_ptr() != base + 4 * off):
                return None
            off += g.numel()
        start = (base - st) // 4
        return torch.empty(0, dtype=torch.float32, device=g0.device).set_(
            g0.untyped_storage(), start, (off,), (1,))

    def _key(self):
        return (_PARAM_GENERATION[0],) + tuple((p.data_ptr(), p._version) for p in self.params)

    def get(self, dtype: int, direction: int) -> torch.Tensor:
        dtype = pack_code(dtype, direction)
        key = self._key()
        ent = self._cache.get((dtype, direction))
        if ent is not None and ent[0] == key:
            return ent[1]
        dev = self.params[0].device
        for p in self.params:
            if p.dtype != torch.float32 or not p.is_contiguous() or p.device != dev:
                raise TypeError("NeRF parameters must be contiguous float32 tensors on one device")
        nbytes = lib().nerf_mlp_packed_bytes(dtype, direction)
        buf = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        arr = _ctypes.cast((_ctypes.c_void_p * 24)(*[p.data_ptr() for p in self.params]), _ctypes.c_void_p)
        fwd = buf if direction == 0 else None
        bwd = buf if direction == 1 else None
        check(lib().nerf_mlp_pack(arr, dtype, ptr(fwd), ptr(bwd), stream_of(self.params[0])), "nerf_mlp_pack")
        self._cache[(dtype, direction)] = (key, buf)
        return buf


class _MLP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pts, viewdirs, dir_index, spd, packer, dtype, density_only, want_grad, *params):
        pts = _f32c(pts.reshape(-1, 3), "pts")
        M = pts.shape[0]
        dev = pts.device
        store = bool(want_grad) and any(ctx.needs_input_grad[8:])
        if dtype == BF16X6 and (store or density_only):
            raise RuntimeError("the bf16x6 MLP is an inference forward only (no autograd, no density-only pass)")
        raw = torch.empty(M, 4, device=dev, dtype=torch.float32)
        if M == 0:
            ctx.M = 0
            return raw
        if viewdirs is not None:
            viewdirs = _f32c(viewdirs.reshape(-1, 3), "viewdirs")
        if dir_index is not None:
            dir_index = dir_index.to(torch.int32).contiguous()
        act = masks = None
        flags = 0
        if store:
            act = torch.empty(lib().nerf_mlp_act_bytes(dtype, M), dtype=torch.uint8, device=dev)
            masks = torch.empty(lib().nerf_mlp_mask_bytes(M), dtype=torch.uint8, device=dev)
            flags |= 1
        if density_only:
            flags |= 2
        packed = packer.get(dtype, 0)
        with kernel_timer("mlp_fwd_train" if store else ("mlp_fwd_density" if density_only else "mlp_fwd"), M):
            check(lib().nerf_mlp_fwd(ptr(packed), dtype, ptr(pts), ptr(viewdirs), int(spd), ptr(dir_index), M, flags,
                                     ptr(raw), ptr(act), ptr(masks), stream_of(pts)), "nerf_mlp_fwd")
        ctx.M, ctx.dtype, ctx.packer = M, dtype, packer
        ctx.act, ctx.masks = act, masks
        if store:
            ctx.packed_bwd = packer.get(dtype, 1)
            packer.forward_started()
        return raw

    @staticmethod
    def backward(ctx, g_raw):
        params = ctx.packer.params
        nones = (None,) * 8
        if ctx.M == 0:
            return nones + tuple(torch.zeros_like(p) for p in params)
        dev = g_raw.device
        g_raw = g_raw.contiguous()
        dz = torch.empty(lib().nerf_mlp_dz_bytes(ctx.dtype, ctx.M), dtype=torch.uint8, device=dev)
        # inside ops.direct_grad() (a training step's loss.backward()), accumulate straight into
        # the parameters' .grad when they are one flat buffer (the dW partial sums are added in a
        # fixed order by the reduce kernel, or with atomics when DETERMINISTIC_DW is off): no
        # zero-fill, no 24 autograd accumulation kernels
        direct = ctx.packer.flat_grad() if _DIRECT_GRAD[0] > 0 else None
        grad = direct if direct is not None else torch.zeros(lib().nerf_mlp_net_params(), device=dev,
                                                              dtype=torch.float32)
        s = stream_of(g_raw)
        L = lib()
        # the backward in chunks of BWD_CHUNK samples (dX then dW per chunk; the stores are
        # block-major, so a chunk is a contiguous byte range of each); off by default (BWD_CHUNK)
        C = BWD_CHUNK.get(pack_code(ctx.dtype, 1), ctx.M)
        C = ctx.M if C >= ctx.M else C
        ws = torch.empty(L.nerf_mlp_dw_workspace_bytes(ctx.dtype, C), dtype=torch.uint8, device=dev) \
            if DETERMINISTIC_DW else None
        z_blk, a_blk = L.nerf_mlp_dz_bytes(ctx.dtype, 256) // 8, L.nerf_mlp_act_bytes(ctx.dtype, 256) // 8
        m_blk = L.nerf_mlp_mask_bytes(256) // 8
        side = dw_stream(dev) if direct is not None and DW_STREAM and dev.type == "cuda" else None
        for s0 in range(0, ctx.M, C):
            m, b0 = min(C, ctx.M - s0), s0 // 32
            with kernel_timer("mlp_bwd_dx", m):
                check(L.nerf_mlp_bwd_dx(ptr(ctx.packed_bwd), ctx.dtype, g_raw.data_ptr() + 16 * s0, m,
                                        ctx.masks.data_ptr() + b0 * m_blk, dz.data_ptr() + b0 * z_blk, s),
                      "nerf_mlp_bwd_dx")
            if side is not None:  # this chunk's dW after its dX, on the dW stream
                side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side) if side is not None else contextlib.nullcontext():
                with kernel_timer("mlp_bwd_dw", m):
                    check(L.nerf_mlp_bwd_dw_ws(ctx.dtype, m, ctx.act.data_ptr() + b0 * a_blk,
                                               dz.data_ptr() + b0 * z_blk, ptr(grad), ptr(ws),
                                               side.cuda_stream if side is not None else s), "nerf_mlp_bwd_dw")
        if side is not None:
            for t in (ctx.act, dz, ws):  # (freed by this function; the dW stream still reads them)
                if t is not None:
                    t.record_stream(side)
            ev = torch.cuda.Event()
            ev.record(side)
            _DW_PENDING.append((dev, ev))
        ctx.act = ctx.masks = None
        # the net's data-parallel bucket starts after its last pending chunk's dW only (with the
        # dW stream current, the bucket's collective is enqueued behind the dW)
        with torch.cuda.stream(side) if side is not None else contextlib.nullcontext():
            ctx.packer.backward_done(grad if direct is not None else None)
        if direct is not None:
            return nones + (None,) * len(params)
        out, off = [], 0
        for p in params:
            n = p.numel()
            out.append(grad[off:off + n].view_as(p))
            off += n
        return nones + tuple(out)


def mlp(packer: PackedMLP, pts: torch.Tensor, viewdirs: Optional[torch.Tensor], samples_per_dir: int = 1,
        dir_index: Optional[torch.Tensor] = None, dtype=F32, density_only: bool = False) -> torch.Tensor:
    """NeRF MLP on points [...,3] -> raw [M,4] (differentiable w.r.t. the packer's params)."""
    want_grad = torch.is_grad_enabled() and any(p.requires_grad for p in packer.params)
    return _MLP.apply(pts, viewdirs, dir_index, samples_per_dir, packer, dtype_code(dtype), density_only, want_grad,
                      *packer.params)


# --------------------------------------------------------------------------------------
# occupancy grid
# --------------------------------------------------------------------------------------
def _bbox_arr(bbox):
    flat = [float(v) for v in bbox[0]] + [float(v) for v in bbox[1]]
    arr = (_ctypes.c_float * 6)(*flat)
    _keepalive.append(arr)
    if len(_keepalive) > 64:
        del _keepalive[:32]
    return _ctypes.cast(arr, _ctypes.c_void_p)


_keepalive = []


def grid_index(pts: torch.Tensor, grid: Optional[torch.Tensor], res: int, bbox=SCENE_BBOX, want_idx: bool = True):
    pts = _f32c(pts.reshape(-1, 3), "pts")
    M = pts.shape[0]
    idx = torch.empty(M, 3, dtype=torch.int64, device=pts.device) if want_idx else None
    occ = torch.empty(M, dtype=torch.uint8, device=pts.device) if grid is not None else None
    g = grid.to(torch.uint8).contiguous() if grid is not None else None
    check(lib().nerf_grid_index(ptr(pts), M, _bbox_arr(bbox), res, ptr(g), ptr(idx), ptr(occ), stream_of(pts)),
          "nerf_grid_index")
    return idx, (occ.bool() if occ is not None else None)


def bake_lattice_exact(res: int, bbox=SCENE_BBOX) -> bool:
    """True when bmin + L*voxel == (bmin + (L-1)*voxel) + voxel in fp32 for every lattice L,
    i.e. the (res+1)^3 shared-corner evaluation is bit-identical to the 8-corner one."""
    import numpy as np
    for k in range(3):
        mn, mx = np.float32(bbox[0][k]), np.float32(bbox[1][k])
        vs = np.float32(np.float32(mx - mn) / np.float32(res))
        L = np.arange(1, res + 1, dtype=np.float32)
        a = np.float32(mn) + (L * vs).astype(np.float32)
        b = (np.float32(mn) + ((L - 1) * vs).astype(np.float32)).astype(np.float32) + vs
        if not np.array_equal(a.astype(np.float32), b.astype(np.float32)):
            return False
    return True


def bake(packer: PackedMLP, res: int, threshold: float, bbox=SCENE_BBOX, dtype=F32, device=None,
         dedup: Optional[bool] = None, return_sigma: bool = False, slab=None):
    """Occupancy grid bake -> bool [res,res,res] (occupancy_grid.py:15-80); with slab=(x0, x1)
    only the voxels x0 <= ix < x1 -> bool [x1-x0,res,res] (one rank's share)."""
    device = device or packer.params[0].device
    if dedup is None:
        dedup = bake_lattice_exact(res, bbox)
    x0, x1 = (0, res) if slab is None else (int(slab[0]), int(slab[1]))
    L = lib()
    P = L.nerf_bake_num_points_slab(res, int(dedup), x0, x1)
    if P < 0:
        raise ValueError(f"bake: bad slab {(x0, x1)} for res {res}")
    grid = torch.zeros(x1 - x0, res, res, device=device, dtype=torch.uint8)
    if P == 0:  # an empty slab (more ranks than voxel planes)
        if return_sigma:
            return grid.bool(), torch.empty(0, device=device), torch.empty(0, 3, device=device)
        return grid.bool()
    pts = torch.empty(P, 3, device=device, dtype=torch.float32)
    s = stream_of(pts)
    check(L.nerf_bake_points_slab(res, _bbox_arr(bbox), int(dedup), x0, x1, ptr(pts), s), "nerf_bake_points")
    with torch.no_grad():
        raw = mlp(packer, pts, None, 1, None, dtype, density_only=True)
    check(L.nerf_bake_reduce_slab(ptr(raw), res, int(dedup), x0, x1, float(threshold), ptr(grid), s),
          "nerf_bake_reduce")
    if return_sigma:
        return grid.bool(), raw[:, 3].clamp_min(0), pts
    return grid.bool()


MARCH_POINT_BYTES = 4 + 4 + 12 + 16  # out_ray, out_step, out_pts, raw per gathered point


def mlp_count(packer: PackedMLP, pts: torch.Tensor, viewdirs: torch.Tensor, dir_index: torch.Tensor,
              M_dev: torch.Tensor, raw: torch.Tensor, dtype=F32) -> torch.Tensor:
    """Inference MLP on the first min(M_dev[0], cap) points, the count read on the device
    (nerf_mlp_fwd_count): no host round trip sizes the launch.  raw: [cap,4] (output)."""
    code = dtype_code(dtype)
    cap = int(raw.shape[0])
    check(lib().nerf_mlp_fwd_count(ptr(packer.get(code, 0)), code, ptr(pts), ptr(viewdirs), 1, ptr(dir_index),
                                   ptr(M_dev), cap, ptr(raw), stream_of(pts)), "nerf_mlp_fwd_count")
    return raw


def march(packer: PackedMLP, rays: torch.Tensor, near: float, far: float, grid: torch.Tensor, step_size: float = 0.005,
          t_thresh: float = 1e-4, bbox=SCENE_BBOX, white_bkgd: bool = True, dtype=F32,
          t_table: Optional[torch.Tensor] = None, k_schedule=(12, 24, 48, 96, 192, 384, 768),
          round_bytes: int = 1 << 31, k_low: int = 8, t_split: float = 0.9, sync_every: int = 4,
          use_macro: bool = True, one_pass: bool = True, k_low_grow: int = 8):
    """Grid-accelerated march with early termination -> dict(rgb_map_f, depth_map_f,
    acc_map_f, n_queried, n_evaluated, rounds).

    Each round gathers up to K occupied steps of every alive ray into one point buffer of
    ``cap`` points (round_bytes / MARCH_POINT_BYTES, <= INT32_MAX), evaluates them in one MLP
    launch and composites them; compositing stops at T < t_thresh, so points past a ray's
    termination were evaluated speculatively; a ray whose transmittance is already below
    t_split gathers at most k_low steps (it is about to terminate; on the trained fixture net's
    800x800 view this cut the speculative evaluations from 48 % to 6 % of the queries,
    profiles/r2/march_sweep.json).  The rounds run without host round trips: the MLP reads the
    gather's point count on the device (mlp_count), a ray that finds no room in the buffer
    gathers again next round, and the host checks for live rays every ``sync_every`` rounds
    (rounds after the last live one find nothing and cost a few empty launches).  The walk
    skips empty cells, and whole empty 8^3 blocks of cells (use_macro), exactly; one_pass
    writes the points from the runs the counting walk recorded (no second walk).  With
    k_low_grow = g > 0 the low-transmittance rays' k_low doubles every round from round g on
    (fewer straggler rounds; the trained fixture's 800x800 view: 20 -> 12 rounds, bf16 frame
    0.0172 s two-pass / 0.0155 one-pass / 0.0146 with k_low_grow 8, tools/march_bench.py,
    profiles/r3/march_sweep.json).  n_queried
    counts the composited points only -- exactly the reference's MLP queries
    (volume_renderer.py:324) -- and n_evaluated every point the MLP ran on.  ``rounds`` counts
    the rounds that had live rays (``rounds_launched`` also counts the up to sync_every - 1
    empty rounds after the last one).  The point buffer is sized once per call for the
    largest round the byte budget allows (up to round_bytes, ~2.1 GB at the default); it
    comes from PyTorch's caching allocator, so consecutive frames (and in-training
    validation) reuse one block rather than allocating it again."""
    rays = _f32c(rays.reshape(-1, 6), "rays")
    dev, N = rays.device, rays.shape[0]
    L = lib()
    s = stream_of(rays)
    if N == 0:
        z = torch.zeros(0, device=dev)
        return {"rgb_map_f": torch.zeros(0, 3, device=dev), "depth_map_f": z, "acc_map_f": z.clone(), "n_queried": 0,
                "n_evaluated": 0, "rounds": 0}
    if t_table is None:
        t_table = device_table("arange", float(near), float(far), float(step_size), dev)
    t_table = _f32c(t_table.to(dev), "t_table")
    n_steps = t_table.numel()
    g = grid.to(device=dev, dtype=torch.uint8).contiguous()
    res = grid.shape[0]
    T = torch.empty(N, device=dev)
    rgb = torch.empty(N, 3, device=dev)
    depth = torch.empty(N, device=dev)
    acc = torch.empty(N, device=dev)
    nxt = torch.empty(N, dtype=torch.int32, device=dev)
    alive = torch.empty(N, dtype=torch.uint8, device=dev)
    exh = torch.empty(N, dtype=torch.uint8, device=dev)
    one_pass = one_pass and n_steps < 65536  # (the one-pass runs hold 16-bit step indices)
    start = None if one_pass else torch.empty(N, dtype=torch.int32, device=dev)
    off = torch.empty(N, dtype=torch.int32, device=dev)
    cnt = torch.empty(N, dtype=torch.int32, device=dev)
    counters = torch.zeros(2, dtype=torch.int32, device=dev)
    stats = torch.zeros(2, dtype=torch.int64, device=dev)  # [0] composited (queried), [1] evaluated
    # the largest K times every ray, or the byte budget (a ray that does not fit waits a round)
    cap = max(1, min(N * max(k_schedule), round_bytes // MARCH_POINT_BYTES, 2 ** 31 - 1))
    cap = max(cap, max(k_schedule))
    out_ray = torch.empty(cap, dtype=torch.int32, device=dev)
    out_step = torch.empty(cap, dtype=torch.int32, device=dev)
    out_pts = torch.empty(cap, 3, device=dev)
    raw = torch.empty(cap, 4, device=dev)
    # unit view directions of every ray (d / |d|), as render_accelerated computes per query
    _, _, vd = sample_stratified(rays, near, far, 1, False, want_pts=False)
    check(L.nerf_march_init(ptr(T), ptr(rgb), ptr(depth), ptr(acc), ptr(nxt), ptr(alive), ptr(exh), N, s),
          "nerf_march_init")
    bb = _bbox_arr(bbox)
    macro = torch.empty(L.nerf_march_macro_bytes(res), dtype=torch.uint8, device=dev) if use_macro else None
    if macro is not None:
        check(L.nerf_march_macro(ptr(g), res, ptr(macro), s), "nerf_march_macro")
    packer.get(dtype_code(dtype), 0)  # (pack before the rounds)
    rounds = 0
    live_hist = torch.zeros(64, dtype=torch.int32, device=dev)  # rays alive entering each round
    while True:
        # (the gather's int32 reservation counter: alive rays x K < 2^31)
        K = max(1, min(k_schedule[min(rounds, len(k_schedule) - 1)], cap, (2 ** 31 - 1) // max(N, 1)))
        kl = k_low if k_low_grow <= 0 or rounds < k_low_grow else k_low << min(20, rounds - k_low_grow + 1)
        kl = max(1, min(kl, K))
        counters.zero_()
        check(L.nerf_march_gather(ptr(rays), N, ptr(t_table), n_steps, ptr(g), res, ptr(macro), bb, K, int(kl),
                                  float(t_split),
                                  ptr(T), ptr(rgb), ptr(depth), ptr(acc), ptr(nxt), ptr(alive), ptr(exh),
                                  ptr(counters), stats[1:].data_ptr(), ptr(start), ptr(out_ray), ptr(out_step),
                                  ptr(out_pts), ptr(off), ptr(cnt), cap, s), "nerf_march_gather")
        with torch.no_grad():
            mlp_count(packer, out_pts, vd, out_ray, counters, raw, dtype)
        check(L.nerf_march_composite(ptr(raw), ptr(rays), N, ptr(t_table), ptr(off), ptr(cnt), ptr(out_step), ptr(T),
                                     ptr(rgb), ptr(depth), ptr(acc), ptr(nxt), ptr(alive), ptr(exh),
                                     float(step_size), float(t_thresh), stats.data_ptr(), s), "nerf_march_composite")
        if rounds >= live_hist.numel():
            live_hist = torch.cat([live_hist, torch.zeros_like(live_hist)])
        live_hist[rounds:rounds + 1].copy_(counters[1:2])
        rounds += 1
        if rounds % sync_every == 0 and int(counters[1]) == 0:
            break
    check(L.nerf_march_finish(ptr(rgb), ptr(acc), N, int(bool(white_bkgd)), s), "nerf_march_finish")
    st = stats.tolist()
    live_rounds = int((live_hist[:rounds] > 0).sum())
    return {"rgb_map_f": rgb, "depth_map_f": depth, "acc_map_f": acc, "n_queried": int(st[0]),
            "n_evaluated": int(st[1]), "rounds": live_rounds, "rounds_launched": rounds}


# --------------------------------------------------------------------------------------
# evaluator metrics
# --------------------------------------------------------------------------------------
def image_metrics(pred: torch.Tensor, gt: torch.Tensor):
    """(psnr, ssim) of fp32 [H,W,3] device images (src/evaluators/nerf.py:23-45): PSNR on the
    floats, skimage-default SSIM on uint8(x*255) with the prediction's uint8 range."""
    pred, gt = _f32c(pred, "pred"), _f32c(gt, "gt")
    if pred.dim() != 3 or pred.shape[-1] != 3 or pred.shape != gt.shape:
        raise ValueError(f"image_metrics: expected two [H,W,3] images, got {tuple(pred.shape)} / {tuple(gt.shape)}")
    H, W = int(pred.shape[0]), int(pred.shape[1])
    ws = torch.empty(lib().nerf_metrics_workspace_bytes(H, W), dtype=torch.uint8, device=pred.device)
    out = torch.empty(4, dtype=torch.float64, device=pred.device)
    check(lib().nerf_image_metrics(ptr(pred), ptr(gt), H, W, ptr(ws), ptr(out), stream_of(pred)), "nerf_image_metrics")
    o = out.tolist()
    return o[0], o[1]


# --------------------------------------------------------------------------------------
# optimizer
# --------------------------------------------------------------------------------------
def adam_step(param: torch.Tensor, grad: torch.Tensor, exp_avg: torch.Tensor, exp_avg_sq: torch.Tensor, lr: float,
              step: int, betas=(0.9, 0.999), eps: float = 1e-8, clip_value: float = 0.0):
    """Fused clip_grad_value_ + Adam over flat contiguous fp32 buffers (in place)."""
    for t in (param, grad, exp_avg, exp_avg_sq):
        if t.dtype != torch.float32 or not t.is_contiguous():
            raise TypeError("adam_step needs contiguous float32 buffers")
    check(lib().nerf_adam_step(ptr(param), ptr(grad), ptr(exp_avg), ptr(exp_avg_sq), param.numel(), float(lr),
                               float(betas[0]), float(betas[1]), float(eps), int(step), float(clip_value),
                               stream_of(param)), "nerf_adam_step")


def param_list(module: torch.nn.Module) -> List[torch.Tensor]:
    """The 24 parameters of one NeRF module in the kernel's (state_dict) order."""
    sd = dict(module.named_parameters())
    return [sd[n] for n in NET_PARAM_NAMES]
