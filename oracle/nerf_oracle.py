"""CPU restatement of the reference NeRF hot path -- TEST INFRASTRUCTURE ONLY.

This module is the *checker* for the HIP path.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it.
The product path (``nerf-replication_amd/``) never imports, calls or falls back to
anything here.

It restates, op for op and in fp32 on torch-CPU, the algorithm of
echo636/nerf-replication (snapshot mounted at /root/reference):

  * pinhole rays                    src/datasets/nerf/blender.py:13-32
  * spherical poses                 render_video.py:9-19
  * frequency positional encoding   src/models/encoding/freq.py:7-32, encoding/__init__.py:6-18
  * NeRF MLP (8x256, skip@4, views) src/models/nerf/network.py:9-74, 161-192
  * raw2outputs (alpha compositing) src/models/nerf/renderer/volume_renderer.py:20-80
  * sample_pdf (inverse CDF)        volume_renderer.py:82-134
  * render (coarse + fine)          volume_renderer.py:137-247
  * world_to_grid_indices           volume_renderer.py:261-265
  * render_accelerated (grid march) volume_renderer.py:268-357
  * occupancy-grid bake             occupancy_grid.py:15-80
  * loss                            src/train/trainers/nerf.py:15-50
  * PSNR                            src/evaluators/nerf.py:23-26

Parity pinning: every function here is checked against golden vectors produced by
running the reference itself in the build container (``tests/golden/make_golden.py``,
fixtures in ``tests/golden/*.npz``; test ``tests/test_oracle_golden.py``).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, Optional

import numpy as np
import torch
import torch.nn.functional as F

# --------------------------------------------------------------------------------------
# lego.yaml constants (configs/nerf/lego.yaml:13-36, 38-52)
# --------------------------------------------------------------------------------------
N_SAMPLES = 64
N_IMPORTANCE = 128
CHUNK = 4096
XYZ_FREQ = 10
DIR_FREQ = 4
SCENE_BBOX = ((-1.5, -1.5, -1.5), (1.5, 1.5, 1.5))
STEP_SIZE = 0.005
T_THRESHOLD = 1e-4
GRID_RES = 128
GRID_THRESHOLD = 1.0

# parameter order of one NeRF MLP (network.py:22-44: pts_linears, views_linears,
# feature_linear, alpha_linear, rgb_linear) -- also the state_dict order.
LAYER_NAMES = (
    [f"pts_linears.{i}" for i in range(8)]
    + ["views_linears.0", "feature_linear", "alpha_linear", "rgb_linear"]
)


# --------------------------------------------------------------------------------------
# cameras and rays
# --------------------------------------------------------------------------------------
def pose_spherical(theta: float, phi: float, radius: float) -> torch.Tensor:
    """c2w of a camera on a sphere (render_video.py:9-19). fp32 [4,4]."""
    def tr(t):
        return torch.tensor([[1, 0, 0, 0], [0, 1, 0, 0], [0, 0, 1, t], [0, 0, 0, 1]],
                            dtype=torch.float32)

    def rphi(p):
        c, s = np.cos(p), np.sin(p)
        return torch.tensor([[1, 0, 0, 0], [0, c, -s, 0], [0, s, c, 0], [0, 0, 0, 1]],
                            dtype=torch.float32)

    def rth(t):
        c, s = np.cos(t), np.sin(t)
        return torch.tensor([[c, 0, -s, 0], [0, 1, 0, 0], [s, 0, c, 0], [0, 0, 0, 1]],
                            dtype=torch.float32)

    m = tr(radius)
    m = rphi(phi / 180.0 * np.pi) @ m
    m = rth(theta / 180.0 * np.pi) @ m
    flip = torch.tensor(np.array([[-1, 0, 0, 0], [0, 0, 1, 0], [0, 1, 0, 0], [0, 0, 0, 1]]),
                        dtype=torch.float32)
    return flip @ m


def focal_from_angle(W: int, camera_angle_x: float) -> float:
    """blender.py:74-75 (float64 numpy, as the reference)."""
    return float(0.5 * W / np.tan(0.5 * camera_angle_x))


def get_rays(H: int, W: int, focal: float, c2w: torch.Tensor):
    """Pinhole rays, no half-pixel offset, d not normalised (blender.py:13-32).

    Returns rays_o, rays_d, each fp32 [H, W, 3]; flat pixel id = j*W + i.
    """
    ii, jj = torch.meshgrid(torch.arange(W, dtype=torch.float32),
                            torch.arange(H, dtype=torch.float32), indexing="xy")
    cam = torch.stack([(ii - W * 0.5) / focal, -(jj - H * 0.5) / focal,
                       -torch.ones_like(ii)], -1)
    d = (c2w[:3, :3] @ cam[..., None]).squeeze(-1)
    o = c2w[:3, 3].expand(d.shape)
    return o, d


# --------------------------------------------------------------------------------------
# positional encoding
# --------------------------------------------------------------------------------------
def positional_encoding(x: torch.Tensor, n_freqs: int) -> torch.Tensor:
    """[x, sin(2^0 x), cos(2^0 x), ..., sin(2^{L-1} x), cos(2^{L-1} x)] (freq.py:7-32).

    Frequencies are 2.**linspace(0, L-1, L) (exact powers of two).
    """
    bands = 2.0 ** torch.linspace(0.0, n_freqs - 1, steps=n_freqs)  # CPU table (exact powers of two)
    parts = [x]
    for f in bands.to(x.device):
        parts.append(torch.sin(x * f))
        parts.append(torch.cos(x * f))
    return torch.cat(parts, -1)


# --------------------------------------------------------------------------------------
# the MLP (functional form over a {layer_name: (weight, bias)} dict)
# --------------------------------------------------------------------------------------
def split_params(state: Dict[str, torch.Tensor], prefix: str):
    """state_dict -> {layer: (W [out,in], b [out])} for one of 'model' / 'model_fine'."""
    return {n: (state[f"{prefix}.{n}.weight"], state[f"{prefix}.{n}.bias"]) for n in LAYER_NAMES}


def mlp(p, x63: torch.Tensor, d27: torch.Tensor) -> torch.Tensor:
    """NeRF.forward with use_viewdirs=True (network.py:49-74): [M,63],[M,27] -> [M,4]."""
    h = x63
    for i in range(8):
        h = F.relu(F.linear(h, *p[f"pts_linears.{i}"]))
        if i == 4:  # skips=[4]: concat PE(xyz) in front of the hidden state
            h = torch.cat([x63, h], -1)
    alpha = F.linear(h, *p["alpha_linear"])
    feat = F.linear(h, *p["feature_linear"])
    hv = F.relu(F.linear(torch.cat([feat, d27], -1), *p["views_linears.0"]))
    rgb = F.linear(hv, *p["rgb_linear"])
    return torch.cat([rgb, alpha], -1)


def network_forward(p, pts: torch.Tensor, viewdirs: torch.Tensor, chunk: int = CHUNK):
    """Network.forward (network.py:171-192): PE, broadcast view dirs, 4096-row batchify."""
    flat = pts.reshape(-1, pts.shape[-1])
    emb = positional_encoding(flat, XYZ_FREQ)
    dirs = viewdirs[:, None].expand(pts.shape).reshape(-1, 3)
    emb = torch.cat([emb, positional_encoding(dirs, DIR_FREQ)], -1).to(torch.float32)
    outs = [mlp(p, emb[i:i + chunk, :63], emb[i:i + chunk, 63:]) for i in range(0, emb.shape[0], chunk)]
    out = torch.cat(outs, 0)
    return out.reshape(list(pts.shape[:-1]) + [out.shape[-1]])


# --------------------------------------------------------------------------------------
# volume rendering
# --------------------------------------------------------------------------------------
def composite(raw: torch.Tensor, z: torch.Tensor, rays_d: torch.Tensor, white_bkgd: bool = True):
    """raw2outputs (volume_renderer.py:20-80), raw_noise_std = 0.

    Returns rgb [R,3], depth [R], acc [R], weights [R,S].
    """
    delta = z[..., 1:] - z[..., :-1]
    delta = torch.cat([delta, torch.tensor([1e10], device=z.device).expand(delta[..., :1].shape)], -1)
    delta = delta * torch.norm(rays_d[..., None, :], dim=-1)
    color = torch.sigmoid(raw[..., :3])
    sigma = F.relu(raw[..., 3])
    alpha = 1.0 - torch.exp(-sigma * delta)
    ones = torch.ones((alpha.shape[0], 1), device=alpha.device)
    trans = torch.cumprod(torch.cat([ones, 1.0 - alpha + 1e-10], -1), -1)[:, :-1]
    w = alpha * trans
    rgb = torch.sum(w[..., None] * color, -2)
    depth = torch.sum(w * z, -1)
    acc = torch.sum(w, -1)
    if white_bkgd:
        rgb = rgb + (1.0 - acc[..., None])
    return rgb, depth, acc, w


@dataclass
class PdfResult:
    samples: torch.Tensor   # [R, N]
    cdf: torch.Tensor       # [R, nb]
    inds: torch.Tensor      # [R, N] int64 (searchsorted, right=True)
    u: torch.Tensor         # [R, N]


def sample_pdf(bins: torch.Tensor, weights: torch.Tensor, n: int, det: bool,
               u: Optional[torch.Tensor] = None) -> PdfResult:
    """Inverse-CDF sampling (volume_renderer.py:82-134). ``u`` injects the uniforms."""
    w = weights + 1e-5
    pdf = w / torch.sum(w, -1, keepdim=True)
    cdf = torch.cat([torch.zeros_like(pdf[..., :1]), torch.cumsum(pdf, -1)], -1)
    if u is None:
        if det:
            u = torch.linspace(0.0, 1.0, steps=n).to(cdf.device).expand(list(cdf.shape[:-1]) + [n])
        else:
            u = torch.rand(list(cdf.shape[:-1]) + [n], device=cdf.device)
    u = u.contiguous()
    inds = torch.searchsorted(cdf, u, right=True)
    lo = torch.clamp(inds - 1, min=0)
    hi = torch.clamp(inds, max=cdf.shape[-1] - 1)
    idx = torch.stack([lo, hi], -1)
    shape = [idx.shape[0], idx.shape[1], cdf.shape[-1]]
    cdf_g = torch.gather(cdf.unsqueeze(1).expand(shape), 2, idx)
    bins_g = torch.gather(bins.unsqueeze(1).expand(shape), 2, idx)
    den = cdf_g[..., 1] - cdf_g[..., 0]
    den = torch.where(den < 1e-5, torch.ones_like(den), den)
    t = (u - cdf_g[..., 0]) / den
    s = bins_g[..., 0] + t * (bins_g[..., 1] - bins_g[..., 0])
    return PdfResult(s, cdf, inds, u)


def samples_from_cdf(bins: torch.Tensor, cdf: torch.Tensor, u: torch.Tensor):
    """Second half of sample_pdf (volume_renderer.py:117-132) on a given CDF.

    Lets tests check the kernel's searchsorted/interpolation bit for bit on the kernel's own
    CDF (whose normalising sum may differ from torch's CPU reduction by an ulp).
    Returns (samples, inds).
    """
    inds = torch.searchsorted(cdf, u.contiguous(), right=True)
    lo = torch.clamp(inds - 1, min=0)
    hi = torch.clamp(inds, max=cdf.shape[-1] - 1)
    cb, ca = torch.gather(cdf, 1, lo), torch.gather(cdf, 1, hi)
    bb, ba = torch.gather(bins, 1, lo), torch.gather(bins, 1, hi)
    den = ca - cb
    den = torch.where(den < 1e-5, torch.ones_like(den), den)
    t = (u - cb) / den
    return bb + t * (ba - bb), inds


def stratified_z(n_rays: int, near, far, n: int = N_SAMPLES, t_rand: Optional[torch.Tensor] = None, device=None):
    """Stratified depths (volume_renderer.py:165-181); t_rand given => perturbed."""
    t = torch.linspace(0.0, 1.0, steps=n, dtype=torch.float32).to(device or "cpu")  # CPU linspace, as the reference
    if torch.is_tensor(near):
        near, far = near.to(t.device), far.to(t.device)
    z = near * (1.0 - t) + far * t
    z = z.expand([n_rays, n])
    if t_rand is not None:
        mids = 0.5 * (z[..., 1:] + z[..., :-1])
        upper = torch.cat([mids, z[..., -1:]], -1)
        lower = torch.cat([z[..., :1], mids], -1)
        z = lower + (upper - lower) * t_rand
    return z


def render(coarse, fine, rays: torch.Tensor, near, far, perturb: bool = False,
           t_rand: Optional[torch.Tensor] = None, u: Optional[torch.Tensor] = None,
           white_bkgd: bool = True, chunk: int = CHUNK, keep: bool = False):
    """Renderer.render (volume_renderer.py:137-247) for [N,6] rays.

    ``coarse``/``fine`` are split_params() dicts.  When ``perturb`` the stratified
    jitter and the importance uniforms are ``t_rand`` [N,64] / ``u`` [N,128] if given
    (else torch.rand).  Returns the six rgb/depth/acc maps; with ``keep`` also the
    intermediates (z, weights_c, z_fine, raw).
    """
    rays = rays.reshape(-1, 6)
    outs = {}
    for s in range(0, rays.shape[0], chunk):
        rc = rays[s:s + chunk]
        o, d = rc[:, 0:3], rc[:, 3:6]
        R = o.shape[0]
        tr = None
        if perturb:
            tr = t_rand[s:s + chunk] if t_rand is not None else torch.rand([R, N_SAMPLES], device=rc.device)
        z = stratified_z(R, near, far, N_SAMPLES, tr, device=rc.device)
        pts = o[..., None, :] + d[..., None, :] * z[..., :, None]
        vd = d / torch.norm(d, dim=-1, keepdim=True)
        raw_c = network_forward(coarse, pts, vd)
        rgb_c, dep_c, acc_c, w_c = composite(raw_c, z, d, white_bkgd)
        zmid = 0.5 * (z[..., 1:] + z[..., :-1])
        uc = None if (u is None or not perturb) else u[s:s + chunk]
        pdf = sample_pdf(zmid, w_c[..., 1:-1], N_IMPORTANCE, det=not perturb, u=uc)
        zs = pdf.samples.detach()
        zf, _ = torch.sort(torch.cat([z, zs], -1), -1)
        pts_f = o[..., None, :] + d[..., None, :] * zf[..., :, None]
        raw_f = network_forward(fine, pts_f, vd)
        rgb_f, dep_f, acc_f, _ = composite(raw_f, zf, d, white_bkgd)
        ret = dict(rgb_map_c=rgb_c, depth_map_c=dep_c, acc_map_c=acc_c,
                   rgb_map_f=rgb_f, depth_map_f=dep_f, acc_map_f=acc_f)
        if keep:
            ret.update(z_vals=z, weights_c=w_c, z_vals_f=zf, raw_c=raw_c, raw_f=raw_f,
                       cdf=pdf.cdf, inds=pdf.inds, z_samples=pdf.samples)
        for k, v in ret.items():
            outs.setdefault(k, []).append(v)
    return {k: torch.cat(v, 0) for k, v in outs.items()}


def loss_fn(ret, gt_rgb: torch.Tensor):
    """MSE(c) + MSE(f) (src/train/trainers/nerf.py:21-29)."""
    lc = F.mse_loss(ret["rgb_map_c"], gt_rgb)
    lf = F.mse_loss(ret["rgb_map_f"], gt_rgb)
    return lc + lf, lc, lf


# --------------------------------------------------------------------------------------
# occupancy grid
# --------------------------------------------------------------------------------------
def grid_indices(pts: torch.Tensor, bbox=SCENE_BBOX, res: int = GRID_RES) -> torch.Tensor:
    """world_to_grid_indices (volume_renderer.py:261-265): clamp, normalise, x(res-1), trunc."""
    bmin = torch.tensor(bbox[0], dtype=torch.float32)
    bmax = torch.tensor(bbox[1], dtype=torch.float32)
    p = torch.clamp(pts, bmin, bmax)
    n = (p - bmin) / (bmax - bmin)
    return (n * (torch.tensor([res] * 3) - 1)).long()


def arange_table(near: float, far: float, step: float = STEP_SIZE) -> torch.Tensor:
    """The march's t table, torch.arange on CPU (volume_renderer.py:298)."""
    return torch.arange(near, far, step)


def render_accelerated(fine, rays: torch.Tensor, near: float, far: float,
                       grid: torch.Tensor, t_table: Optional[torch.Tensor] = None,
                       bbox=SCENE_BBOX, white_bkgd: bool = True, step: float = STEP_SIZE,
                       t_thresh: float = T_THRESHOLD):
    """Occupancy-grid ray march with early termination (volume_renderer.py:268-357).

    Returns rgb_map_f [N,3], depth_map_f [N], acc_map_f [N] and the number of MLP-queried
    points.
    """
    rays = rays.reshape(-1, 6)
    o, d = rays[:, 0:3], rays[:, 3:6]
    N = o.shape[0]
    res = grid.shape[0]
    rgb = torch.zeros_like(o)
    depth = torch.zeros(N)
    acc = torch.zeros(N)
    T = torch.ones(N)
    alive = torch.ones(N, dtype=torch.bool)
    queried = 0
    if t_table is None:
        t_table = arange_table(near, far, step)
    for t in t_table:
        if not bool(alive.any()):
            break
        ai = torch.where(alive)[0]
        ao, ad = o[ai], d[ai]
        p = ao + t * ad
        gi = grid_indices(p, bbox, res)
        occ = grid[gi[:, 0], gi[:, 1], gi[:, 2]]
        if not bool(occ.any()):
            continue
        qp, qd = p[occ], ad[occ]
        vd = qd / torch.norm(qd, dim=-1, keepdim=True)
        raw = network_forward(fine, qp.unsqueeze(1), vd).squeeze(1)
        queried += qp.shape[0]
        c = torch.sigmoid(raw[..., :3])
        sig = F.relu(raw[..., 3])
        a = 1.0 - torch.exp(-sig * (step * torch.norm(qd, dim=-1)))
        gidx = ai[occ]
        Tq = T[gidx]
        rgb[gidx] += Tq.unsqueeze(-1) * a.unsqueeze(-1) * c
        acc[gidx] += Tq * a
        depth[gidx] += Tq * a * t
        T[gidx] *= (1.0 - a)
        alive[gidx[T[gidx] < t_thresh]] = False
    if white_bkgd:
        rgb += (1.0 - acc).unsqueeze(-1) * torch.ones_like(rgb)
    return dict(rgb_map_f=rgb, depth_map_f=depth, acc_map_f=acc, n_queried=queried)


def bake_points(res: int = GRID_RES, bbox=SCENE_BBOX, block=None) -> torch.Tensor:
    """Voxel-corner points (occupancy_grid.py:24-41) -> [V, 8, 3].

    ``block`` = ((x0,x1),(y0,y1),(z0,z1)) restricts to a sub-block of voxels.
    """
    bmin = torch.tensor(bbox[0], dtype=torch.float32)
    bmax = torch.tensor(bbox[1], dtype=torch.float32)
    voxel = (bmax - bmin) / torch.tensor([res, res, res], dtype=torch.float32)
    corner = [torch.linspace(0.0, 1.0, 2) * voxel[k] for k in range(3)]
    corner = torch.stack(torch.meshgrid(*corner, indexing="ij"), -1).view(-1, 3)
    if block is None:
        block = ((0, res), (0, res), (0, res))
    rng = [torch.arange(a, b) for a, b in block]
    idx = torch.stack(torch.meshgrid(*rng, indexing="ij"), -1).float()
    base = bmin + idx * voxel
    pts = base.unsqueeze(3) + corner.view(1, 1, 1, 8, 3)
    return pts.view(-1, 8, 3)


def bake_grid(coarse, res: int = GRID_RES, bbox=SCENE_BBOX, threshold: float = GRID_THRESHOLD,
              block=None, batch: int = 4096):
    """occupancy_grid.py:43-70: sigma=relu(coarse raw[3]) at 8 corners, any(sigma>thr).

    Returns (occupancy bool [bx,by,bz], sigma [V,8]).
    """
    pts = bake_points(res, bbox, block)
    V = pts.shape[0]
    sig = torch.empty(V, 8)
    with torch.no_grad():
        for s in range(0, V, batch):
            e = min(s + batch, V)
            raw = network_forward(coarse, pts[s:e], torch.zeros(e - s, 3))
            sig[s:e] = F.relu(raw[..., 3])
    if block is None:
        block = ((0, res), (0, res), (0, res))
    shp = [b - a for a, b in block]
    return (sig > threshold).any(-1).view(*shp), sig


# --------------------------------------------------------------------------------------
# metrics
# --------------------------------------------------------------------------------------
def psnr(pred: np.ndarray, gt: np.ndarray) -> float:
    """evaluators/nerf.py:23-26 (float64 numpy)."""
    mse = np.mean((pred - gt) ** 2)
    return float(-10 * np.log(mse) / np.log(10))


def seeded_network_state(seed: int = 0) -> Dict[str, torch.Tensor]:
    """Parameters of Network() right after torch.manual_seed(seed) (network.py:141-159).

    nn.Linear default init, created in the reference's order: for model then
    model_fine: pts_linears[0..7], views_linears[0], feature, alpha, rgb.
    """
    torch.manual_seed(seed)
    state = {}
    shapes = [(256, 63)] + [(256, 256)] * 4 + [(256, 319)] + [(256, 256)] * 2
    shapes += [(128, 283), (256, 256), (1, 256), (3, 128)]
    for prefix in ("model", "model_fine"):
        for name, (o, i) in zip(LAYER_NAMES, shapes):
            lin = torch.nn.Linear(i, o)
            state[f"{prefix}.{name}.weight"] = lin.weight.detach().clone()
            state[f"{prefix}.{name}.bias"] = lin.bias.detach().clone()
    return state
