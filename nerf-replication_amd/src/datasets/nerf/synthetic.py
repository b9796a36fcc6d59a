"""A procedural blender-like scene (no dataset is available offline).

Three Lambertian spheres on a checkered slab inside the lego bbox ([-1.5, 1.5]^3), lit by
one directional light, composited on white like the blender loader (blender.py:93-95).
Cameras are ``pose_spherical(theta, phi, 4.0)`` (render_video.py:14-19) with the lego
camera_angle_x, and pixel rays follow Dataset.get_rays (blender.py:13-32: no half-pixel
offset, d not normalised).  Ground truth is analytic ray casting in plain torch, so a scene
of N views builds on any device in milliseconds.  Hard surfaces and the checker texture
give the NeRF a sharp, learnable density -- what the parity fixtures of a trained net and
the PSNR tests need.
"""
import math

import torch

from src.utils.camera import focal_for, pose_spherical

SPHERES = (  # center, radius, albedo
    ((0.0, 0.0, 0.2), 0.55, (0.85, 0.25, 0.2)),
    ((0.6, -0.5, -0.3), 0.35, (0.2, 0.6, 0.9)),
    ((-0.55, 0.45, -0.4), 0.3, (0.3, 0.8, 0.3)),
)
SLAB = ((-0.9, -0.9, -0.75), (0.9, 0.9, -0.6))
CHECKER = ((0.9, 0.85, 0.6), (0.35, 0.3, 0.25))
LIGHT = (0.4, 0.3, 0.85)
AMBIENT = 0.35


def camera_rays(c2w: torch.Tensor, H: int, W: int, focal: float):
    """(o, d) [H*W, 3] of one camera, flat id j*W + i (blender.py:13-32)."""
    dev = c2w.device
    i, j = torch.meshgrid(torch.arange(W, dtype=torch.float32, device=dev),
                          torch.arange(H, dtype=torch.float32, device=dev), indexing="xy")
    dirs = torch.stack([(i - W * 0.5) / focal, -(j - H * 0.5) / focal, -torch.ones_like(i)], -1)
    d = (dirs[..., None, :] * c2w[:3, :3]).sum(-1).reshape(-1, 3)
    o = c2w[:3, 3].expand(d.shape)
    return o, d


def shade(o: torch.Tensor, d: torch.Tensor) -> torch.Tensor:
    """Analytic colour of rays (o, d) [N,3]: nearest hit, Lambert + ambient, white background."""
    dn = d / d.norm(dim=-1, keepdim=True)
    N = o.shape[0]
    dev = o.device
    inf = torch.full((N,), float("inf"), device=dev)
    t_best = inf.clone()
    normal = torch.zeros(N, 3, device=dev)
    albedo = torch.ones(N, 3, device=dev)
    for c, r, a in SPHERES:
        c = torch.tensor(c, device=dev)
        oc = o - c
        b = (oc * dn).sum(-1)
        disc = b * b - ((oc * oc).sum(-1) - r * r)
        t = -b - torch.sqrt(disc.clamp_min(0.0))
        hit = (disc > 0) & (t > 0) & (t < t_best)
        t_best = torch.where(hit, t, t_best)
        p = o + t[:, None] * dn
        normal = torch.where(hit[:, None], (p - c) / r, normal)
        albedo = torch.where(hit[:, None], torch.tensor(a, device=dev).expand(N, 3), albedo)
    lo, hi = torch.tensor(SLAB[0], device=dev), torch.tensor(SLAB[1], device=dev)
    inv = 1.0 / torch.where(dn.abs() < 1e-12, torch.full_like(dn, 1e-12), dn)
    t0, t1 = (lo - o) * inv, (hi - o) * inv
    tmin, tmax = torch.minimum(t0, t1), torch.maximum(t0, t1)
    t_in, axis = tmin.max(-1)
    t_out = tmax.min(-1).values
    hit = (t_in < t_out) & (t_in > 0) & (t_in < t_best)
    t_best = torch.where(hit, t_in, t_best)
    n_box = torch.zeros(N, 3, device=dev)
    n_box[torch.arange(N, device=dev), axis] = -torch.sign(dn[torch.arange(N, device=dev), axis])
    p = o + t_in[:, None] * dn
    parity = (torch.floor(p[:, 0] * 2.5) + torch.floor(p[:, 1] * 2.5)).remainder(2.0)
    chk = torch.where(parity[:, None] > 0.5, torch.tensor(CHECKER[0], device=dev), torch.tensor(CHECKER[1], device=dev))
    normal = torch.where(hit[:, None], n_box, normal)
    albedo = torch.where(hit[:, None], chk, albedo)
    light = torch.tensor(LIGHT, device=dev)
    light = light / light.norm()
    lam = AMBIENT + (1.0 - AMBIENT) * (normal * light).sum(-1).clamp_min(0.0)
    rgb = albedo * lam[:, None]
    return torch.where(torch.isfinite(t_best)[:, None], rgb, torch.ones_like(rgb))


def view_poses(n: int, seed: int, phi_range=(-60.0, -20.0)) -> torch.Tensor:
    """n cameras on the radius-4 sphere: theta uniform over a turn, phi in phi_range."""
    g = torch.Generator().manual_seed(seed)
    th = torch.rand(n, generator=g) * 360.0 - 180.0
    ph = phi_range[0] + torch.rand(n, generator=g) * (phi_range[1] - phi_range[0])
    return torch.stack([pose_spherical(float(a), float(b), 4.0) for a, b in zip(th, ph)])


def make_scene(n_views: int, H: int, W: int, device, seed: int = 0):
    """-> images [n,H,W,3] fp32, poses [n,4,4] fp32 (device), focal (lego camera angle)."""
    poses = view_poses(n_views, seed).to(device)
    focal = focal_for(W)
    imgs = []
    for k in range(n_views):
        o, d = camera_rays(poses[k], H, W, focal)
        imgs.append(shade(o, d).reshape(H, W, 3))
    return torch.stack(imgs), poses, focal


def psnr(pred: torch.Tensor, gt: torch.Tensor) -> float:
    """-10 log10(mean squared error) (src/evaluators/nerf.py:23-26), in float64."""
    mse = float(((pred.double() - gt.double()) ** 2).mean())
    return -10.0 * math.log10(mse)
