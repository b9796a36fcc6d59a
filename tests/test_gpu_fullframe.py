"""BASELINE configs 2 and 4 at full size on the trained net.

Fixture: tests/golden/golden_v4.npz, written by the REFERENCE on the CPU (make_golden_v4.py):
the trained weights (trained_v2.npz) render the WHOLE 800x800 held-out view of golden_v2 with
``render()`` (hierarchical, volume_renderer.py:137-247) and with ``render_accelerated()`` (the
grid march, :268-357) on the reference's own res-128 bake of those weights
(occupancy_grid.main(), golden_v2).  It keeps every key of 4,096 of the frame's rays (3,072
uniform + 1,024 over the object's central crop), the float64 row sums of every key, the
evaluator's uint8 frame and the march's query count over the frame.

Here the whole 640,000-ray frame goes through the drop-in Renderer -- render() in its
262,144-ray render chunks (M = 50.3 M fine samples per MLP launch), render_accelerated() in one
march -- and is compared with NO exclusions:
  * the 4,096 rays, every key: fp32 within 1e-4 (measured 4.6e-5); bf16x3 / bf16x3f every value
    within the north_star's 2e-3 and >= 95 % within 1e-4.  Their render() evaluates the coarse
    net at fp32 (Network.mlp_dtype_for): with a split-bf16 coarse net one fine depth of the 4,096
    was off by 3.4e-3 and four frame pixels by 2-6 uint8 levels, every one of them an importance
    sample moved across a CDF bin by the coarse net's ~1e-5 relative error, which an exact
    (fp64) MLP does not move by more than 1.4e-4 (tools/fullframe_conditioning.py,
    profiles/r5/fullframe_conditioning.json); bf16 (operands rounded to bf16): >= 95 % within 2e-3,
    its documented non-conforming tier, held to 1.5x its own measurement
    (max error, fraction beyond 2e-3 and row-sum error per key; uint8 frame; query count);
  * every row sum within 800 x the per-value bound (so every row of the frame is covered, not
    only the sampled rays);
  * the uint8 frame (clip(rgb) x 255, truncated): fp32 / bf16x3 / bf16x3f every pixel within
    one level (an error below 1/255 moves a truncated value by at most one level), >= 99.9 %
    identical;
  * the march's MLP query count over the frame: within 16 of the reference's 12,383,297
    (measured: fp32 -2, bf16x3 +2; the 256-ray count of test_gpu_trained.py is exact).  A ray
    stops after the first queried step whose transmittance falls below 1e-4
    (volume_renderer.py:340-341), a running product of 1 - alpha over the queried steps; with
    alpha from an MLP that agrees with the reference's to fp32 rounding, not bit for bit, a ray
    whose product lands within an ulp or so of 1e-4 stops one step earlier or later.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
os.environ.setdefault("NERF_AMD_NO_ARGV", "1")
HERE = os.path.dirname(os.path.abspath(__file__))
H = W = 800
RENDER_KEYS = ["rgb_map_c", "depth_map_c", "acc_map_c", "rgb_map_f", "depth_map_f", "acc_map_f"]
MARCH_KEYS = ["rgb_map_f", "depth_map_f", "acc_map_f"]
CONTRACT = 2e-3  # north_star: rgb/depth within 2e-3 for an MLP below fp32
# per tier: (tol, fraction of values within tol, bound on every value, uint8 frame: max levels,
# fraction identical)
BOUNDS = {"fp32": (1e-4, 1.0, 1e-4, 1, 0.999),
          "bf16x3": (1e-4, 0.95, CONTRACT, 1, 0.999),
          "bf16x3f": (1e-4, 0.95, CONTRACT, 1, 0.999)}
# bf16 (operands rounded to bf16: the documented non-conforming tier) is held to its own measurement
# instead (round 6, gpurun_out/r6/fullframe.log; bf16 is bit-reproducible run to run and box to box, so
# a bound 1.5x the measurement trips on a regression, not on noise): per key (max error, fraction of the
# sampled values beyond 2e-3, largest row-sum error), per frame (largest uint8 difference, pixels more than
# one level off), and the march's query-count offset from the reference's.
BF16_MEASURED = {
    "render": {"keys": {"rgb_map_c": (1.8e-2, 0.0157, 0.42), "depth_map_c": (1.0e-1, 0.0217, 1.3),
                        "acc_map_c": (2.1e-2, 0.0085, 0.34), "rgb_map_f": (1.8e-1, 0.0151, 0.73),
                        "depth_map_f": (7.5e-1, 0.0225, 2.0), "acc_map_f": (1.5e-1, 0.0039, 0.52)},
               "u8_max": 121, "u8_px_over_1": 4183},
    "march": {"keys": {"rgb_map_f": (1.1e-2, 0.0076, 0.38), "depth_map_f": (3.9e-2, 0.0125, 0.52),
                       "acc_map_f": (1.0e-2, 0.0049, 0.14)},
              "u8_max": 5, "u8_px_over_1": 564, "queried_offset": 3979}}
BF16_MARGIN = 1.5
TIERS = list(BOUNDS) + ["bf16"]


@pytest.fixture(scope="module")
def g4():
    return np.load(os.path.join(HERE, "golden", "golden_v4.npz"), allow_pickle=False)


@pytest.fixture(scope="module")
def frame(g4, cuda):
    """The frame's 640,000 rays (oracle get_rays = blender.get_rays, pixel j*W + i); the
    sampled rays must be the reference's own, bit for bit."""
    from oracle import nerf_oracle as O
    o, d = O.get_rays(H, W, float(g4["focal"]), torch.from_numpy(g4["pose"]))
    rays = torch.cat([o.reshape(-1, 3), d.reshape(-1, 3)], 1)
    np.testing.assert_array_equal(rays[torch.from_numpy(g4["pix"])].numpy(), g4["rays"])
    return rays.to(cuda)


@pytest.fixture()
def renderer(cuda):
    from src.config import cfg
    from src.models.nerf.network import Network
    from src.models.nerf.renderer.volume_renderer import Renderer
    z = np.load(os.path.join(HERE, "golden", "trained_v2.npz"), allow_pickle=False)
    cfg.task_arg.perturb = 0
    torch.manual_seed(0)
    net = Network()
    net.load_state_dict({k: torch.from_numpy(z[k]) for k in z.files}, strict=True)
    net = net.to(cuda).eval()
    yield net, Renderer(net)
    cfg.task_arg.mlp_dtype = "fp32"


def _compare(out, g4, prefix, keys, dtype):
    pix = torch.from_numpy(g4["pix"]).to(out[keys[0]].device)
    report = {}
    for k in keys:
        full = out[k]
        assert full.shape[0] == H * W, (k, tuple(full.shape))
        got, ref = full[pix].cpu().numpy(), g4[f"{prefix}_{k}"]
        err = np.abs(got.astype(np.float64) - ref)
        rows = full.double().reshape(H, W, -1).sum(1).cpu().numpy()
        rerr = float(np.abs(rows - g4[f"{prefix}_rowsum_{k}"].reshape(H, -1)).max())
        over = float((err > CONTRACT).mean())
        report[k] = (float(err.max()), float((err <= 1e-4).mean()), 1 - over, rerr)
        if dtype == "bf16":
            mx, ov, rw = BF16_MEASURED[prefix]["keys"][k]
            assert err.max() <= BF16_MARGIN * mx and over <= BF16_MARGIN * ov and rerr <= BF16_MARGIN * rw, \
                (prefix, k, dtype, err.max(), over, rerr)
            continue
        tol, frac_min, maxerr, _, _ = BOUNDS[dtype]
        assert err.max() <= maxerr and float((err <= tol).mean()) >= frac_min, (prefix, k, dtype, err.max())
        assert rerr <= W * maxerr, (prefix, k, dtype, rerr)
    print(f"\n{prefix} {dtype}: " + ", ".join(f"{k} max {m:.1e} (<= 1e-4: {f:.4f}, <= 2e-3: {c:.4f}, row {r:.1e})"
                                           for k, (m, f, c, r) in report.items()))
    img = (out["rgb_map_f"].clamp(0, 1) * 255).to(torch.uint8).reshape(H, W, 3).cpu().numpy()
    d = np.abs(img.astype(int) - g4[f"{prefix}_frame_u8"].astype(int))
    over1 = int((d.max(-1) > 1).sum())
    print(f"{prefix} {dtype} uint8 frame: max {d.max()}, identical {(d == 0).mean():.5f}, "
          f"within one level {(d <= 1).mean():.6f}, pixels off by > 1: {over1}")
    if dtype == "bf16":
        m = BF16_MEASURED[prefix]
        assert d.max() <= BF16_MARGIN * m["u8_max"] and over1 <= BF16_MARGIN * m["u8_px_over_1"], (prefix, d.max(), over1)
    else:
        _, _, _, max_levels, ident_min = BOUNDS[dtype]
        assert d.max() <= max_levels and (d == 0).mean() >= ident_min, (prefix, dtype, d.max(), (d == 0).mean())


@pytest.mark.parametrize("dtype", TIERS)
def test_config2_full_frame_render(g4, frame, renderer, dtype):
    """Config 2: the 800x800 frame through Renderer.render (262,144-ray render chunks)."""
    net, r = renderer
    net.mlp_dtype = dtype
    near, far = torch.tensor([2.0], device=frame.device), torch.tensor([6.0], device=frame.device)
    with torch.no_grad():
        out = r.render({"rays": frame, "near": near, "far": far})
    _compare(out, g4, "render", RENDER_KEYS, dtype)



@pytest.mark.parametrize("dtype", TIERS)
def test_config4_full_frame_march(g4, frame, renderer, dtype):
    """Config 4: the frame through render_accelerated on the reference's res-128 bake of the
    same weights; the MLP query count over all 640,000 rays against the reference's."""
    net, r = renderer
    net.mlp_dtype = dtype
    g2 = np.load(os.path.join(HERE, "golden", "golden_v2.npz"), allow_pickle=False)
    grid = torch.from_numpy(np.unpackbits(g2["bake128_packed"])[: 128 ** 3].reshape(128, 128, 128).astype(bool))
    r.set_occupancy_grid(grid, frame.device)
    np.testing.assert_array_equal(
        torch.arange(2.0, 6.0, 0.005).numpy(), g4["march_t_table"])  # the t table, as the reference built it
    near, far = torch.tensor([2.0], device=frame.device), torch.tensor([6.0], device=frame.device)
    with torch.no_grad():
        out = r.render_accelerated({"rays": frame, "near": near, "far": far})
    _compare(out, g4, "march", MARCH_KEYS, dtype)
    ref_q = int(g4["march_queried"])
    print(f"march {dtype}: queried {out['n_queried']} (reference {ref_q}), evaluated {out['n_evaluated']}")
    allow = 16 if dtype != "bf16" else int(BF16_MARGIN * BF16_MEASURED["march"]["queried_offset"])
    assert abs(out["n_queried"] - ref_q) <= allow, (dtype, out["n_queried"] - ref_q)


@pytest.mark.parametrize("dtype", ["bf16x3", "bf16x3f"])
def test_selective_coarse_pass_scatter(g4, renderer, dtype):
    """The opt-in selective coarse pass (round 6, volume_renderer.py) on the fixture's 4,096 sampled rays: every
    ray flagged (abs_tol 2 > any CDF distance) renders exactly the default fp32-coarse render; with every
    tolerance 0 the rays nerf_composite_pdf_fragile flags render exactly as the fp32-coarse render and all other
    rays exactly as the render with the coarse net in the tier's own arithmetic -- the re-evaluation and its
    scatter change the flagged rays and nothing else, bit for bit."""
    from nerf_amd import ops
    from src.config import cfg
    net, r = renderer
    net.mlp_dtype = dtype
    dev = next(net.parameters()).device
    rays = torch.from_numpy(g4["rays"]).to(dev)
    near, far = torch.tensor([2.0], device=dev), torch.tensor([6.0], device=dev)
    keys = ("fragile_rel_tol", "fragile_abs_tol", "fragile_den_tol", "fragile_z_tol")
    saved = {k: cfg.task_arg.get(k) for k in ("coarse_inference_dtype",) + keys}

    def render(mode, tols=(0.0, 0.0, 0.0, 0.0)):
        cfg.task_arg.coarse_inference_dtype = mode
        for k, v in zip(keys, tols):
            cfg.task_arg[k] = v
        r.fragile_rays = 0
        with torch.no_grad():
            return r.render({"rays": rays, "near": near, "far": far}), r.fragile_rays

    try:
        fp32, _ = render("fp32")
        tier, _ = render(dtype)
        allf, n_all = render("selective", (0.0, 2.0, 0.0, 0.0))
        zero, n_zero = render("selective")
        with torch.no_grad():  # the flags of the all-zero tolerances, as the renderer computes them
            z, pts, vd = ops.sample_stratified(rays, near, far, int(cfg.task_arg.N_samples), False)
            raw = net(pts, vd, "coarse", dtype=dtype)
            flag = ops.composite_sample_pdf_fragile(raw, z, rays, bool(cfg.task_arg.white_bkgd),
                                                    int(cfg.task_arg.N_importance), 0.0, 0.0)[4].bool()
    finally:
        for k, v in saved.items():
            if v is None:
                cfg.task_arg.pop(k, None)
            else:
                cfg.task_arg[k] = v
    assert n_all == rays.shape[0] and n_zero == int(flag.sum()), (n_all, n_zero, int(flag.sum()))
    assert any(not torch.equal(fp32[k], tier[k]) for k in RENDER_KEYS)  # (the two coarse passes differ)
    print(f"\nselective {dtype}: {n_zero} of {rays.shape[0]} rays flagged at zero tolerances")
    for k in RENDER_KEYS:
        assert torch.equal(allf[k], fp32[k]), k
        assert torch.equal(zero[k][flag], fp32[k][flag]), k
        assert torch.equal(zero[k][~flag], tier[k][~flag]), k
