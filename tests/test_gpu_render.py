"""End-to-end GPU parity of the drop-in modules against the reference goldens:
Network + Renderer.render (perturb 0 and injected-uniform perturb 1), loss gradients,
render_accelerated on the real baked lego grid, and the grid bake."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

os.environ.setdefault("NERF_AMD_NO_ARGV", "1")


@pytest.fixture(scope="module")
def stack(cuda, seeded_state):
    from src.config import cfg
    from src.models.nerf.network import Network
    from src.models.nerf.renderer.volume_renderer import Renderer
    cfg.task_arg.mlp_dtype = "fp32"
    cfg.task_arg.perturb = 0
    torch.manual_seed(0)
    net = Network()
    sd = net.state_dict()
    for k in sd:  # the drop-in reproduces the reference's seeded init bit for bit
        assert torch.equal(sd[k], seeded_state[k]), k
    net = net.to(cuda)
    return cfg, net, Renderer(net)


def _batch(golden, cuda, n=64):
    rays = torch.from_numpy(golden["rays"][:n]).to(cuda)
    return {"rays": rays[None], "near": torch.tensor([2.0], device=cuda), "far": torch.tensor([6.0], device=cuda)}


KEYS = ["rgb_map_c", "depth_map_c", "acc_map_c", "rgb_map_f", "depth_map_f", "acc_map_f"]

# End to end, the fine pass sees the CDF of the coarse weights.  With the seed-0 (untrained)
# net the coarse weights are ~1e-3 and alpha = 1 - exp(-sigma*delta) carries an absolute
# rounding error of ~1 ulp(1.0) on either side (CPU vs GPU exp, MKL vs MFMA accumulation
# order), i.e. ~1e-4 relative: CDF entries move by ~1e-5, a few importance samples move to
# the neighbouring bin, and the fine depth (range 2..6) moves by up to ~3e-4.  Given the
# *same* CDF (north_star: indices bit-exact for identical CDF inputs) the fine pass is held to
# 1e-4 below (test_fine_pass_given_reference_samples).
E2E_FINE_DEPTH_TOL = 6e-4
# Everything else is held to the measured error with ~5-10x margin (MI355X, round 3: fp32
# coarse/rgb/acc <= 1.5e-6, fine depth 2.5e-4; bf16 rgb/acc <= 1.4e-4, coarse depth 2.3e-4,
# fine depth 6.1e-3 -- bf16 moves more fine samples to the neighbouring bin).
E2E_TOL = 1e-5
BF16_TOL = {"depth_map_c": 1.5e-3, "depth_map_f": 1.2e-2}


@pytest.mark.parametrize("dtype,tol", [("fp32", E2E_TOL), ("bf16", 5e-4)])
def test_render_perturb0(golden, cuda, stack, dtype, tol):
    cfg, net, r = stack
    cfg.task_arg.mlp_dtype = dtype
    net.mlp_dtype = dtype
    with torch.no_grad():
        out = r.render(_batch(golden, cuda))
    for k in KEYS:
        ref = golden[f"render0_{k}"]
        t = BF16_TOL.get(k, tol) if dtype == "bf16" else tol
        if k == "depth_map_f" and dtype == "fp32":
            t = E2E_FINE_DEPTH_TOL
        np.testing.assert_allclose(out[k].cpu().numpy(), ref, rtol=0, atol=t, err_msg=k)
    net.mlp_dtype = "fp32"


@pytest.mark.parametrize("perturb", [False, True])
def test_fine_pass_given_reference_samples(golden, cuda, stack, perturb):
    """Fine MLP + compositing on the reference's own merged depths (captured from its
    torch.sort in make_golden.py): rgb/depth/acc within 1e-4 of the reference's outputs."""
    from nerf_amd import ops
    cfg, net, r = stack
    tag = "render1" if perturb else "render0"
    rc = torch.from_numpy(golden["rays"][:64]).to(cuda)
    zf = torch.from_numpy(golden[f"{tag}_z_vals_f"]).to(cuda)
    with torch.no_grad():
        pts = rc[:, None, :3] + rc[:, None, 3:] * zf[..., None]
        vd = rc[:, 3:] / torch.norm(rc[:, 3:], dim=-1, keepdim=True)
        raw_f = net(pts, vd, "fine")
        rgb, dep, acc, _ = ops.composite(raw_f, zf, rc[:, 3:6], True)
    np.testing.assert_allclose(rgb.cpu().numpy(), golden[f"{tag}_rgb_map_f"], rtol=0, atol=1e-4)
    np.testing.assert_allclose(dep.cpu().numpy(), golden[f"{tag}_depth_map_f"], rtol=0, atol=1e-4)
    np.testing.assert_allclose(acc.cpu().numpy(), golden[f"{tag}_acc_map_f"], rtol=0, atol=1e-4)


def test_render_perturb1_injected(golden, cuda, stack, O=None):
    """perturb=1 with the reference's uniforms injected (t_rand [64,64], u [64,128])."""
    from nerf_amd import ops
    cfg, net, r = stack
    rays = torch.from_numpy(golden["rays"][:64]).to(cuda)
    t_rand = torch.from_numpy(golden["render1_t_rand"]).to(cuda)
    u = torch.from_numpy(golden["render1_u"]).to(cuda)
    with torch.no_grad():
        z, pts, vd = ops.sample_stratified(rays, 2.0, 6.0, 64, True, t_rand=t_rand)
        raw_c = net(pts, vd, "coarse")
        rgb_c, dep_c, acc_c, w_c = ops.composite(raw_c, z, rays[:, 3:6], True)
        pdf = ops.sample_pdf(z, w_c, 128, det=False, u=u, rays=rays)
        raw_f = net(pdf["pts_fine"], vd, "fine")
        rgb_f, dep_f, acc_f, _ = ops.composite(raw_f, pdf["z_fine"], rays[:, 3:6], True)
    got = dict(rgb_map_c=rgb_c, depth_map_c=dep_c, acc_map_c=acc_c, rgb_map_f=rgb_f, depth_map_f=dep_f,
               acc_map_f=acc_f)
    for k in KEYS:
        t = E2E_FINE_DEPTH_TOL if k == "depth_map_f" else E2E_TOL
        np.testing.assert_allclose(got[k].cpu().numpy(), golden[f"render1_{k}"], rtol=0, atol=t, err_msg=k)


def test_loss_gradients_match_reference(golden, cuda, stack):
    from src.train.trainers.nerf import NetworkWrapper
    cfg, net, _ = stack
    wrapper = NetworkWrapper(net)
    net.zero_grad()
    batch = _batch(golden, cuda)
    batch["rgbs"] = torch.from_numpy(golden["grad_gt"]).to(cuda)
    _, loss, stats = wrapper(batch)
    loss.backward()
    np.testing.assert_allclose([float(stats["loss_c"]), float(stats["loss_f"])], golden["grad_loss"], rtol=1e-5)
    params = dict(net.named_parameters())
    for i, name in enumerate(golden["grad_names"]):
        g = params[str(name)].grad.reshape(-1).cpu()
        norm = float(torch.linalg.vector_norm(g.double()))
        sel = g[torch.from_numpy(golden["grad_sel_idx"][i])].numpy()
        scale = np.abs(golden["grad_sel_val"][i]).max() + 1e-12
        # coarse grads see no resampling: measured <= 1.1e-6 (norm) / 4.2e-6 (entries);
        # fine grads inherit the fine-sample moves above: <= 2.9e-4 / 7.3e-4
        rn, rs = (2e-3, 4e-3) if str(name).startswith("model_fine.") else (1e-5, 4e-5)
        np.testing.assert_allclose(norm, golden["grad_norms"][i], rtol=rn, err_msg=str(name))
        assert np.abs(sel - golden["grad_sel_val"][i]).max() / scale < rs, name
    net.zero_grad()


def _real_grid():
    path = os.path.join(os.path.dirname(__file__), "golden", "lego_occupancy_grid.npz")
    z = np.load(path)
    shape = tuple(int(v) for v in z["shape"])
    return torch.from_numpy(np.unpackbits(z["packed"])[: int(np.prod(shape))].reshape(shape).astype(bool))


@pytest.mark.parametrize("tag", ["sparse", "dense"])
def test_render_accelerated_real_grid(golden, cuda, stack, tag):
    cfg, net, r = stack
    grid = _real_grid()
    r.set_occupancy_grid(grid, cuda)
    rays = torch.from_numpy(golden["march_rays"]).to(cuda)
    bias = 50.0 if tag == "dense" else 0.0
    with torch.no_grad():
        net.model_fine.alpha_linear.bias += bias
        out = r.render_accelerated({"rays": rays[None], "near": torch.tensor([2.0]), "far": torch.tensor([6.0])})
        net.model_fine.alpha_linear.bias -= bias
    # n_queried counts composited points (the reference's pts_mask count): equal, and the maps
    # within 5x of the measured error (rgb/acc <= 2.3e-6, depth <= 1.0e-5)
    assert out["n_queried"] == int(golden[f"march_{tag}_queried"])
    for k in ("rgb_map_f", "depth_map_f", "acc_map_f"):
        np.testing.assert_allclose(out[k].cpu().numpy(), golden[f"march_{tag}_{k}"], rtol=0,
                                   atol=5e-5 if "depth" in k else 1e-5, err_msg=k)


def test_grid_occupancy_lookup(golden, cuda):
    from nerf_amd import ops
    grid = _real_grid()
    pts = torch.from_numpy(golden["grid_pts"]).to(cuda)
    idx, occ = ops.grid_index(pts, grid.to(cuda), 128)
    np.testing.assert_array_equal(idx.cpu().numpy(), golden["grid_idx"])
    np.testing.assert_array_equal(occ.cpu().numpy(), golden["grid_occ"])


@pytest.mark.parametrize("dedup", [True, False])
def test_bake_res8(golden, cuda, stack, dedup):
    from nerf_amd import ops
    cfg, net, _ = stack
    with torch.no_grad():
        net.model.alpha_linear.bias += float(golden["bake8_alpha_bias_shift"])
        grid = ops.bake(net.model.packer(), 8, 1.0, dtype="fp32", dedup=dedup)
        net.model.alpha_linear.bias -= float(golden["bake8_alpha_bias_shift"])
    np.testing.assert_array_equal(grid.cpu().numpy(), golden["bake8_grid"])


def test_bake_lattice_exact_for_lego():
    from nerf_amd import ops
    assert ops.bake_lattice_exact(128)
    assert ops.bake_lattice_exact(8)


def test_render_video_frames(cuda, stack):
    """render_video.py (reference render_video.py:21-70): turntable poses, GPU ray
    generation, hierarchical render; here 3 frames of a 48x48 camera, no files written."""
    import render_video
    cfg, _, _ = stack
    H, W = cfg.test_dataset.H, cfg.test_dataset.W
    cfg.test_dataset.H, cfg.test_dataset.W = 48, 48
    try:
        frames = render_video.render_360_video(num_frames=3, write=False)
    finally:
        cfg.test_dataset.H, cfg.test_dataset.W = H, W
    assert len(frames) == 3
    for f in frames:
        assert f.shape == (48, 48, 3) and f.dtype == np.uint8
    assert not np.array_equal(frames[0], frames[1])  # the camera moved


def test_march_repeat_frames_and_grid_change(golden, cuda, stack):
    """Two frames of the same rays and grid are bit-identical (counts included), and an
    in-place change of the grid is seen by the next frame.  (Keeping the uint8 grid, its macro
    blocks and the work buffers between frames was measured and not kept: bf16 0.0148 s vs
    0.0146 s per 800x800 frame -- the launches run ahead of the GPU, host setup is hidden.)"""
    from nerf_amd import ops
    cfg, net, r = stack
    grid = _real_grid().to(cuda)
    rays = torch.from_numpy(golden["march_rays"]).to(cuda)
    p = net.model_fine.packer()
    with torch.no_grad():
        a = ops.march(p, rays, 2.0, 6.0, grid)
        b = ops.march(p, rays, 2.0, 6.0, grid)
        grid.zero_()
        c = ops.march(p, rays, 2.0, 6.0, grid)
    for k in ("rgb_map_f", "depth_map_f", "acc_map_f"):
        assert torch.equal(a[k], b[k]), k
    assert a["n_queried"] == b["n_queried"] > 0 and a["n_evaluated"] == b["n_evaluated"]
    assert c["n_queried"] == 0 and float(c["acc_map_f"].abs().max()) == 0.0
