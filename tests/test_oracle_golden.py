"""CPU: the oracle (tests-only restatement) reproduces the reference's own outputs.

Golden vectors come from running the reference in the build container
(tests/golden/make_golden.py); the oracle must match them bit for bit (same torch CPU op
sequence), which pins it before it is used as the GPU checker.
"""
import hashlib

import numpy as np
import torch

from oracle import nerf_oracle as O


def T(g, k):
    return torch.from_numpy(g[k])


def test_seeded_weights_are_the_reference_init(golden, seeded_state):
    h = hashlib.sha256()
    for k, v in seeded_state.items():
        h.update(k.encode())
        h.update(v.numpy().tobytes())
    assert h.hexdigest() == str(golden["state_sha256"])
    assert sum(v.numel() for v in seeded_state.values()) == 1191688


def test_rays(golden):
    poses = torch.stack([O.pose_spherical(a, -30.0, 4.0) for a in (-180.0, -36.0, 72.0)])
    np.testing.assert_array_equal(poses.numpy(), golden["poses"])
    f16 = O.focal_from_angle(16, 0.6911112070083618)
    o, d = O.get_rays(16, 16, f16, poses[0])
    np.testing.assert_array_equal(o.numpy(), golden["rays16_o"])
    np.testing.assert_array_equal(d.numpy(), golden["rays16_d"])
    o, d = O.get_rays(800, 800, O.focal_from_angle(800, 0.6911112070083618), poses[1])
    pix = T(golden, "pix800")
    np.testing.assert_array_equal(d.reshape(-1, 3)[pix].numpy(), golden["rays800_d"])


def test_positional_encoding(golden):
    x = T(golden, "pe_x")
    np.testing.assert_array_equal(O.positional_encoding(x, 10).numpy(), golden["pe_xyz"])
    vd = x / torch.norm(x, dim=-1, keepdim=True)
    np.testing.assert_array_equal(O.positional_encoding(vd, 4).numpy(), golden["pe_dir"])


def test_mlp(golden, seeded_state):
    pts, vd = T(golden, "mlp_pts"), T(golden, "mlp_vd")
    with torch.no_grad():
        for prefix, key in (("model", "mlp_raw_coarse"), ("model_fine", "mlp_raw_fine")):
            out = O.network_forward(O.split_params(seeded_state, prefix), pts, vd)
            np.testing.assert_array_equal(out.numpy(), golden[key])


def test_composite(golden):
    rgb, dep, acc, w = O.composite(T(golden, "comp_raw"), T(golden, "comp_z"), T(golden, "comp_d"), True)
    for a, k in ((rgb, "comp_rgb"), (dep, "comp_depth"), (acc, "comp_acc"), (w, "comp_w")):
        np.testing.assert_array_equal(a.numpy(), golden[k])


def test_sample_pdf(golden):
    bins, w = T(golden, "pdf_bins"), T(golden, "pdf_w")
    det = O.sample_pdf(bins, w, 128, det=True)
    np.testing.assert_array_equal(det.samples.numpy(), golden["pdf_det_samples"])
    np.testing.assert_array_equal(det.cdf.numpy(), golden["pdf_det_cdf"])
    np.testing.assert_array_equal(det.inds.numpy(), golden["pdf_det_inds"])
    ru = O.sample_pdf(bins, w, 128, det=False, u=T(golden, "pdf_u"))
    np.testing.assert_array_equal(ru.samples.numpy(), golden["pdf_u_samples"])
    np.testing.assert_array_equal(ru.inds.numpy(), golden["pdf_u_inds"])
    s2, i2 = O.samples_from_cdf(bins, det.cdf, det.u)
    np.testing.assert_array_equal(s2.numpy(), golden["pdf_det_samples"])


def test_render_both_modes(golden, seeded_state):
    C, F = O.split_params(seeded_state, "model"), O.split_params(seeded_state, "model_fine")
    rays = T(golden, "rays")[:64]
    near, far = torch.tensor([2.0]), torch.tensor([6.0])
    with torch.no_grad():
        r0 = O.render(C, F, rays, near, far, keep=True)
        r1 = O.render(C, F, rays, near, far, perturb=True, t_rand=T(golden, "render1_t_rand"),
                      u=T(golden, "render1_u"), keep=True)
    for tag, r in (("render0_", r0), ("render1_", r1)):
        for k in ("rgb_map_c", "depth_map_c", "acc_map_c", "rgb_map_f", "depth_map_f", "acc_map_f", "z_vals_f"):
            np.testing.assert_array_equal(r[k].numpy(), golden[tag + k], err_msg=tag + k)


def test_gradients(golden, seeded_state):
    params = {k: v.clone().requires_grad_(True) for k, v in seeded_state.items()}
    C, F = O.split_params(params, "model"), O.split_params(params, "model_fine")
    ret = O.render(C, F, T(golden, "rays")[:64], torch.tensor([2.0]), torch.tensor([6.0]))
    loss, lc, lf = O.loss_fn(ret, T(golden, "grad_gt"))
    loss.backward()
    np.testing.assert_allclose([float(lc), float(lf)], golden["grad_loss"], rtol=0, atol=0)
    for i, name in enumerate(golden["grad_names"]):
        g = params[str(name)].grad.reshape(-1)
        np.testing.assert_allclose(float(torch.linalg.vector_norm(g.double())), golden["grad_norms"][i], rtol=1e-6)
        np.testing.assert_array_equal(g[T(golden, "grad_sel_idx")[i]].numpy(), golden["grad_sel_val"][i])


def test_grid_indices_and_march(golden, seeded_state):
    z = np.load(__file__.replace("test_oracle_golden.py", "golden/lego_occupancy_grid.npz"))
    shape = tuple(int(v) for v in z["shape"])
    grid = np.unpackbits(z["packed"])[: int(np.prod(shape))].reshape(shape).astype(bool)
    assert hashlib.sha256(grid.tobytes()).hexdigest() == str(golden["grid_sha256"])
    grid = torch.from_numpy(grid)
    gi = O.grid_indices(T(golden, "grid_pts"))
    np.testing.assert_array_equal(gi.numpy(), golden["grid_idx"])
    np.testing.assert_array_equal(grid[gi[:, 0], gi[:, 1], gi[:, 2]].numpy(), golden["grid_occ"])
    np.testing.assert_array_equal(O.arange_table(2.0, 6.0).numpy(), golden["march_t_table"])
    F = O.split_params(seeded_state, "model_fine")
    with torch.no_grad():
        m = O.render_accelerated(F, T(golden, "march_rays"), 2.0, 6.0, grid, T(golden, "march_t_table"))
    assert m["n_queried"] == int(golden["march_sparse_queried"])
    for k in ("rgb_map_f", "depth_map_f", "acc_map_f"):
        np.testing.assert_array_equal(m[k].numpy(), golden["march_sparse_" + k])


def test_bake_res8(golden, seeded_state):
    st = dict(seeded_state)
    st["model.alpha_linear.bias"] = st["model.alpha_linear.bias"] + float(golden["bake8_alpha_bias_shift"])
    occ, sig = O.bake_grid(O.split_params(st, "model"), res=8)
    np.testing.assert_array_equal(occ.numpy(), golden["bake8_grid"])


def test_psnr():
    a = np.zeros((4, 4, 3), np.float32)
    b = np.full((4, 4, 3), 0.1, np.float32)
    assert abs(O.psnr(a, b) - 20.0) < 1e-5
