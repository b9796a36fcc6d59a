"""Generate golden vectors by running the REFERENCE implementation (build container only).

Usage (from the repo root, where /root/reference exists):
    python tests/golden/make_golden.py

It imports echo636/nerf-replication from /root/reference with the minimal stubs the
survey recipe lists: ``ipdb`` (not installed), ``imageio``/``cv2`` for the
dataset module, and host replacements for torch.cuda.Event/synchronize inside
render_accelerated.  Nothing from the reference is copied into the repo: only the
numbers it computes are saved, as small .npz fixtures next to this script.

Weights are the reference's own ``Network()`` right after ``torch.manual_seed(0)``;
the fixture stores the sha256 of the state_dict bytes so the tests can check that the
oracle's ``seeded_network_state(0)`` regenerates them bit for bit.
"""
import hashlib
import os
import sys
import types

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def _import_reference(perturb="0"):
    sys.dont_write_bytecode = True
    for name in ("ipdb", "imageio", "cv2"):
        sys.modules.setdefault(name, types.ModuleType(name))
    tc = types.ModuleType("termcolor")
    tc.colored = lambda s, *a, **k: s
    sys.modules.setdefault("termcolor", tc)
    os.chdir(REF)
    sys.path.insert(0, REF)
    sys.argv = ["make_golden", "--cfg_file", "configs/nerf/lego.yaml", "task_arg.perturb", perturb]
    import torch  # noqa: F401
    from src.config import cfg
    from src.models import make_network
    from src.models.nerf.renderer import make_renderer
    return cfg, make_network, make_renderer


def state_sha256(state):
    h = hashlib.sha256()
    for k, v in state.items():
        h.update(k.encode())
        h.update(v.detach().cpu().contiguous().numpy().tobytes())
    return h.hexdigest()


def main():
    cfg, make_network, make_renderer = _import_reference()
    import torch
    import render_video
    from src.datasets.nerf.blender import Dataset

    torch.manual_seed(0)
    net = make_network(cfg)
    net.eval()
    state = net.state_dict()
    sha = state_sha256(state)
    renderer = make_renderer(cfg, net)
    out = {"state_sha256": np.array(sha)}

    # ---- (a1) rays: lego focal, three spherical poses, 16x16 full view + 1024 pixels of 800x800
    cam_x = 0.6911112070083618
    focal800 = 0.5 * 800 / np.tan(0.5 * cam_x)
    poses = torch.stack([render_video.pose_spherical(a, -30.0, 4.0) for a in (-180.0, -36.0, 72.0)])
    out["poses"] = poses.numpy()
    o16, d16 = Dataset.get_rays(None, 16, 16, 0.5 * 16 / np.tan(0.5 * cam_x), poses[0])
    out["rays16_o"], out["rays16_d"] = o16.numpy(), d16.numpy()
    o8, d8 = Dataset.get_rays(None, 800, 800, focal800, poses[1])
    g = torch.Generator().manual_seed(0)
    pix = torch.randint(0, 800 * 800, (1024,), generator=g)
    out["pix800"] = pix.numpy()
    out["rays800_o"] = o8.reshape(-1, 3)[pix].numpy()
    out["rays800_d"] = d8.reshape(-1, 3)[pix].numpy()
    rays = torch.cat([o8.reshape(-1, 3)[pix], d8.reshape(-1, 3)[pix]], 1)  # [1024, 6]
    out["rays"] = rays.numpy()

    # ---- (a4) positional encoding, 256 points
    g1 = torch.Generator().manual_seed(1)
    x = (torch.rand(256, 3, generator=g1) * 4 - 2).float()
    out["pe_x"] = x.numpy()
    out["pe_xyz"] = net.embed_fn(x).numpy()
    out["pe_dir"] = net.embeddirs_fn(x / torch.norm(x, dim=-1, keepdim=True)).numpy()

    # ---- (a5/a6) MLP: [32 rays, 8 samples] coarse and fine
    pts = (torch.rand(32, 8, 3, generator=g1) * 3 - 1.5).float()
    vd = torch.randn(32, 3, generator=g1)
    vd = vd / torch.norm(vd, dim=-1, keepdim=True)
    out["mlp_pts"], out["mlp_vd"] = pts.numpy(), vd.numpy()
    with torch.no_grad():
        out["mlp_raw_coarse"] = net(pts, vd, "coarse").numpy()
        out["mlp_raw_fine"] = net(pts, vd, "fine").numpy()

    # ---- (a7) raw2outputs: 64 rays x 64 samples, random raw, stratified z
    near, far = torch.tensor([2.0]), torch.tensor([6.0])
    raw = torch.randn(64, 64, 4, generator=g1) * 2.0
    raw[..., 3] = raw[..., 3] * 3.0
    tv = torch.linspace(0.0, 1.0, steps=64)
    z = (near * (1.0 - tv) + far * tv).expand(64, 64).contiguous()
    rd = rays[:64, 3:6]
    with torch.no_grad():
        rgb, dep, acc, w = renderer.raw2outputs(raw, z, rd, 0, True)
    out.update(comp_raw=raw.numpy(), comp_z=z.numpy(), comp_d=rd.numpy(), comp_rgb=rgb.numpy(),
               comp_depth=dep.numpy(), comp_acc=acc.numpy(), comp_w=w.numpy())

    # ---- (a8) sample_pdf det and injected-u (the reference's own function)
    zmid = 0.5 * (z[..., 1:] + z[..., :-1])
    wpdf = w[..., 1:-1]
    calls = {}
    orig_ss = torch.searchsorted

    def spy_ss(cdf, u, right=False):
        r = orig_ss(cdf, u, right=right)
        calls["cdf"], calls["inds"] = cdf.clone(), r.clone()
        return r

    torch.searchsorted = spy_ss
    try:
        s_det = renderer.sample_pdf(zmid, wpdf, 128, det=True)
        out.update(pdf_bins=zmid.numpy(), pdf_w=wpdf.numpy(), pdf_det_samples=s_det.numpy(),
                   pdf_det_cdf=calls["cdf"].numpy(), pdf_det_inds=calls["inds"].numpy())
        u = torch.rand(64, 128, generator=g1)
        orig_rand = torch.rand
        torch.rand = lambda *a, **k: u.clone()
        try:
            s_u = renderer.sample_pdf(zmid, wpdf, 128, det=False)
        finally:
            torch.rand = orig_rand
        out.update(pdf_u=u.numpy(), pdf_u_samples=s_u.numpy(), pdf_u_inds=calls["inds"].numpy())
    finally:
        torch.searchsorted = orig_ss

    # ---- (a3/a9) full render, 64 rays, perturb 0, and perturb 1 with injected uniforms
    batch = {"rays": rays[None, :64].clone(), "near": near, "far": far}
    sorted_z = []
    orig_sort = torch.sort

    def spy_sort(*a, **k):  # the merged fine depths (coarse + importance samples, sorted)
        r = orig_sort(*a, **k)
        sorted_z.append(r[0].clone())
        return r

    torch.sort = spy_sort
    try:
        with torch.no_grad():
            r0 = renderer.render(batch)
    finally:
        torch.sort = orig_sort
    out["render0_z_vals_f"] = sorted_z.pop().numpy()
    for k, v in r0.items():
        out["render0_" + k] = v.numpy()
    t_rand = torch.rand(64, 64, generator=g1)
    u_imp = torch.rand(64, 128, generator=g1)
    seq = [t_rand, u_imp]
    orig_rand = torch.rand

    def fake_rand(*a, **k):
        return seq.pop(0).clone()

    cfg.task_arg.perturb = 1
    torch.rand = fake_rand
    torch.sort = spy_sort
    try:
        with torch.no_grad():
            r1 = renderer.render(batch)
    finally:
        torch.rand = orig_rand
        torch.sort = orig_sort
        cfg.task_arg.perturb = 0
    out["render1_z_vals_f"] = sorted_z.pop().numpy()
    out["render1_t_rand"], out["render1_u"] = t_rand.numpy(), u_imp.numpy()
    for k, v in r1.items():
        out["render1_" + k] = v.numpy()

    # ---- (a10) loss and gradients, 64 rays, perturb 0
    gt = torch.rand(1, 64, 3, generator=g1)
    out["grad_gt"] = gt.numpy()
    net.zero_grad()
    ret = renderer.render(batch)
    lc = torch.nn.functional.mse_loss(ret["rgb_map_c"], gt)
    lf = torch.nn.functional.mse_loss(ret["rgb_map_f"], gt)
    (lc + lf).backward()
    out["grad_loss"] = np.array([float(lc), float(lf)])
    gsel = torch.Generator().manual_seed(7)
    names, norms, sel_idx, sel_val = [], [], [], []
    for name, p in net.named_parameters():
        gflat = p.grad.reshape(-1)
        idx = torch.randint(0, gflat.numel(), (64,), generator=gsel)
        names.append(name)
        norms.append(float(torch.linalg.vector_norm(gflat.double())))
        sel_idx.append(idx.numpy())
        sel_val.append(gflat[idx].numpy())
    out.update(grad_names=np.array(names), grad_norms=np.array(norms),
               grad_sel_idx=np.stack(sel_idx), grad_sel_val=np.stack(sel_val))
    net.zero_grad()

    # ---- (a11) world_to_grid_indices with the real baked grid
    grid = torch.load(os.path.join(REF, "logs/lego/occupancy_grid.pt"), weights_only=True)
    out["grid_sha256"] = np.array(hashlib.sha256(grid.numpy().tobytes()).hexdigest())
    renderer.occupancy_grid = grid
    renderer.grid_resolution = torch.tensor(grid.shape)
    renderer.scene_bbox = torch.tensor(cfg.train_dataset.scene_bbox, dtype=torch.float32)
    gp = (torch.rand(4096, 3, generator=g1) * 4.0 - 2.0).float()  # includes out-of-box points
    gp[:8] = torch.tensor([[-1.5, -1.5, -1.5], [1.5, 1.5, 1.5], [0.0, 0.0, 0.0], [-1.5, 1.5, 0.0],
                           [1.4999999, -1.4999999, 0.0234375], [-2, 2, 0.5], [3, -3, 1], [0.75, -0.75, 1.25]])
    gi = renderer.world_to_grid_indices(gp)
    out.update(grid_pts=gp.numpy(), grid_idx=gi.numpy(), grid_occ=grid[gi[:, 0], gi[:, 1], gi[:, 2]].numpy())

    # ---- (a12) render_accelerated, 256 rays, real grid (seed-0 net, and a dense variant)
    torch.cuda.Event = lambda *a, **k: types.SimpleNamespace(record=lambda: None, elapsed_time=lambda e: 0.0)
    torch.cuda.synchronize = lambda *a, **k: None
    rays256 = rays[256:512].clone()
    out["march_rays"] = rays256.numpy()
    out["march_t_table"] = torch.arange(2.0, 6.0, 0.005).numpy()
    counter = {"n": 0}
    orig_fwd = net.forward

    def counting_forward(inputs, viewdirs, model=""):
        counter["n"] += inputs.shape[0] * inputs.shape[1]
        return orig_fwd(inputs, viewdirs, model)

    net.forward = counting_forward
    try:
        for tag, bias in (("sparse", 0.0), ("dense", 50.0)):
            counter["n"] = 0
            with torch.no_grad():
                net.model_fine.alpha_linear.bias += bias
                r = renderer.render_accelerated({"rays": rays256[None], "near": near, "far": far})
                net.model_fine.alpha_linear.bias -= bias
            for k in ("rgb_map_f", "depth_map_f", "acc_map_f"):
                out[f"march_{tag}_{k}"] = r[k].numpy()
            out[f"march_{tag}_queried"] = np.array(counter["n"])
    finally:
        net.forward = orig_fwd

    # ---- (a13) grid bake through occupancy_grid.main() at resolution 8 (same code path)
    import occupancy_grid as og

    saved = {}

    def fake_save(obj, path):
        saved["grid"] = obj

    og.make_network = lambda c: types.SimpleNamespace(cuda=lambda: bake_net)
    bake_net = net
    bake_net.cuda = lambda: bake_net
    og.load_network = lambda *a, **k: 0
    orig_tensor, orig_zeros, orig_save = torch.tensor, torch.zeros, torch.save
    torch.Tensor.cuda = lambda self, *a, **k: self

    def no_dev(f):
        def g(*a, **k):
            k.pop("device", None)
            return f(*a, **k)
        return g

    torch.tensor, torch.zeros, torch.save = no_dev(orig_tensor), no_dev(orig_zeros), fake_save
    cfg.task_arg.occupancy_grid_res = 8
    sys.modules["tqdm"] = types.SimpleNamespace(tqdm=lambda it, **k: it)
    try:
        with torch.no_grad():
            net.model.alpha_linear.bias += 1.0  # make the threshold bite on a random net
            og.main()
            bias_shift = 1.0
            pts8 = None
            net.model.alpha_linear.bias -= 1.0
    finally:
        torch.tensor, torch.zeros, torch.save = orig_tensor, orig_zeros, orig_save
    out["bake8_grid"] = saved["grid"].numpy()
    out["bake8_alpha_bias_shift"] = np.array(bias_shift)
    del pts8

    np.savez_compressed(os.path.join(OUT, "golden_v1.npz"), **out)
    print("wrote", os.path.join(OUT, "golden_v1.npz"), "sha", sha)


if __name__ == "__main__":
    main()


def dump_lego_grid():
    """The reference's baked lego grid (logs/lego/occupancy_grid.pt, a data artefact) as
    packed bits, loaded with torch.load(weights_only=True)."""
    import hashlib
    import torch
    g = torch.load(os.path.join(REF, "logs/lego/occupancy_grid.pt"), weights_only=True).numpy()
    np.savez_compressed(os.path.join(OUT, "lego_occupancy_grid.npz"), packed=np.packbits(g.reshape(-1)),
                        shape=np.array(g.shape), sha256=np.array(hashlib.sha256(g.tobytes()).hexdigest()))
