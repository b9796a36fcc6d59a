"""Full-size golden vectors (v4) for BASELINE configs 2 and 4 on the trained net, generated
by running the REFERENCE on the CPU (build container only; takes ~10-20 minutes).

    python tests/golden/make_golden_v4.py [tests/golden/trained_v2.npz]

The reference Network loaded with the trained fixture weights (tests/golden/trained_v2.npz,
input data) renders the WHOLE 800x800 held-out view of golden_v2 (pose
view_poses(2, seed=1)[0], lego focal; blender.get_rays) twice, perturb 0:

  * ``render()`` -- the hierarchical 64 + 128 path (volume_renderer.py:137-247), config 2;
  * ``render_accelerated()`` -- the grid march (volume_renderer.py:268-357), config 4, on the
    reference's own res-128 bake of the same weights (golden_v2 ``bake128_packed``, made by
    occupancy_grid.main()), with the exact count of MLP-queried points over the frame.

A 640,000-ray fp32 frame is 12.8 MB per mode, so only numbers that pin it are saved:
  * every key of 4,096 rays (3,072 uniform over the frame + 1,024 over the central 400x400
    crop that the object covers) -- rays are independent, so a subset of the frame's rays,
    rendered as part of the frame, must equal these;
  * the float64 sum of every key per image row (800 rows);
  * the evaluator's uint8 frame (clip(rgb) * 255 truncated, evaluators/nerf.py:49-56);
  * the march's query count over the whole frame.
Only numbers are saved; the ATen CPU capability that produced them is recorded.
"""
import os
import sys
import time
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import _import_reference, state_sha256  # noqa: E402
from make_golden_v2 import CAM_X, held_out_pose  # noqa: E402

H = W = 800
N_UNIFORM, N_CENTRAL = 3072, 1024


def row_sums(v: np.ndarray) -> np.ndarray:
    """float64 sum over each image row: [H] or [H, c]."""
    r = v.astype(np.float64).reshape(H, W, -1).sum(1)
    return r[:, 0] if r.shape[1] == 1 else r


def main(weights_path):
    weights_path = os.path.abspath(weights_path)
    cfg, make_network, make_renderer = _import_reference()
    import torch
    import render_video
    from src.datasets.nerf.blender import Dataset

    torch.set_num_threads(os.cpu_count() or 1)
    z = np.load(weights_path, allow_pickle=False)
    torch.manual_seed(0)
    net = make_network(cfg)
    net.load_state_dict({k: torch.from_numpy(z[k]) for k in z.files}, strict=True)
    net.eval()
    renderer = make_renderer(cfg, net)
    v2 = np.load(os.path.join(HERE, "golden_v2.npz"), allow_pickle=False)
    out = {"state_sha256": np.array(state_sha256(net.state_dict())),
           "cpu_capability": np.array(torch.backends.cpu.get_cpu_capability()),
           "torch_version": np.array(torch.__version__)}
    assert str(out["state_sha256"]) == str(v2["state_sha256"])
    near, far = torch.tensor([2.0]), torch.tensor([6.0])

    pose = held_out_pose(render_video.pose_spherical)
    assert np.array_equal(pose.numpy(), v2["pose"])
    focal = 0.5 * 800 / np.tan(0.5 * CAM_X)
    o8, d8 = Dataset.get_rays(None, H, W, focal, pose)
    rays = torch.cat([o8.reshape(-1, 3), d8.reshape(-1, 3)], 1)  # [640000, 6], pixel j*W + i
    g = torch.Generator().manual_seed(4)
    pix_u = torch.randperm(H * W, generator=g)[:N_UNIFORM]
    ij = torch.randint(0, 400, (N_CENTRAL, 2), generator=g) + 200
    pix = torch.cat([pix_u, ij[:, 0] * W + ij[:, 1]])
    out.update(pose=pose.numpy(), focal=np.array(focal), pix=pix.numpy(), rays=rays[pix].numpy())

    # ---- config 2: hierarchical render of the whole frame (perturb 0); the full outputs are
    # cached outside the repo (a rerun after a later failure skips the ~20 minutes)
    cfg.task_arg.perturb = 0
    cache = os.environ.get("GOLDEN_V4_CACHE", "/tmp/golden_v4_render_cache.npz")
    if os.path.exists(cache):
        c = np.load(cache, allow_pickle=False)
        r = {k: torch.from_numpy(c[k]) for k in c.files if k != "seconds"}
        out["render_seconds_cpu"] = c["seconds"]
    else:
        t0 = time.time()
        with torch.no_grad():
            r = renderer.render({"rays": rays[None], "near": near, "far": far})
        out["render_seconds_cpu"] = np.array(time.time() - t0)
        np.savez(cache, seconds=out["render_seconds_cpu"], **{k: v.numpy() for k, v in r.items()})
    print(f"render: {float(out['render_seconds_cpu']):.1f} s", flush=True)
    for k, v in r.items():
        v = v.numpy()
        out[f"render_{k}"] = v[pix.numpy()]
        out[f"render_rowsum_{k}"] = row_sums(v)
    out["render_frame_u8"] = (np.clip(r["rgb_map_f"].numpy().reshape(H, W, 3), 0, 1) * 255).astype(np.uint8)

    # ---- config 4: render_accelerated of the whole frame on the reference's res-128 bake
    res = 128
    grid = torch.from_numpy(np.unpackbits(v2["bake128_packed"])[: res ** 3].reshape(res, res, res).astype(bool))
    torch.cuda.Event = lambda *a, **k: types.SimpleNamespace(record=lambda: None, elapsed_time=lambda e: 0.0)
    torch.cuda.synchronize = lambda *a, **k: None
    renderer.occupancy_grid = grid
    renderer.grid_resolution = torch.tensor(grid.shape)
    renderer.scene_bbox = torch.tensor(cfg.train_dataset.scene_bbox, dtype=torch.float32)
    out["march_t_table"] = torch.arange(2.0, 6.0, 0.005).numpy()
    counter = {"n": 0}
    orig_fwd = net.forward

    def counting_forward(inputs, viewdirs, model=""):
        counter["n"] += inputs.shape[0] * inputs.shape[1]
        return orig_fwd(inputs, viewdirs, model)

    net.forward = counting_forward
    t0 = time.time()
    try:
        with torch.no_grad():
            m = renderer.render_accelerated({"rays": rays[None], "near": near, "far": far})
    finally:
        net.forward = orig_fwd
    out["march_seconds_cpu"] = np.array(time.time() - t0)
    print(f"march: {time.time() - t0:.1f} s, queried {counter['n']}", flush=True)
    for k in ("rgb_map_f", "depth_map_f", "acc_map_f"):
        v = m[k].numpy()
        out[f"march_{k}"] = v[pix.numpy()]
        out[f"march_rowsum_{k}"] = row_sums(v)
    out["march_frame_u8"] = (np.clip(m["rgb_map_f"].numpy().reshape(H, W, 3), 0, 1) * 255).astype(np.uint8)
    out["march_queried"] = np.array(counter["n"])

    dst = os.path.join(HERE, "golden_v4.npz")
    np.savez_compressed(dst, **out)
    print("wrote", dst, "queried", counter["n"], "capability", out["cpu_capability"])


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(HERE, "trained_v2.npz"))
