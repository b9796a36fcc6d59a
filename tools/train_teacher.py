"""Train the NeRF on the procedural scene (src/datasets/nerf/synthetic.py) with this build's
training step (Trainer + FusedAdam, fp32 MLP by default) and save the weights.

The weights are INPUT DATA for the trained-net parity fixtures: tests/golden/make_golden.py
loads them into the REFERENCE Network (CPU, this container) and records its outputs, and
the GPU tests render the same weights through the kernels.  A trained net has the sharp,
surface-like density of a real scene, so its coarse CDF is well conditioned (the seed-0
net's is noise-level) and its march terminates early.

    gpurun -- python tools/train_teacher.py --steps 3000 --out gpurun_out/trained_v2.npz
"""
import argparse
import json
import os
import sys
import time

os.environ.setdefault("NERF_AMD_NO_ARGV", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "nerf-replication_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3000)
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--res", type=int, default=200)
    ap.add_argument("--views", type=int, default=100)
    ap.add_argument("--rays", type=int, default=4096)
    ap.add_argument("--eval-res", type=int, default=100)
    ap.add_argument("--out", default="gpurun_out/trained_v2.npz")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    from nerf_amd import ops
    from src.config import cfg
    from src.datasets.nerf.blender import Dataset
    from src.datasets.nerf.synthetic import camera_rays, make_scene, psnr, shade, view_poses
    from src.models import make_network
    from src.models.nerf.renderer.volume_renderer import Renderer
    from src.train.optimizer import make_optimizer
    from src.train.trainers.make_trainer import make_trainer
    from src.utils.camera import focal_for

    cfg.task_arg.mlp_dtype = args.dtype
    cfg.task_arg.train_rays = args.rays
    cfg.task_arg.perturb = 1
    imgs, poses, focal = make_scene(args.views, args.res, args.res, dev, seed=0)
    ds = Dataset.from_arrays(imgs, poses, focal)
    torch.manual_seed(0)
    net = make_network(cfg)
    trainer = make_trainer(cfg, net)
    opt = make_optimizer(cfg, net)
    # held-out views (seed 1 poses), rendered at eval_res with perturb 0
    ev_poses = view_poses(2, seed=1).to(dev)
    f_ev = focal_for(args.eval_res)

    def evaluate():
        r = Renderer(net)
        cfg.task_arg.perturb = 0
        net.eval()
        out = []
        with torch.no_grad():
            for k in range(ev_poses.shape[0]):
                o, d = camera_rays(ev_poses[k], args.eval_res, args.eval_res, f_ev)
                gt = shade(o, d)
                rays = torch.cat([o, d], -1)
                ret = r.render({"rays": rays, "near": torch.tensor([2.0], device=dev),
                                "far": torch.tensor([6.0], device=dev)})
                out.append(psnr(ret["rgb_map_f"], gt))
        net.train()
        cfg.task_arg.perturb = 1
        return out

    log = []
    t0 = time.time()
    for step in range(1, args.steps + 1):
        rays, rgbs = ds.sample_batch()
        batch = {"rays": rays[None], "rgbs": rgbs[None], "near": ops.device_scalar(2.0, dev),
                 "far": ops.device_scalar(6.0, dev)}
        _, loss, _ = trainer.train_step(batch, opt)
        if step % 500 == 0 or step == args.steps:
            p = evaluate()
            log.append({"step": step, "loss": float(loss), "psnr_heldout": p, "s": round(time.time() - t0, 1)})
            print(json.dumps(log[-1]), flush=True)
    sd = {k: v.detach().cpu().numpy() for k, v in net.state_dict().items()}
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    np.savez_compressed(args.out, **sd)
    with open(os.path.splitext(args.out)[0] + "_log.json", "w") as f:
        json.dump({"args": vars(args), "log": log}, f, indent=1)
    print("saved", args.out)


if __name__ == "__main__":
    main()
