"""Config-3-style training curve on the GPU (BASELINE.json config 3: 4096 rays/step, held-out PSNR
along the way), for each MLP precision from the same seed and the same ray stream: the procedural
scene of tests/test_gpu_training.py (100 training views, 100x100; 4 held-out views), the
production step (Trainer.train_step: render perturb 1, MSE(c)+MSE(f), backward, fused clip 40 +
Adam) and the reference's ExponentialLR (lr 5e-4 x 0.1^(epoch/500), stepped every 500 steps,
train.py:43-46).  Prints a progress line per evaluation and writes gpurun_out/psnr_curve.json.

    python tools/psnr_curve.py [--steps 15000] [--every 1000] [--dtypes fp32,bf16x3,bf16]

A run longer than one GPU call (config 3's 200k steps: 94 min at fp32) continues across calls:
--ckpt-out DIR saves <dtype>.pt (weights, the reference-format Adam state, scheduler, the ray
stream's and the renderer's Philox counters, the curve so far) at every evaluation and when
--max-seconds of wall time are used up; --ckpt-in DIR resumes from it (same ray stream, same
schedule).
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
    ap.add_argument("--steps", type=int, default=15000)
    ap.add_argument("--every", type=int, default=1000)
    ap.add_argument("--epoch_steps", type=int, default=500)
    ap.add_argument("--dtypes", default="fp32,bf16x3,bf16")
    ap.add_argument("--ckpt-in", default=None)
    ap.add_argument("--ckpt-out", default=None)
    ap.add_argument("--max-seconds", type=float, default=0.0)
    ap.add_argument("--seed", type=int, default=0, help="torch seed: initial weights and the ray / sample streams")
    args = ap.parse_args()
    t_start = time.time()
    dev = torch.device("cuda:0")
    from nerf_amd import ops
    from src.config import cfg
    from src.datasets.nerf.blender import Dataset
    from src.datasets.nerf.synthetic import camera_rays, make_scene, psnr, shade, view_poses
    from src.models import make_network
    from src.models.nerf.renderer.volume_renderer import Renderer
    from src.train.optimizer import make_optimizer
    from src.train.scheduler import ExponentialLR
    from src.train.trainers.make_trainer import make_trainer
    from src.utils.camera import focal_for
    imgs, poses, focal = make_scene(100, 100, 100, dev, seed=0)
    ev = view_poses(4, seed=1).to(dev)
    gts, evrays = [], []
    for k in range(ev.shape[0]):
        o, d = camera_rays(ev[k], 100, 100, focal_for(100))
        gts.append(shade(o, d))
        evrays.append(torch.cat([o, d], -1))

    def heldout(net):
        cfg.task_arg.perturb = 0
        net.eval()
        r = Renderer(net)
        ps = []
        with torch.no_grad():
            for rr, gt in zip(evrays, gts):
                out = r.render({"rays": rr, "near": torch.tensor([2.0], device=dev),
                                "far": torch.tensor([6.0], device=dev)})
                ps.append(psnr(out["rgb_map_f"], gt))
        net.train()
        cfg.task_arg.perturb = 1
        return float(np.mean(ps))

    out = {"seed": args.seed, "steps": args.steps, "every": args.every, "rays_per_step": int(cfg.task_arg.train_rays),
           "epoch_steps": args.epoch_steps, "lr": "5e-4 x 0.1^(epoch/500)", "heldout_views": 4, "res": 100,
           "scene": "procedural (src/datasets/nerf/synthetic.py make_scene seed 0), 100 views 100x100"}
    for dtype in args.dtypes.split(","):
        cfg.task_arg.mlp_dtype = dtype
        cfg.task_arg.perturb = 1
        torch.manual_seed(args.seed)
        net = make_network(cfg)
        trainer = make_trainer(cfg, net)
        opt = make_optimizer(cfg, net)
        sched = ExponentialLR(opt, decay_epochs=500, gamma=0.1)
        ds = Dataset.from_arrays(imgs, poses, focal)
        curve, t_train, first = [], 0.0, 1
        renderer = trainer.network.renderer
        src = os.path.join(args.ckpt_in, f"{dtype}.pt") if args.ckpt_in else None
        if src and os.path.exists(src):
            ck = torch.load(src, map_location="cpu", weights_only=True)
            net.load_state_dict(ck["net"], strict=True)
            opt.load_state_dict(ck["optim"])
            sched.load_state_dict(ck["sched"])
            ds.draws, renderer._calls = int(ck["draws"]), int(ck["calls"])
            curve, t_train, first = [tuple(x) for x in ck["curve"].tolist()], float(ck["t_train"]), int(ck["step"]) + 1
            ops.params_updated()
            print(json.dumps({"dtype": dtype, "resumed_at": first - 1}), flush=True)

        def save(step):
            if not args.ckpt_out:
                return
            os.makedirs(args.ckpt_out, exist_ok=True)
            tmp = os.path.join(args.ckpt_out, f"{dtype}.pt.tmp")
            torch.save({"net": {k: v.detach().cpu() for k, v in net.state_dict().items()}, "optim": opt.state_dict(),
                        "sched": sched.state_dict(), "draws": ds.draws, "calls": renderer._calls, "step": step,
                        "curve": torch.tensor(curve, dtype=torch.float64).reshape(-1, 2), "t_train": t_train}, tmp)
            os.replace(tmp, os.path.join(args.ckpt_out, f"{dtype}.pt"))
        stopped = False
        for step in range(first, args.steps + 1):
            if args.max_seconds and time.time() - t_start > args.max_seconds:
                save(step - 1)
                print(json.dumps({"dtype": dtype, "paused_at": step - 1}), flush=True)
                stopped = True
                break
            rays, rgbs = ds.sample_batch()
            t0 = time.perf_counter()
            trainer.train_step({"rays": rays[None], "rgbs": rgbs[None], "near": ops.device_scalar(2.0, dev),
                                "far": ops.device_scalar(6.0, dev)}, opt)
            if step % args.epoch_steps == 0:
                sched.step()
            if step % args.every == 0:
                torch.cuda.synchronize()
                t_train += time.perf_counter() - t0
                p = heldout(net)
                curve.append((step, round(p, 3)))
                print(json.dumps({"dtype": dtype, "step": step, "psnr": round(p, 3)}), flush=True)
                save(step)
            else:
                t_train += time.perf_counter() - t0
        if stopped:
            break
        out[f"psnr_curve_{dtype}"] = [[int(a), float(b)] for a, b in curve]
        out[f"train_s_{dtype}"] = round(t_train, 1)
        del net, trainer, opt, ds
        torch.cuda.empty_cache()
    dts = [d for d in args.dtypes.split(",") if f"psnr_curve_{d}" in out]
    if "fp32" in dts:
        for dt in dts:
            if dt == "fp32":
                continue
            a, b = out["psnr_curve_fp32"], out[f"psnr_curve_{dt}"]
            out[f"delta_db_{dt}"] = [round(y[1] - x[1], 3) for x, y in zip(a, b)]
            out[f"mean_delta_db_{dt}"] = round(float(np.mean([y[1] - x[1] for x, y in zip(a, b)])), 3)
            tail = max(1, len(a) // 3)
            out[f"mean_delta_db_last_third_{dt}"] = round(float(np.mean([y[1] - x[1] for x, y in
                                                                         zip(a[-tail:], b[-tail:])])), 3)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(args.ckpt_out or os.path.join(ROOT, "gpurun_out"),
                           "psnr_curve_" + "_".join(dts) + ".json" if args.ckpt_out else "psnr_curve.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
