"""Grid-march schedule sweep on the trained fixture net (tests/golden/trained_v2.npz): its own
res-128 bake, an 800x800 held-out view, render_accelerated's kernels (ops.march) with several
K schedules; prints one JSON line per schedule (s/frame, queried = composited points,
evaluated = MLP points, rounds).

    python tools/march_bench.py [--dtype fp32]
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

SCHEDULES = {
    "16x2": (16, 32, 64, 128, 256, 512, 1024),
    "8x2": (8, 16, 32, 64, 128, 256, 512, 1024),
    "4x2": (4, 8, 16, 32, 64, 128, 256, 512, 1024),
    "8x4": (8, 32, 128, 512, 1024),
    "12x2": (12, 24, 48, 96, 192, 384, 768),
    "6x2": (6, 12, 24, 48, 96, 192, 384, 768),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--lib", default=None, help="alternative build of libnerf_amd.so")
    ap.add_argument("--schedule", default=None, help="time only these schedules (comma-separated names)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    from nerf_amd import _lib
    if args.lib:
        _lib.LIB_PATH = os.path.abspath(args.lib)
    from nerf_amd import ops
    from src.config import cfg
    from src.datasets.nerf.synthetic import view_poses
    from src.models import make_network
    from src.utils.camera import focal_for
    z = np.load(os.path.join(ROOT, "tests", "golden", "trained_v2.npz"), allow_pickle=False)
    torch.manual_seed(0)
    net = make_network(cfg)
    net.load_state_dict({k: torch.from_numpy(z[k]) for k in z.files}, strict=True)
    net = net.to(dev).eval()
    with torch.no_grad():
        grid = ops.bake(net.model.packer(), 128, 1.0, dtype=args.dtype)
        pose = view_poses(2, seed=1)[0].to(dev)
        rays, _, _ = ops.raygen(pose.reshape(1, 4, 4), 800, 800, focal_for(800), pix=torch.arange(640000, device=dev))
        ref = None
        variants = [(n, sc, 1024, 2.0) for n, sc in SCHEDULES.items()]  # t_split 2: k_low never used
        variants += [(f"{n}_klow{kl}_t{tsp}", SCHEDULES[n], kl, tsp) for n in ("12x2", "16x2")
                     for kl in (2, 4, 8, 16) for tsp in (0.5, 0.7, 0.9)]
        variants = [(n + (f"_sync{se}" if se != 4 else ""), sc, kl, tsp, se) for n, sc, kl, tsp in variants
                    for se in (4, 8)]
        # _2pass: gather + emit walking twice (round 2); _g<r>: k_low doubling from round r on
        variants = [(n + sfx, sc, kl, tsp, se, op, gr) for n, sc, kl, tsp, se in variants
                    for sfx, op, gr in (("", True, 0), ("_2pass", False, 0), ("_g4", True, 4), ("_g6", True, 6),
                                        ("_g8", True, 8), ("_g10", True, 10))]
        for name, sched, kl, tsp, se, op, gr in variants:
            if args.schedule and name not in args.schedule.split(","):
                continue
            run = lambda: ops.march(net.model_fine.packer(), rays, 2.0, 6.0, grid, dtype=args.dtype,  # noqa: E731
                                    k_schedule=sched, k_low=kl, t_split=tsp, sync_every=se, one_pass=op,
                                    k_low_grow=gr)
            run()
            torch.cuda.synchronize()
            ts = []
            for _ in range(args.reps):
                t0 = time.perf_counter()
                o = run()
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            if ref is None:
                ref = o
            same = all(torch.equal(o[k], ref[k]) for k in ("rgb_map_f", "depth_map_f", "acc_map_f"))
            print(json.dumps({"schedule": name, "s": round(min(ts), 4), "queried": o["n_queried"],
                              "evaluated": o["n_evaluated"], "rounds": o["rounds"], "identical_outputs": same}),
                  flush=True)


if __name__ == "__main__":
    main()
