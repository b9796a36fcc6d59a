"""A/B of the whole training step (bench.py's step: 4096 rays, 64 + 128 samples, fwd + bwd +
clip + Adam) under backward-scheduling knobs that ops reads at call time, in interleaved
rounds in one process (cross-process and DVFS drift otherwise look like differences).

    python tools/step_ab.py --dtype bf16x3f [--rounds 5] [--steps 20]

Configurations (ops.BWD_CHUNK x ops.DW_STREAM):
  one      every backward one dX + one dW launch, one stream
  chunk    the backward in 262,144-sample chunks (dX, dW per chunk)
  stream   one launch each, dW on the dW stream (the next dX -- the coarse net's -- overlaps it)
  chunk+stream
  unfused  one, with the round-4 fused launches split again (composite + sample_pdf, the MSE pair)
  events   one, with bench.py's per-kernel HIP timing events recorded (ops.KERNEL_TIMES)
  noplan   one, with the weight repack walking the units on the device (NERF_PACK_PLAN=0) instead of
           gathering through the cached pack plan
Prints one JSON line: median ms/step per configuration.
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "nerf-replication_amd"))
os.environ.setdefault("NERF_AMD_NO_ARGV", "1")

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16x3f")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--chunk", type=int, default=262144)
    ap.add_argument("--configs", default="one,chunk,stream,chunk+stream")
    a = ap.parse_args()
    from nerf_amd import ops
    dev = torch.device("cuda:0")
    args = bench.parse(["--dtype", a.dtype])
    cfg, net, trainer, opt, ds = bench.build(args, dev, a.dtype)
    code = ops.pack_code(ops.dtype_code(a.dtype), 1)
    configs = a.configs.split(",")

    def setup(c):
        ops.BWD_CHUNK = {code: a.chunk} if "chunk" in c else {}
        ops.DW_STREAM = "stream" in c
        # "unfused": coarse composite + sample_pdf as two launches, MSE(c) + MSE(f) through torch
        cfg.task_arg.fuse_composite_pdf = cfg.task_arg.fuse_mse = "unfused" not in c
        # "events": bench.py's per-launch HIP timing events (ops.kernel_timer) recorded around every kernel
        ops.KERNEL_TIMES.reset()
        ops.KERNEL_TIMES.enabled = "events" in c
        os.environ["NERF_PACK_PLAN"] = "0" if "noplan" in c else "1"

    times = {c: [] for c in configs}
    for r in range(a.rounds + 1):
        for c in configs:
            setup(c)
            for _ in range(3):
                bench.train_step(cfg, trainer, opt, ds, dev)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                bench.train_step(cfg, trainer, opt, ds, dev)
            torch.cuda.synchronize()
            if r:
                times[c].append((time.perf_counter() - t0) / a.steps * 1e3)
        print(f"round {r}: " + ", ".join(f"{c} {times[c][-1]:.3f}" for c in configs if times[c]), flush=True)
    print(json.dumps({"dtype": a.dtype, "steps": a.steps, "rounds": a.rounds, "chunk": a.chunk,
                      "ms_per_step_median": {c: round(statistics.median(v), 4) for c, v in times.items()},
                      "ms_per_step_all": {c: [round(x, 3) for x in v] for c, v in times.items()}}), flush=True)


if __name__ == "__main__":
    main()
