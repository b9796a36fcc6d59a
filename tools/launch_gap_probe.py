"""Kernel-to-kernel gap on one stream, eager vs a captured HIP graph (torch.cuda.CUDAGraph on
ROCm), for tiny dependent kernels and for our own ctypes launches.  Diagnostic:
    python tools/launch_gap_probe.py"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nerf-replication_amd"))


def timed(fn, reps):
    torch.cuda.synchronize()
    a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return a.elapsed_time(e) / reps


def main():
    dev = torch.device("cuda:0")
    x = torch.zeros(1024, device=dev)
    N = 200

    def chain():
        for _ in range(N):
            x.add_(1.0)

    out = {}
    chain()
    out["eager_us_per_kernel"] = timed(chain, 5) * 1000 / N
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        chain()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        chain()
    g.replay()
    out["graph_us_per_kernel"] = timed(g.replay, 5) * 1000 / N
    # a host-bound check: the same eager chain with the GPU kept busy first (host far ahead)
    big = torch.empty(256 * 1024 * 1024 // 4, device=dev)

    def busy_then_chain():
        big.mul_(1.0)
        chain()
    out["eager_after_busy_us_per_kernel"] = (timed(busy_then_chain, 5) - timed(lambda: big.mul_(1.0), 5)) * 1000 / N
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
