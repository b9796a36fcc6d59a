"""HBM rates of plain streaming kernels on this GPU, for the store floors of DESIGN.md 8:
write-only (torch fill_), read-only (torch sum), copy (clone), 2 GiB buffers, median of 10.

    python tools/hbm_rates.py
"""
import json
import statistics

import torch


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e-3)
    return statistics.median(ts)


def main():
    n = (2 << 30) // 4
    x = torch.empty(n, device="cuda", dtype=torch.float32)
    y = torch.empty_like(x)
    x.uniform_()
    nbytes = n * 4
    out = {"bytes": nbytes}
    t = timed(lambda: y.fill_(1.0))
    out["write_TBps"] = round(nbytes / t / 1e12, 3)
    t = timed(lambda: x.sum())
    out["read_TBps"] = round(nbytes / t / 1e12, 3)
    t = timed(lambda: y.copy_(x))
    out["copy_TBps_read_plus_write"] = round(2 * nbytes / t / 1e12, 3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
