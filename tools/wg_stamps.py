"""Per-workgroup timeline of the training forward from a NERF_DIAG_STAMPS build (diagnostic only).

    python tools/wg_stamps.py --lib ab/stamps.so --dtype bf16x3f [--M 524288]

Each workgroup records its hardware id (CU / SIMD / wave slot, s_getreg HW_ID), XCC id and three
s_memrealtime stamps (100 MHz): entry, prologue done (group 0's weights landed), end.  Prints the
prologue share, the gap between consecutive workgroups on one CU (dispatch + retire), and the
launch's span.
"""
import argparse
import collections
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nerf-replication_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from nerf_amd import _lib, ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", required=True)
    ap.add_argument("--dtype", default="bf16x3f")
    ap.add_argument("--M", type=int, default=524288)
    args = ap.parse_args()
    _lib.LIB_PATH = os.path.abspath(args.lib)
    from nerf_amd._lib import check, lib, ptr
    L = lib()
    dev = torch.device("cuda:0")
    dt = ops.dtype_code(args.dtype)
    torch.manual_seed(0)
    shapes = [(256, 63), (256,)] + [(256, 256), (256,)] * 4 + [(256, 319), (256,)] + [(256, 256), (256,)] * 2 + \
             [(128, 283), (128,), (256, 256), (256,), (1, 256), (1,), (3, 128), (3,)]
    params = [(torch.rand(s, device=dev) - 0.5) * (0.2 if len(s) == 2 else 0.1) for s in shapes]
    import ctypes
    arr = ctypes.cast((ctypes.c_void_p * 24)(*[p.data_ptr() for p in params]), ctypes.c_void_p)
    s = torch.cuda.current_stream().cuda_stream
    M = args.M
    pf = torch.empty(L.nerf_mlp_packed_bytes(dt, 0), dtype=torch.uint8, device=dev)
    check(L.nerf_mlp_pack(arr, dt, ptr(pf), None, s), "pack")
    pts = (torch.rand(M, 3, device=dev) - 0.5) * 3
    vd = torch.nn.functional.normalize(torch.randn(M // 192 + 1, 3, device=dev), dim=-1)
    raw = torch.empty(M, 4, device=dev)
    act = torch.empty(L.nerf_mlp_act_bytes(dt, M), dtype=torch.uint8, device=dev)
    masks = torch.empty(L.nerf_mlp_mask_bytes(M), dtype=torch.uint8, device=dev)
    spb = 128 if args.dtype in ("bf16x3", "bf16x3f", "fp32") else 256
    out = {}
    for rep in range(3):
        check(L.nerf_mlp_fwd(ptr(pf), dt, ptr(pts), ptr(vd), 192, None, M, 1, ptr(raw), ptr(act), ptr(masks), s), "fwd")
        torch.cuda.synchronize()
    w = raw.view(torch.int32).cpu().numpy().reshape(-1, spb * 4)[:, :8].astype(np.int64) & 0xFFFFFFFF
    hw, xcc = w[:, 0], w[:, 1]
    t0, t1, t2 = (w[:, 2] | (w[:, 3] << 32)), (w[:, 4] | (w[:, 5] << 32)), (w[:, 6] | (w[:, 7] << 32))
    cu = (xcc & 0xF) * 1000 + ((hw >> 13) & 0x7) * 100 + ((hw >> 12) & 1) * 16 + ((hw >> 8) & 0xF)  # XCC, SE, SH, CU
    tick_us = 0.01  # s_memrealtime: 100 MHz
    span = (t2.max() - t0.min()) * tick_us
    per = collections.defaultdict(list)
    for i in range(len(cu)):
        per[int(cu[i])].append((int(t0[i]), int(t1[i]), int(t2[i])))
    gaps, lives, pro = [], [], []
    for c, v in per.items():
        v.sort()
        for k, (a0, a1, a2) in enumerate(v):
            lives.append((a2 - a0) * tick_us)
            pro.append((a1 - a0) * tick_us)
            if k + 1 < len(v):
                gaps.append((v[k + 1][0] - a2) * tick_us)
    out = {"dtype": args.dtype, "M": M, "workgroups": int(len(cu)), "cus_seen": len(per), "span_us": round(span, 1),
           "wg_life_us": [round(float(np.percentile(lives, q)), 2) for q in (5, 50, 95)],
           "prologue_us": [round(float(np.percentile(pro, q)), 2) for q in (5, 50, 95)],
           "gap_between_wgs_on_a_cu_us": [round(float(np.percentile(gaps, q)), 2) for q in (5, 50, 95)] if gaps else None,
           "wgs_per_cu": [min(len(v) for v in per.values()), max(len(v) for v in per.values())],
           "first_start_spread_us": round(float((np.sort(t0)[len(per) - 1] - t0.min()) * tick_us), 2),
           "last_end_spread_us": round(float((t2.max() - np.sort(t2)[-len(per)]) * tick_us), 2)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
