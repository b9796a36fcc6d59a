"""Run-to-run determinism diagnostic of the MLP training kernels across builds (round 6).

    python tools/race_diag.py --libs a.so,b.so,... [--M 524288] [--runs 3] [--dtype bf16]

For every build: the training forward `runs` times on the same inputs into freshly zeroed buffers, and the
dX `runs` times on the FIRST build's masks (the same input for every build).  Reports, per build:
  * whether raw / act / masks are identical run to run, and raw against the first build;
  * masks against the masks implied by the same run's stored activations (a ReLU bit is set iff the
    stored post-ReLU value is non-zero): mismatching dwords per mask group (layer);
  * which dZ tiles (mlp_tables.h DzTile) differ run to run and against the first build.
Prints one JSON line.  (dtypes bf16, bf16x3, bf16x3f: the mask bits follow the bf16 / hi halves; fp32: the fp32
activations.)
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nerf-replication_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

from nerf_amd import ops  # noqa: E402
from nerf_amd._lib import ptr  # noqa: E402
from mlp_bench import load_handle  # noqa: E402

AT_TILES, AT_H, AT_V, ZT_TILES, MASK_GROUPS = 79, 3, 75, 78, 9


def expected_masks(act, nblk, fp32=False):
    """[nblk, 9, 64, 4] int32 masks implied by act tile-blocks: bf16 [nblk, 79, 2 chunks, 64 lanes, 8] (chunks 0, 1:
    registers 0-7, 8-15; bf16x3 adds its lo chunks 2, 3), fp32 [nblk, 79, 4 chunks, 64 lanes, 4]."""
    if fp32:
        a = act.view(torch.float32).view(nblk, AT_TILES, 4, 64, 4).permute(0, 1, 3, 2, 4).reshape(nblk, AT_TILES, 64, 16)
        a = a.reshape(nblk, AT_TILES, 64, 2, 8).permute(0, 1, 3, 2, 4)  # -> [b, tau, chunk-of-8, lane, 8] as bf16's
    else:
        nch = act.numel() // (nblk * AT_TILES * 1024)  # 2 (bf16 / bf16x3f) or 4 (bf16x3: hi, lo)
        a = act.view(torch.int16).view(nblk, AT_TILES, nch, 64, 8)[:, :, :2]
    out = torch.zeros(nblk, MASK_GROUPS, 64, 4, dtype=torch.int64, device=act.device)
    rho = torch.arange(16, device=act.device)
    bitpos = (rho >> 1) + 16 * (rho & 1)
    for grp in range(MASK_GROUPS):
        ntile = 8 if grp < 8 else 4
        for n in range(ntile):
            tau = AT_H + 8 * grp + n if grp < 8 else AT_V + n
            nz = (a[:, tau] != 0).permute(0, 2, 1, 3).reshape(nblk, 64, 16).to(torch.int64)  # [b, lane, rho]
            bits = (nz << (bitpos + 8 * (n & 1))).sum(-1)
            out[:, grp, :, n >> 1] |= bits
    return out.to(torch.int64) & 0xFFFFFFFF


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", required=True)
    ap.add_argument("--M", type=int, default=524288)
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--dtype", default="bf16")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    dt = ops.dtype_code(args.dtype)
    M = args.M
    nblk = M // 32
    torch.manual_seed(0)
    shapes = [(256, 63), (256,)] + [(256, 256), (256,)] * 4 + [(256, 319), (256,)] + [(256, 256), (256,)] * 2 + \
             [(128, 283), (128,), (256, 256), (256,), (1, 256), (1,), (3, 128), (3,)]
    params = [(torch.rand(s, device=dev) - 0.5) * (0.2 if len(s) == 2 else 0.1) for s in shapes]
    arr = ctypes.cast((ctypes.c_void_p * 24)(*[p.data_ptr() for p in params]), ctypes.c_void_p)
    pts = (torch.rand(M, 3, device=dev) - 0.5) * 3
    vd = torch.nn.functional.normalize(torch.randn(M // 192 + 1, 3, device=dev), dim=-1)
    d_raw = torch.randn(M, 4, device=dev) * 1e-3
    s = torch.cuda.current_stream().cuda_stream
    out = {"M": M, "dtype": args.dtype, "runs": args.runs, "builds": {}}
    ref = None
    for path in args.libs.split(","):
        name = os.path.basename(path).replace(".so", "")
        L = load_handle(path)
        pf = torch.empty(L.nerf_mlp_packed_bytes(dt, 0), dtype=torch.uint8, device=dev)
        pb = torch.empty(L.nerf_mlp_packed_bytes(dt, 1), dtype=torch.uint8, device=dev)
        assert L.nerf_mlp_pack(arr, dt, ptr(pf), ptr(pb), s) == 0
        fw = []
        for _ in range(args.runs):
            raw = torch.zeros(M, 4, device=dev)
            act = torch.zeros(L.nerf_mlp_act_bytes(dt, M), dtype=torch.uint8, device=dev)
            masks = torch.zeros(L.nerf_mlp_mask_bytes(M), dtype=torch.uint8, device=dev)
            assert L.nerf_mlp_fwd(ptr(pf), dt, ptr(pts), ptr(vd), 192, None, M, 1, ptr(raw), ptr(act), ptr(masks),
                                  s) == 0
            torch.cuda.synchronize()
            fw.append((raw, act, masks))
        if ref is None:
            ref = {"raw": fw[0][0], "masks": fw[0][2], "act": fw[0][1]}
        rec = {"raw_same_runs": all(torch.equal(f[0], fw[0][0]) for f in fw),
               "act_same_runs": all(torch.equal(f[1], fw[0][1]) for f in fw),
               "masks_same_runs": all(torch.equal(f[2], fw[0][2]) for f in fw),
               "raw_equal_first_build": bool(torch.equal(fw[0][0], ref["raw"])),
               "raw_max_abs_diff_first_build": float((fw[0][0] - ref["raw"]).abs().max()),
               "raw_max_rel_diff_first_build": float(((fw[0][0] - ref["raw"]).abs() /
                                                      ref["raw"].abs().clamp_min(1e-3)).max()),
               "act_bf16_differing_first_build": float((fw[0][1].view(torch.int16) != ref["act"].view(torch.int16))
                                                       .float().mean()) if fw[0][1].numel() == ref["act"].numel()
               else None,
               "mask_bits_differing_first_build": float(
                   (fw[0][2].view(torch.uint8) ^ ref["masks"].view(torch.uint8)).to(torch.int32).bitwise_and(255)
                   .ne(0).float().mean())}
        mism = []
        for raw, act, masks in fw:
            exp = expected_masks(act, nblk, fp32=args.dtype == "fp32")
            got = masks.view(torch.int32).view(nblk, MASK_GROUPS, 64, 4).to(torch.int64) & 0xFFFFFFFF
            bad = (exp != got)
            mism.append([int(bad[:, g].sum()) for g in range(MASK_GROUPS)])
        rec["mask_dwords_not_implied_by_act_per_group"] = mism
        dzs = []
        for _ in range(args.runs):
            dz = torch.zeros(L.nerf_mlp_dz_bytes(dt, M), dtype=torch.uint8, device=dev)
            assert L.nerf_mlp_bwd_dx(ptr(pb), dt, ptr(d_raw), M, ptr(ref["masks"]), ptr(dz), s) == 0
            torch.cuda.synchronize()
            dzs.append(dz.view(nblk, ZT_TILES, -1))
        if "dz" not in ref:
            ref["dz"] = dzs[0]
        rec["dz_tiles_differing_runs"] = sorted({t for d in dzs[1:] for t in range(ZT_TILES)
                                                 if not torch.equal(d[:, t], dzs[0][:, t])})
        rec["dz_tiles_differing_first_build"] = [t for t in range(ZT_TILES) if not torch.equal(dzs[0][:, t],
                                                                                             ref["dz"][:, t])]
        out["builds"][name] = rec
        print(name, json.dumps(rec), file=sys.stderr, flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
