"""The wide dX (round 6, DxWave16: PF32W / PBF3W) against the 32x32 one (diagnostic; GPU).

    python tools/dx_compare.py --libs old.so,new.so [--dtype fp32|bf16x3|bf16|bf16x3f] [--M 524288]

One training forward (the first build) gives the masks and activations; each build packs its own W^T layout and runs
its dX on those masks and one d_raw, twice.  Reports: the new dX bit-identical run to run; dZ of the two builds
(fp32 values; bf16x3 hi + lo) -- largest difference relative to each tile's largest value; and the gradients the
first build's dW makes of each dZ -- largest difference relative to each parameter's largest.  Prints one JSON line.
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

ZT_TILES = 78


def dz_values(dz, nblk, fp32):
    """[nblk, 78, 64 lanes, 16 registers] float64 of a dZ store (fp32: 4 chunks of 4; bf16x3: hi chunks 0, 1 + lo 2, 3)."""
    if fp32:
        v = dz.view(torch.float32).view(nblk, ZT_TILES, 4, 64, 4).permute(0, 1, 3, 2, 4).reshape(nblk, ZT_TILES, 64, 16)
        return v.double()
    nch = dz.numel() // (nblk * ZT_TILES * 1024)  # 4 (bf16x3: hi, lo) or 2 (bf16)
    b = dz.view(torch.int16).view(nblk, ZT_TILES, nch, 64, 8)
    f = (b.to(torch.int32) << 16).view(torch.float32).double()  # bf16 -> fp32 exactly
    hi = f[:, :, 0:2].permute(0, 1, 3, 2, 4).reshape(nblk, ZT_TILES, 64, 16)
    if nch == 2:
        return hi
    lo = f[:, :, 2:4].permute(0, 1, 3, 2, 4).reshape(nblk, ZT_TILES, 64, 16)
    return hi + lo


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", required=True)
    ap.add_argument("--M", type=int, default=524288)
    ap.add_argument("--dtype", default="fp32")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    dt = ops.dtype_code(args.dtype)
    M, nblk = args.M, args.M // 32
    torch.manual_seed(0)
    shapes = [(256, 63), (256,)] + [(256, 256), (256,)] * 4 + [(256, 319), (256,)] + [(256, 256), (256,)] * 2 + \
             [(128, 283), (128,), (256, 256), (256,), (1, 256), (1,), (3, 128), (3,)]
    params = [(torch.rand(s, device=dev) - 0.5) * (0.2 if len(s) == 2 else 0.1) for s in shapes]
    arr = ctypes.cast((ctypes.c_void_p * 24)(*[p.data_ptr() for p in params]), ctypes.c_void_p)
    pts = (torch.rand(M, 3, device=dev) - 0.5) * 3
    vd = torch.nn.functional.normalize(torch.randn(M // 192 + 1, 3, device=dev), dim=-1)
    d_raw = torch.randn(M, 4, device=dev) * 1e-3
    s = torch.cuda.current_stream().cuda_stream
    libs = [load_handle(p) for p in args.libs.split(",")]
    A = libs[0]
    pf = torch.empty(A.nerf_mlp_packed_bytes(dt, 0), dtype=torch.uint8, device=dev)
    assert A.nerf_mlp_pack(arr, dt, ptr(pf), None, s) == 0
    raw = torch.zeros(M, 4, device=dev)
    act = torch.zeros(A.nerf_mlp_act_bytes(dt, M), dtype=torch.uint8, device=dev)
    masks = torch.zeros(A.nerf_mlp_mask_bytes(M), dtype=torch.uint8, device=dev)
    assert A.nerf_mlp_fwd(ptr(pf), dt, ptr(pts), ptr(vd), 192, None, M, 1, ptr(raw), ptr(act), ptr(masks), s) == 0
    out = {"M": M, "dtype": args.dtype}
    dzs, grads = [], []
    for k, L in enumerate(libs):
        pb = torch.empty(L.nerf_mlp_packed_bytes(dt, 1), dtype=torch.uint8, device=dev)
        assert L.nerf_mlp_pack(arr, dt, None, ptr(pb), s) == 0
        runs = []
        for _ in range(2):
            dz = torch.zeros(L.nerf_mlp_dz_bytes(dt, M), dtype=torch.uint8, device=dev)
            assert L.nerf_mlp_bwd_dx(ptr(pb), dt, ptr(d_raw), M, ptr(masks), ptr(dz), s) == 0
            runs.append(dz)
        torch.cuda.synchronize()
        out[f"build{k}_dx_bitwise_run_to_run"] = bool(torch.equal(runs[0], runs[1]))
        dzs.append(dz_values(runs[0], nblk, args.dtype == "fp32"))
        g = torch.zeros(A.nerf_mlp_net_params(), device=dev)
        ws = torch.empty(A.nerf_mlp_dw_workspace_bytes(dt, M), dtype=torch.uint8, device=dev)
        assert A.nerf_mlp_bwd_dw_ws(dt, M, ptr(act), ptr(runs[0]), ptr(g), ptr(ws), s) == 0 \
            if hasattr(A, "nerf_mlp_bwd_dw_ws") else A.nerf_mlp_bwd_dw(dt, M, ptr(act), ptr(runs[0]), ptr(g), s) == 0
        torch.cuda.synchronize()
        grads.append(g.double())
    d0, d1 = dzs
    scale = d0.abs().amax(dim=(0, 2, 3)).clamp_min(1e-30)  # per dZ tile
    rel = ((d1 - d0).abs().amax(dim=(0, 2, 3)) / scale)
    out["dz_max_rel_diff_per_tile_max"] = float(rel.max())
    out["dz_tiles_with_rel_diff_over_1e-5"] = [int(t) for t in torch.nonzero(rel > 1e-5).flatten()]
    out["dz_zero_pattern_equal"] = bool(torch.equal(d0 == 0, d1 == 0))
    gr = []
    for i in range(24):
        o0, o1 = int(A.nerf_mlp_param_offset(i)), int(A.nerf_mlp_param_offset(i + 1))
        a0, a1 = grads[0][o0:o1], grads[1][o0:o1]
        gr.append(float((a1 - a0).abs().max() / a0.abs().max().clamp_min(1e-30)))
    out["grad_max_rel_diff_per_param"] = [round(x, 9) for x in gr]
    out["grad_max_rel_diff"] = max(gr)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
