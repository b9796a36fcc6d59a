"""Microbenchmark of the MLP kernels alone (no renderer), for kernel iteration.

    python tools/mlp_bench.py [--M 786432] [--reps 10] [--dtype bf16]

Times nerf_mlp_fwd (inference and training store), nerf_mlp_bwd_dx, nerf_mlp_bwd_dw and
nerf_mlp_pack with HIP events on the launching stream and prints one JSON line with
ms and TFLOP/s per kernel (algorithmic FLOP).
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nerf-replication_amd"))

import torch  # noqa: E402

from nerf_amd import _lib, ops  # noqa: E402
from nerf_amd._lib import check, lib, ptr, stream_of  # noqa: E402

FLOP = {"fwd": 2 * 593408, "fwd_train": 2 * 593408, "dx": 2 * 557696, "dw": 2 * 593408, "density": 2 * 491264}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=786432)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--lib", default=None, help="alternative build of libnerf_amd.so (kernel experiments)")
    ap.add_argument("--libs", default=None, help="comma-separated builds, timed in interleaved rounds in this process")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--chunks", default=None,
                    help="comma-separated sample counts: time the backward (dX then dW) run per chunk of that many "
                         "samples, so dW reads each chunk's dZ soon after dX wrote it (Infinity Cache, 256 MiB), "
                         "against the one-launch backward")
    ap.add_argument("--overlap", type=int, default=0,
                    help="with --chunks: the training step's backward (the M-sample fine net in chunks, then an "
                         "N-sample coarse net) with every dW on a second stream, so that the next dX overlaps it; "
                         "N = this value")
    args = ap.parse_args()
    if args.lib:
        _lib.LIB_PATH = os.path.abspath(args.lib)
    if args.libs:
        return compare(args)
    dev = torch.device("cuda:0")
    dt = ops.dtype_code(args.dtype)
    torch.manual_seed(0)
    shapes = [(256, 63), (256,)] + [(256, 256), (256,)] * 4 + [(256, 319), (256,)] + [(256, 256), (256,)] * 2 + \
             [(128, 283), (128,), (256, 256), (256,), (1, 256), (1,), (3, 128), (3,)]
    params = [(torch.rand(s, device=dev) - 0.5) * (0.2 if len(s) == 2 else 0.1) for s in shapes]
    packer = ops.PackedMLP(params)
    L = lib()
    M = args.M
    pts = (torch.rand(M, 3, device=dev) - 0.5) * 3
    vd = torch.nn.functional.normalize(torch.randn(M // 192 + 1, 3, device=dev), dim=-1)
    raw = torch.empty(M, 4, device=dev)
    act = torch.empty(L.nerf_mlp_act_bytes(dt, M), dtype=torch.uint8, device=dev)
    masks = torch.empty(L.nerf_mlp_mask_bytes(M), dtype=torch.uint8, device=dev)
    dz = torch.empty(L.nerf_mlp_dz_bytes(dt, M), dtype=torch.uint8, device=dev)
    grad = torch.zeros(L.nerf_mlp_net_params(), device=dev)
    d_raw = torch.randn(M, 4, device=dev) * 1e-3
    pf, pb = packer.get(dt, 0), packer.get(dt, 1)
    s = stream_of(pts)
    arr = None

    def pack():
        import ctypes
        nonlocal arr
        arr = ctypes.cast((ctypes.c_void_p * 24)(*[p.data_ptr() for p in params]), ctypes.c_void_p)
        check(L.nerf_mlp_pack(arr, dt, ptr(pf), ptr(pb), s), "pack")

    kern = {
        "fwd": lambda: check(L.nerf_mlp_fwd(ptr(pf), dt, ptr(pts), ptr(vd), 192, None, M, 0, ptr(raw), None, None, s),
                             "fwd"),
        "fwd_train": lambda: check(L.nerf_mlp_fwd(ptr(pf), dt, ptr(pts), ptr(vd), 192, None, M, 1, ptr(raw), ptr(act),
                                                  ptr(masks), s), "fwd_train"),
        "dx": lambda: check(L.nerf_mlp_bwd_dx(ptr(pb), dt, ptr(d_raw), M, ptr(masks), ptr(dz), s), "dx"),
        "dw": lambda: check(L.nerf_mlp_bwd_dw(dt, M, ptr(act), ptr(dz), ptr(grad), s), "dw"),
        "density": lambda: check(L.nerf_mlp_fwd(ptr(pf), dt, ptr(pts), None, 1, None, M, 2, ptr(raw), None, None, s),
                                 "density"),
        "pack": pack,
    }
    out = {"M": M, "dtype": args.dtype}
    if args.chunks:
        kern["fwd_train"]()  # (act and masks of a real forward)
        if args.overlap:
            return overlapped_backward(args, L, dt, M, pb, d_raw, masks, act, dz, grad)
        return chunked_backward(args, L, dt, M, pb, d_raw, masks, act, dz, grad, s)
    for name, fn in kern.items():
        fn()
        torch.cuda.synchronize()
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(args.reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        ms = a.elapsed_time(b) / args.reps
        ent = {"ms": round(ms, 4)}
        if name in FLOP:
            ent["tflops"] = round(FLOP[name] * M / (ms * 1e-3) / 1e12, 1)
        out[name] = ent
    print(json.dumps(out), flush=True)


def chunked_backward(args, L, dt, M, pb, d_raw, masks, act, dz, grad, s):
    """dX + dW (deterministic workspace form) over the whole M, against the same work in chunks of C
    samples (C a multiple of 256: the stores are block-major, a chunk is a contiguous byte range of
    every store).  Prints ms per variant, and whether the chunked gradient equals the one-launch
    one (it need not be bit-equal: the per-item partial sums add in another order)."""
    z_blk = L.nerf_mlp_dz_bytes(dt, 256) // 8    # bytes per 32-sample block of each store
    a_blk = L.nerf_mlp_act_bytes(dt, 256) // 8
    m_blk = L.nerf_mlp_mask_bytes(256) // 8
    sizes = [M] + [int(c) for c in args.chunks.split(",")]
    ws = torch.empty(L.nerf_mlp_dw_workspace_bytes(dt, M), dtype=torch.uint8, device=act.device)
    out = {"M": M, "dtype": args.dtype, "ms": {}}
    grads = {}

    def run(C):
        for s0 in range(0, M, C):
            m = min(C, M - s0)
            b0 = s0 // 32
            check(L.nerf_mlp_bwd_dx(ptr(pb), dt, d_raw.data_ptr() + s0 * 16, m, masks.data_ptr() + b0 * m_blk,
                                    dz.data_ptr() + b0 * z_blk, s), "dx")
            check(L.nerf_mlp_bwd_dw_ws(dt, m, act.data_ptr() + b0 * a_blk, dz.data_ptr() + b0 * z_blk, ptr(grad),
                                       ptr(ws), s), "dw")
    for C in sizes:
        assert C % 256 == 0
        grad.zero_()
        run(C)
        torch.cuda.synchronize()
        grads[C] = grad.clone()
        times = []
        for _ in range(args.rounds):
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(args.reps):
                run(C)
            b.record()
            torch.cuda.synchronize()
            times.append(a.elapsed_time(b) / args.reps)
        times.sort()
        out["ms"][str(C)] = round(times[len(times) // 2], 4)
    g0 = grads[M]
    out["max_rel_diff_vs_one_launch"] = {str(C): float((grads[C] - g0).abs().max() / g0.abs().max()) for C in sizes[1:]}
    print(json.dumps(out), flush=True)


def overlapped_backward(args, L, dt, M, pb, d_raw, masks, act, dz, grad):
    """The step's two MLP backwards (fine: M samples in chunks of C; then coarse: N samples, its
    own buffers) run sequentially on one stream, against the same launches with every dW on a
    second stream (event-ordered after its dX), so the next dX -- the fine net's next chunk, or
    the coarse net's -- runs while the previous dW streams its dZ.  Prints median ms of each
    form and whether the two gradients are bit-equal (they must be: the same launches)."""
    dev = act.device
    N = args.overlap
    z_blk, a_blk = L.nerf_mlp_dz_bytes(dt, 256) // 8, L.nerf_mlp_act_bytes(dt, 256) // 8
    m_blk = L.nerf_mlp_mask_bytes(256) // 8
    main, side = torch.cuda.current_stream(), torch.cuda.Stream()
    dz2 = torch.empty(L.nerf_mlp_dz_bytes(dt, N), dtype=torch.uint8, device=dev)
    grad2 = torch.zeros_like(grad)
    ws = [torch.empty(L.nerf_mlp_dw_workspace_bytes(dt, M), dtype=torch.uint8, device=dev) for _ in range(2)]
    out = {"M": M, "N": N, "dtype": args.dtype, "ms": {}}
    grads = {}

    def job(C):  # (samples, dX args, dW args) per launch pair, in step order
        jobs = []
        for s0 in range(0, M, C):
            m, b0 = min(C, M - s0), s0 // 32
            jobs.append((m, d_raw.data_ptr() + s0 * 16, masks.data_ptr() + b0 * m_blk, dz.data_ptr() + b0 * z_blk,
                         act.data_ptr() + b0 * a_blk, grad))
        jobs.append((N, d_raw.data_ptr(), masks.data_ptr(), dz2.data_ptr(), act.data_ptr(), grad2))
        return jobs

    def run(C, overlap):
        for i, (m, draw, msk, dzp, actp, g) in enumerate(job(C)):
            check(L.nerf_mlp_bwd_dx(ptr(pb), dt, draw, m, msk, dzp, main.cuda_stream), "dx")
            if overlap:
                e = torch.cuda.Event()
                e.record(main)
                side.wait_event(e)
                check(L.nerf_mlp_bwd_dw_ws(dt, m, actp, dzp, ptr(g), ptr(ws[1]), side.cuda_stream), "dw")
            else:
                check(L.nerf_mlp_bwd_dw_ws(dt, m, actp, dzp, ptr(g), ptr(ws[0]), main.cuda_stream), "dw")
        if overlap:
            e = torch.cuda.Event()
            e.record(side)
            main.wait_event(e)
    for C in [int(c) for c in args.chunks.split(",")]:
        for overlap in (False, True):
            key = f"{C}_{'overlap' if overlap else 'seq'}"
            grad.zero_()
            grad2.zero_()
            run(C, overlap)
            torch.cuda.synchronize()
            grads[key] = (grad.clone(), grad2.clone())
            times = []
            for _ in range(args.rounds):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(main)
                for _ in range(args.reps):
                    run(C, overlap)
                b.record(main)
                torch.cuda.synchronize()
                times.append(a.elapsed_time(b) / args.reps)
            times.sort()
            out["ms"][key] = round(times[len(times) // 2], 4)
        g_s, g_o = grads[f"{C}_seq"], grads[f"{C}_overlap"]
        out[f"{C}_bit_equal"] = bool(torch.equal(g_s[0], g_o[0]) and torch.equal(g_s[1], g_o[1]))
    print(json.dumps(out), flush=True)


def load_handle(path):
    import ctypes
    h = ctypes.CDLL(os.path.abspath(path))
    for name, (res, argt) in _lib.SIGNATURES.items():
        if not hasattr(h, name):  # (an older build: only the MLP entry points are used here)
            continue
        fn = getattr(h, name)
        fn.restype = res
        fn.argtypes = argt
    return h


def compare(args):
    """Interleaved rounds over several builds in one process (cross-process variance and
    DVFS drift otherwise look like kernel differences): median ms per kernel per build."""
    import statistics
    dev = torch.device("cuda:0")
    dt = ops.dtype_code(args.dtype)
    M = args.M
    torch.manual_seed(0)
    shapes = [(256, 63), (256,)] + [(256, 256), (256,)] * 4 + [(256, 319), (256,)] + [(256, 256), (256,)] * 2 + \
             [(128, 283), (128,), (256, 256), (256,), (1, 256), (1,), (3, 128), (3,)]
    params = [(torch.rand(s, device=dev) - 0.5) * (0.2 if len(s) == 2 else 0.1) for s in shapes]
    import ctypes
    arr = ctypes.cast((ctypes.c_void_p * 24)(*[p.data_ptr() for p in params]), ctypes.c_void_p)
    pts = (torch.rand(M, 3, device=dev) - 0.5) * 3
    vd = torch.nn.functional.normalize(torch.randn(M // 192 + 1, 3, device=dev), dim=-1)
    d_raw = torch.randn(M, 4, device=dev) * 1e-3
    s = torch.cuda.current_stream().cuda_stream
    libs = [(os.path.basename(p).replace(".so", ""), load_handle(p)) for p in args.libs.split(",")]
    bufs = {}
    for name, L in libs:
        pf = torch.empty(L.nerf_mlp_packed_bytes(dt, 0), dtype=torch.uint8, device=dev)
        pb = torch.empty(L.nerf_mlp_packed_bytes(dt, 1), dtype=torch.uint8, device=dev)
        L.nerf_mlp_pack(arr, dt, ptr(pf), ptr(pb), s)
        bufs[name] = dict(pf=pf, pb=pb, raw=torch.empty(M, 4, device=dev),
                          act=torch.empty(L.nerf_mlp_act_bytes(dt, M), dtype=torch.uint8, device=dev),
                          masks=torch.empty(L.nerf_mlp_mask_bytes(M), dtype=torch.uint8, device=dev),
                          dz=torch.empty(L.nerf_mlp_dz_bytes(dt, M), dtype=torch.uint8, device=dev),
                          grad=torch.zeros(L.nerf_mlp_net_params(), device=dev))

    def kernels(L, b):
        return {
            "fwd": lambda: L.nerf_mlp_fwd(ptr(b["pf"]), dt, ptr(pts), ptr(vd), 192, None, M, 0, ptr(b["raw"]), None,
                                          None, s),
            "fwd_train": lambda: L.nerf_mlp_fwd(ptr(b["pf"]), dt, ptr(pts), ptr(vd), 192, None, M, 1, ptr(b["raw"]),
                                                ptr(b["act"]), ptr(b["masks"]), s),
            "dx": lambda: L.nerf_mlp_bwd_dx(ptr(b["pb"]), dt, ptr(d_raw), M, ptr(b["masks"]), ptr(b["dz"]), s),
            "dw": lambda: L.nerf_mlp_bwd_dw(dt, M, ptr(b["act"]), ptr(b["dz"]), ptr(b["grad"]), s),
        }
    times = {(n, k): [] for n, _ in libs for k in ("fwd", "fwd_train", "dx", "dw")}
    for r in range(args.rounds + 1):
        for name, L in libs:
            for k, fn in kernels(L, bufs[name]).items():
                fn()
                torch.cuda.synchronize()
                a = torch.cuda.Event(enable_timing=True)
                e = torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(args.reps):
                    st = fn()
                    assert st == 0, (name, k)
                e.record()
                torch.cuda.synchronize()
                if r:
                    times[(name, k)].append(a.elapsed_time(e) / args.reps)
    out = {"M": M, "rounds": args.rounds}
    out["packed_fwd_addr_mod_2MiB"] = {name: bufs[name]["pf"].data_ptr() % (2 << 20) for name, _ in libs}
    # the builds must compute the same thing: forward raw, the stored activations and the dX
    # stores, bit for bit (buffers zeroed first: padding a kernel never writes stays equal)
    n0 = libs[0][0]
    for name, L in libs:
        for key in ("raw", "act", "masks", "dz"):
            bufs[name][key].zero_()
        kernels(L, bufs[name])["fwd_train"]()
        kernels(L, bufs[name])["dx"]()
    torch.cuda.synchronize()
    out["identical_to_" + n0] = {name: {key: bool(torch.equal(bufs[name][key], bufs[n0][key]))
                                        for key in ("raw", "act", "masks", "dz")} for name, _ in libs[1:]}
    # and the inference forward's output
    for name, L in libs:
        bufs[name]["raw"].zero_()
        kernels(L, bufs[name])["fwd"]()
    torch.cuda.synchronize()
    for name, _ in libs[1:]:
        out["identical_to_" + n0][name]["raw_inference"] = bool(torch.equal(bufs[name]["raw"], bufs[n0]["raw"]))
    # and the deterministic dW of each build's own stores (the store layout may differ between builds;
    # the gradient may not)
    for name, L in libs:
        b = bufs[name]
        kernels(L, b)["fwd_train"]()
        kernels(L, b)["dx"]()
        ws = torch.empty(L.nerf_mlp_dw_workspace_bytes(dt, M), dtype=torch.uint8, device=dev)
        b["grad"].zero_()
        assert L.nerf_mlp_bwd_dw_ws(dt, M, ptr(b["act"]), ptr(b["dz"]), ptr(b["grad"]), ptr(ws), s) == 0
    torch.cuda.synchronize()
    for name, _ in libs[1:]:
        out["identical_to_" + n0][name]["grad_deterministic"] = bool(torch.equal(bufs[name]["grad"],
                                                                                 bufs[n0]["grad"]))
    for name, _ in libs:
        out[name] = {k: round(statistics.median(times[(name, k)]), 4) for k in ("fwd", "fwd_train", "dx", "dw")}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
