"""Evidence that the next batch's ray generation and stratified sampling run while the
gradient all-reduce is in flight (north_star: "all-reduced ... and overlapped with the next
ray batch"; trainer.py Trainer.train_step(prefetch=)).

Two ranks share cuda:0 over gloo (RCCL needs one GPU per rank; the trainer's collective calls
are the same).  Each rank runs the production 4096-ray step with prefetch, then profiles 4 steps
with torch.profiler (kineto over the ROCm tracer: GPU kernels and copies with device
timestamps).  gloo reduces a CUDA tensor by copying it to the host on its own stream, reducing
on the host and copying it back, so a bucket's reduction window on the device timeline is
[its producer -- the coarse net's dW -- ends, its host-to-device copy ends].  For every profiled step the
script reports the coarse-net bucket's window (the last one to start: the coarse backward runs
after the fine one) and the raygen / stratified kernels of the NEXT batch, which the trainer
enqueues right after the backward, and whether they ran inside the window.

Writes gpurun_out/dp_overlap.json (+ the per-rank chrome traces)."""
import json
import os
import socket
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
BUCKET_BYTES = 595844 * 4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), NERF_AMD_NO_ARGV="1")
    sys.path[:0] = [ROOT, os.path.join(ROOT, "nerf-replication_amd"), os.path.join(ROOT, "tests")]
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        from test_gpu_dp import _batch, _setup
        cfg, net, trainer, opt, ds, dev = _setup("fp32")

        def nxt():
            r, c = ds.sample_batch()
            return _batch(r, c, dev)
        for _ in range(3):
            batch = trainer.prefetched or trainer.prepare(nxt())
            trainer.train_step(batch, opt, prefetch=nxt)
        torch.cuda.synchronize()
        dist.barrier()
        from torch.profiler import ProfilerActivity, profile
        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
            for _ in range(4):
                batch = trainer.prefetched or trainer.prepare(nxt())
                trainer.train_step(batch, opt, prefetch=nxt)
            torch.cuda.synchronize()
        path = os.path.join(OUT, f"dp_overlap_trace_rank{rank}.json")
        prof.export_chrome_trace(path)
        q.put((rank, path, None))
        dist.destroy_process_group()
    except Exception:  # noqa: BLE001 - reported to the parent
        import traceback
        q.put((rank, None, traceback.format_exc()))


def analyse(path):
    with open(path) as f:
        ev = json.load(f)["traceEvents"]
    gpu = [e for e in ev if e.get("ph") == "X" and e.get("cat") in ("kernel", "gpu_memcpy", "gpu_memset")]
    copies = sorted((e for e in gpu if e["cat"] == "gpu_memcpy"
                     and int(e.get("args", {}).get("bytes", e.get("args", {}).get("memory bandwidth (GB/s)", 0)) or 0)
                     in (BUCKET_BYTES,)), key=lambda e: e["ts"])
    if not copies:  # kineto builds that do not record bytes: take copies by direction only
        copies = sorted((e for e in gpu if e["cat"] == "gpu_memcpy"), key=lambda e: e["ts"])
    d2h = [e for e in copies if "DtoH" in e["name"] or "D2H" in e["name"] or "DeviceToHost" in e["name"]]
    h2d = [e for e in copies if "HtoD" in e["name"] or "H2D" in e["name"] or "HostToDevice" in e["name"]]
    kern = sorted((e for e in gpu if e["cat"] == "kernel"), key=lambda e: e["ts"])
    rg = [e for e in kern if "raygen" in e["name"]]
    st = [e for e in kern if "stratified" in e["name"]]
    adam = [e for e in kern if "adam" in e["name"]]
    dwr = [e for e in kern if "dw_reduce" in e["name"] or ("dw_kernel" in e["name"])]
    steps = []
    for a in adam:  # one Adam per step; its coarse bucket = the last D2H..H2D before it
        d = [c for c in d2h if c["ts"] < a["ts"]]
        h = [c for c in h2d if c["ts"] < a["ts"]]
        if not d or not h:
            continue
        # the reduction is in flight from the moment its bucket is complete (the end of the
        # coarse net's dW, the bucket's producer) until its result is back on the device
        prod = [k for k in dwr if k["ts"] + k["dur"] <= d[-1]["ts"] + 1.0]
        w0 = (prod[-1]["ts"] + prod[-1]["dur"]) if prod else d[-1]["ts"]
        w1 = h[-1]["ts"] + h[-1]["dur"]
        r = [k for k in rg if w0 - 5000 < k["ts"] < a["ts"]]
        s = [k for k in st if w0 - 5000 < k["ts"] < a["ts"]]
        inside = lambda ks: bool(ks) and all(w0 <= k["ts"] and k["ts"] + k["dur"] <= w1 for k in ks)  # noqa: E731
        steps.append({
            "bucket_ready_us": round(w0, 1), "d2h_start_us": round(d[-1]["ts"], 1), "h2d_end_us": round(w1, 1),
            "reduction_in_flight_us": round(w1 - w0, 1),
            "next_raygen_us": [[round(k["ts"], 1), round(k["ts"] + k["dur"], 1)] for k in r],
            "next_stratified_us": [[round(k["ts"], 1), round(k["ts"] + k["dur"], 1)] for k in s],
            "adam_start_us": round(a["ts"], 1),
            "raygen_inside": inside(r), "stratified_inside": inside(s),
            "prefetch_before_adam": bool(r) and bool(s) and max(k["ts"] + k["dur"] for k in r + s) <= a["ts"],
        })
    return {"n_d2h": len(d2h), "n_h2d": len(h2d), "n_adam": len(adam), "steps": steps,
            "copy_names": sorted({c["name"] for c in copies})[:6]}


def main():
    os.makedirs(OUT, exist_ok=True)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    out = {}
    for rank, path, err in sorted(res, key=lambda t: t[0]):
        if err:
            print(err)
            sys.exit(1)
        out[f"rank{rank}"] = analyse(path)
    with open(os.path.join(OUT, "dp_overlap.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1)[:3000])


if __name__ == "__main__":
    main()
