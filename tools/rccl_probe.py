"""RCCL ("nccl" backend) probe at world size 1 -- the only RCCL run a one-GPU box allows (RCCL
refuses two ranks on one device).  It runs the collective calls the data-parallel step makes
(trainer.GradBuckets: async SUM all-reduce of the per-net slices of the flat gradient, then
wait + the 1/W scale; broadcast of the initial weights; bench's all_gather of per-rank
times) on the real 1,191,688-float gradient size, checks the results, times them with HIP
events, and prints one JSON line.

    python tools/rccl_probe.py        (starts torch.distributed.run --nproc-per-node 1 as a child)
"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    import torch
    import torch.distributed as dist
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist.init_process_group("nccl", init_method="env://", device_id=dev)
    n_net = 595844
    g = torch.arange(2 * n_net, dtype=torch.float32, device=dev) * 1e-3
    ref = g.clone()
    works = [dist.all_reduce(g[n_net:], op=dist.ReduceOp.SUM, async_op=True),   # fine bucket first
             dist.all_reduce(g[:n_net], op=dist.ReduceOp.SUM, async_op=True)]
    for w in works:
        w.wait()
    g.mul_(1.0 / dist.get_world_size())
    ok_reduce = bool(torch.equal(g, ref))
    p = torch.randn(1000, device=dev)
    p0 = p.clone()
    dist.broadcast(p, src=0)
    ok_bcast = bool(torch.equal(p, p0))
    parts = [torch.empty(1, dtype=torch.float64, device=dev) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, torch.tensor([1.5], dtype=torch.float64, device=dev))
    ok_gather = float(parts[0]) == 1.5
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for _ in range(5):
        dist.all_reduce(g)
    torch.cuda.synchronize()
    ev[0].record()
    reps = 50
    for _ in range(reps):
        dist.all_reduce(g)
    ev[1].record()
    torch.cuda.synchronize()
    out = {"backend": dist.get_backend(), "world_size": dist.get_world_size(), "ok_bucket_allreduce": ok_reduce,
           "ok_broadcast": ok_bcast, "ok_all_gather": ok_gather,
           "allreduce_4.77MB_ms": round(ev[0].elapsed_time(ev[1]) / reps, 4),
           "rccl": getattr(torch.cuda, "nccl", None) and str(torch.cuda.nccl.version()), "torch": torch.__version__}
    print(json.dumps(out), flush=True)
    dist.destroy_process_group()
    if not (ok_reduce and ok_bcast and ok_gather):
        sys.exit(1)


if __name__ == "__main__":
    if "WORLD_SIZE" not in os.environ:
        import socket
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1", "--master-addr",
               "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)]
        t0 = time.time()
        rc = subprocess.run(cmd).returncode
        print(f"[rccl_probe] rc={rc} in {time.time() - t0:.1f} s", file=sys.stderr)
        sys.exit(rc)
    main()
