"""Benchmark: lego NeRF training rays/s (forward + backward, 64 coarse + 128 fine samples).

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

A step is one full training step of the reference hot path on one GPU's batch:
4096 random rays (GPU ray generation from a 100-view 800x800 synthetic lego-shaped scene)
-> stratified sampling -> coarse MLP -> compositing -> importance sampling + merge -> fine
MLP -> compositing -> MSE(c)+MSE(f) -> backward of everything -> gradient all-reduce
(RCCL, N > 1) -> fused clip_grad_value_(40) + Adam.  Weak scaling: 4096 rays per GPU.
Weights: the reference's seed-0 init (torch.manual_seed(0); Network()).  Data is
synthetic (no dataset offline).  Rank 0 prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

os.environ.setdefault("NERF_AMD_NO_ARGV", "1")
ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "nerf-replication_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "train rays/sec (fwd+bwd, 64+128 samples) + 800x800 render s/frame, 1/2/4/8 GPU"
# algorithmic FLOP per MLP sample: 593,408 MAC forward; backward dX 557,696 MAC
# (no input grad for PE(xyz) at layers 0/5 and PE(dir) at the view layer), dW 593,408 MAC
FLOP_PER_SAMPLE = {"mlp_fwd_train": 2 * 593408, "mlp_fwd": 2 * 593408, "mlp_bwd_dx": 2 * 557696,
                   "mlp_bwd_dw": 2 * 593408}
# the dW GEMMs stream the training stores once: every stored activation tile (79 x 32 rows)
# and output-gradient tile (78 x 32 rows) of a sample, 2 B (bf16) / 4 B (fp32) per value
# (DESIGN.md 4); that makes dW HBM-bound, the other MLP kernels MFMA-bound
STORE_ROWS = (79 + 78) * 32
BOUND = {"mlp_fwd_train": "mfma", "mlp_fwd": "mfma", "mlp_bwd_dx": "mfma", "mlp_bwd_dw": "hbm"}
PEAK_HBM_GBS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md)
PEAK_TFLOPS = {"bf16": 2500.0, "fp32": 157.3}  # MI355X dense MFMA (MI355X_MICROARCH.md)
# HBM-bound sampling / compositing kernels; ops.py counts their algorithmic bytes per launch
STREAM_KERNELS = ("raygen", "sample_stratified", "sample_pdf", "composite_fwd", "composite_bwd")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--rays", type=int, default=4096, help="rays per GPU per step")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--images", type=int, default=100)
    ap.add_argument("--res", type=int, default=800)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-render", action="store_true")
    ap.add_argument("--cpu-rays", type=int, default=1024)
    ap.add_argument("--detail-steps", type=int, default=5,
                    help="extra untimed steps that time the sampling/compositing kernels (after the timed region)")
    return ap.parse_args()


def pmc_traffic(kernel, dtype):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary
    (profiles/r*/traffic.json, written by tools/pmc_traffic.py from rocprofv3 --pmc
    FETCH_SIZE / WRITE_SIZE passes of this bench), or None."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "traffic.json")), reverse=True):
        with open(path) as f:
            d = json.load(f)
        if d.get("dtype") == dtype and kernel in d.get("kernels", {}):
            return d["kernels"][kernel]["traffic_bytes"], os.path.relpath(path, ROOT)
    return None, None


def setup_dist():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", init_method="env://", device_id=torch.device("cuda", local))
    return world, rank, torch.device("cuda", local)


def build(args, device):
    from src.config import cfg
    cfg.task_arg.mlp_dtype = args.dtype
    cfg.task_arg.train_rays = args.rays
    cfg.task_arg.perturb = 1
    from src.datasets.nerf.blender import Dataset
    from src.models import make_network
    from src.train.optimizer import make_optimizer
    from src.train.trainers.make_trainer import make_trainer
    from src.utils.camera import focal_for, pose_spherical

    torch.manual_seed(0)
    net = make_network(cfg)  # reference init order + seed
    trainer = make_trainer(cfg, net)
    opt = make_optimizer(cfg, net)
    thetas = torch.linspace(-180.0, 180.0, args.images + 1)[:-1]
    poses = torch.stack([pose_spherical(float(t), -30.0, 4.0) for t in thetas]).to(device)
    g = torch.Generator(device=device).manual_seed(1234)
    images = torch.rand(args.images, args.res, args.res, 3, device=device, generator=g)
    ds = Dataset.from_arrays(images, poses, focal_for(args.res))
    return cfg, net, trainer, opt, ds


def train_step(cfg, trainer, opt, ds, device):
    rays, rgbs = ds.sample_batch()
    from nerf_amd import ops
    batch = {"rays": rays[None], "rgbs": rgbs[None], "near": ops.device_scalar(2.0, device),
             "far": ops.device_scalar(6.0, device)}
    return trainer.train_step(batch, opt)


def stream_roofline(ktimes, dtype=None):
    """{kernel: launches, avg_ms, achieved GB/s of algorithmic bytes, frac of HBM peak} for the
    HBM-bound sampling and compositing kernels (HIP events on the launching stream).  With
    ``dtype`` (training-step sizes, which the PMC passes run) the PMC traffic per launch is added."""
    out = {}
    for k in STREAM_KERNELS:
        if k not in ktimes:
            continue
        n, ms, nbytes = ktimes[k]
        ach = nbytes / (ms * 1e-3) / 1e9
        out[k] = {"launches": n, "avg_ms": round(ms / n, 4), "bytes_per_launch": nbytes // n, "bound": "hbm",
                  "achieved": round(ach, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": round(ach / PEAK_HBM_GBS, 4)}
        if dtype is not None:
            out[k]["traffic"] = pmc_traffic(k, dtype)[0]
    return out


def detail_times(fn, dtype=None):
    from nerf_amd import ops
    torch.cuda.synchronize()
    ops.KERNEL_TIMES.reset()
    ops.KERNEL_TIMES.enabled = ops.KERNEL_TIMES.detail = True
    try:
        fn()
        torch.cuda.synchronize()
    finally:
        ops.KERNEL_TIMES.enabled = ops.KERNEL_TIMES.detail = False
    return stream_roofline(ops.KERNEL_TIMES.summary(), dtype)


def render_frame_time(cfg, net, ds, device, reps=2):
    from src.models.nerf.renderer.volume_renderer import Renderer
    r = Renderer(net)
    perturb = cfg.task_arg.perturb
    cfg.task_arg.perturb = 0
    rays, _ = ds.image_rays(0)
    batch = {"rays": rays, "near": torch.tensor([2.0], device=device), "far": torch.tensor([6.0], device=device)}
    net.eval()
    times = []
    with torch.no_grad():
        r.render(batch)
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r.render(batch)
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t0)
        # one more frame with the sampling / compositing kernels timed (outside the timed reps)
        stream = detail_times(lambda: r.render(batch))
    net.train()
    cfg.task_arg.perturb = perturb
    return min(times), stream


def grid_times(cfg, net, ds, device, reps=2):
    """BASELINE config 4: the 128^3 x 8-corner occupancy bake (occupancy_grid.py:15-80) and the
    grid-accelerated 800x800 march (render_accelerated, volume_renderer.py:268-357) of test
    view 0 through the reference's own baked lego grid (tests/golden/lego_occupancy_grid.npz,
    packed bits of logs/lego/occupancy_grid.pt).  Weights are the synthetic seed-0 init."""
    import numpy as np
    from nerf_amd import ops
    from src.models.nerf.renderer.volume_renderer import Renderer
    out = {}
    with torch.no_grad():
        def bake():
            return ops.bake(net.model.packer(), 128, 1.0, dtype=cfg.task_arg.mlp_dtype)
        bake()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            grid = bake()
        torch.cuda.synchronize()
        out["bake_s"] = round((time.perf_counter() - t0) / reps, 4)
        out["bake_occupied"] = int(grid.sum())
        z = np.load(os.path.join(ROOT, "tests", "golden", "lego_occupancy_grid.npz"), allow_pickle=False)
        shape = tuple(int(v) for v in z["shape"])
        lego = torch.from_numpy(np.unpackbits(z["packed"])[: int(np.prod(shape))].reshape(shape).astype(bool))
        r = Renderer(net)
        r.set_occupancy_grid(lego, device)
        rays, _ = ds.image_rays(0)
        batch = {"rays": rays, "near": ops.device_scalar(2.0, device), "far": ops.device_scalar(6.0, device)}
        import contextlib
        import io
        with contextlib.redirect_stdout(io.StringIO()):
            r.render_accelerated(batch)
            times = []
            for _ in range(reps):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                o = r.render_accelerated(batch)
                torch.cuda.synchronize()
                times.append(time.perf_counter() - t0)
        out["march_s_per_frame"] = round(min(times), 4)
        out["march_queried_points"] = int(o["n_queried"])
    return out


def cpu_baseline(n_rays):
    """The oracle (tests-only CPU restatement of the reference, torch CPU) on a bounded
    sample: one n_rays forward+backward render (perturb 0), config 1 of BASELINE.json."""
    from oracle import nerf_oracle as O
    torch.set_num_threads(max(1, min(16, os.cpu_count() or 1)))
    state = {k: v.clone().requires_grad_(True) for k, v in O.seeded_network_state(0).items()}
    C, Fn = O.split_params(state, "model"), O.split_params(state, "model_fine")
    pose = O.pose_spherical(30.0, -30.0, 4.0)
    o, d = O.get_rays(800, 800, O.focal_from_angle(800, 0.6911112070083618), pose)
    idx = torch.randint(0, 800 * 800, (n_rays,), generator=torch.Generator().manual_seed(0))
    rays = torch.cat([o.reshape(-1, 3)[idx], d.reshape(-1, 3)[idx]], 1)
    gt = torch.rand(n_rays, 3, generator=torch.Generator().manual_seed(1))

    def once():
        for v in state.values():
            v.grad = None
        ret = O.render(C, Fn, rays, torch.tensor([2.0]), torch.tensor([6.0]))
        O.loss_fn(ret, gt)[0].backward()

    once()
    t0 = time.perf_counter()
    reps = 5
    for _ in range(reps):
        once()
    dt = (time.perf_counter() - t0) / reps
    return {"value": round(n_rays / dt, 2), "unit": "rays/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"{n_rays}-ray forward+backward render (64+128 samples, perturb 0, seed-0 weights), "
                      f"mean of {reps} after 1 warm-up, torch {torch.__version__} CPU"}


def main():
    args = parse()
    world, rank, device = setup_dist()
    from nerf_amd import ops
    cfg, net, trainer, opt, ds = build(args, device)

    for _ in range(args.warmup):
        train_step(cfg, trainer, opt, ds, device)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ops.KERNEL_TIMES.reset()
    ops.KERNEL_TIMES.enabled = True
    t0 = time.perf_counter()
    for _ in range(args.steps):
        train_step(cfg, trainer, opt, ds, device)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    ops.KERNEL_TIMES.enabled = False
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t)
    ktimes = {k: v for k, v in ops.KERNEL_TIMES.summary().items() if k not in STREAM_KERNELS}
    # sampling / compositing kernels per launch, in extra steps after the timed region
    train_stream = detail_times(lambda: [train_step(cfg, trainer, opt, ds, device) for _ in range(args.detail_steps)],
                                 args.dtype) \
        if args.detail_steps > 0 else {}

    rays_total = world * args.rays * args.steps
    value = rays_total / elapsed
    # dominant kernel: largest total device time among the MLP kernels, priced against the
    # roofline that bounds it
    esize = 2 if args.dtype == "bf16" else 4

    def roof(k, n, ms, units):
        avg_ms = ms / n
        if BOUND[k] == "hbm":
            per = STORE_ROWS * esize * units / n
            ach = per / (avg_ms * 1e-3) / 1e9
            return {"bound": "hbm", "achieved": round(ach, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                    "frac": round(ach / PEAK_HBM_GBS, 4), "bytes_per_launch": per, "avg_launch_ms": round(avg_ms, 4)}
        per = FLOP_PER_SAMPLE[k] * units / n
        ach = per / (avg_ms * 1e-3) / 1e12
        return {"bound": "mfma", "achieved": round(ach, 2), "peak": PEAK_TFLOPS[args.dtype], "unit": "TFLOP/s",
                "frac": round(ach / PEAK_TFLOPS[args.dtype], 4), "flop_per_launch": per,
                "avg_launch_ms": round(avg_ms, 4)}

    name, (n_launch, ms, units) = max(ktimes.items(), key=lambda kv: kv[1][1])
    traffic, traffic_src = pmc_traffic(name, args.dtype)
    roofline = dict(kernel=name, **roof(name, n_launch, ms, units), traffic=traffic,
                    traffic_unit="HBM bytes per launch (PMC FETCH_SIZE x2 + WRITE_SIZE)", traffic_source=traffic_src)
    kt = {k: {"launches": n, "avg_ms": round(m / n, 4), "samples_per_launch": u // n,
              "tflops": round(FLOP_PER_SAMPLE.get(k, 0) * (u / n) / (m / n * 1e-3) / 1e12, 2),
              "roofline": roof(k, n, m, u)}
          for k, (n, m, u) in ktimes.items()}

    render_s, grid, render_stream = None, None, None
    if rank == 0 and not args.no_render and world == 1:
        render_s, render_stream = render_frame_time(cfg, net, ds, device)
        grid = grid_times(cfg, net, ds, device)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.cpu_rays)

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "rays/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
            "data": "synthetic (100 spherical 800x800 views, random rgb; seed-0 reference init)",
            "config": {"workload": "lego NeRF train step: coarse 64 + fine 128 samples/ray, 4096 rays/GPU, "
                                   "MSE(c)+MSE(f), clip 40 + Adam",
                       "rays_per_gpu": args.rays, "global_batch_rays": args.rays * world,
                       "samples_per_ray": 64 + 192, "parallelism": f"dp{world}"},
            "roofline": roofline,
            "kernels": kt,
            "stream_kernels": {"train_step": train_stream, "render_800x800": render_stream},
            "render_s_per_frame": None if render_s is None else round(render_s, 4),
            "occupancy_grid": grid,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
