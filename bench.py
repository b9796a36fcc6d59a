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

The headline (``value``, ``dtype`` "fp32") runs the MLP in fp32 MFMA, the reference's own
precision (nn.Linear fp32, network.py:22-74).  Three opt-in MLP precisions are measured in the
same run and reported as nested, labelled lines: ``bf16x3_line`` (split-bf16 operands, three
bf16 MFMAs per product, ~1e-5 relative per dot product; priced against 1/3 of the bf16 peak),
``bf16x3f_line`` (the bf16x3 forward -- its rgb/depth are bf16x3's -- with the bf16 backward)
and ``bf16_line`` (operands rounded to bf16: the non-conforming tier, rgb/depth within the north_star's
2e-3 on >= 95 % of values only -- DESIGN.md section 5; bf16x3 / bf16x3f hold it on every value).
``vs_baseline`` of every line divides by ONE number: the reference's per-step fp32 op graph run
eagerly by PyTorch-ROCm on the same GPU with perturb 1 (``baseline``: median of 21 steps, measured
once per run after the tiers); ``cpu_baseline`` is the same graph on the host cores (config 1).
"""
import argparse
import json
import os
import subprocess
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
# (no input grad for PE(xyz) at layers 0/5 and PE(dir) at the view layer), dW 593,408 MAC.
# Every MLP kernel is priced against the MFMA peak of its dtype (SURVEY.md 8d roofline table).
FLOP_PER_SAMPLE = {"mlp_fwd_train": 2 * 593408, "mlp_fwd": 2 * 593408, "mlp_bwd_dx": 2 * 557696,
                   "mlp_bwd_dw": 2 * 593408}
# bytes the training stores add per sample: 79 activation + 78 output-gradient
# tiles of 32 rows, written once and read once; the MLP's own algorithmic I/O is 44 B/sample
# (pts 12 + raw 16 + d_raw 16)
STORE_ROWS = (79 + 78) * 32
MLP_IO_BYTES = 12 + 16 + 16
PEAK_HBM_GBS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md)
# MI355X dense MFMA (MI355X_MICROARCH.md); bf16x3 spends 3 bf16 MFMAs per fp32 product
PEAK_TFLOPS = {"bf16": 2500.0, "fp32": 157.3, "bf16x3": 2500.0 / 3}
ALL_DTYPES = ("fp32", "bf16x3", "bf16x3f", "bf16")


def kernel_prec(kernel: str, dtype: str) -> str:
    """The arithmetic a kernel of an MLP tier runs in: bf16x3f = bf16x3 forward + bf16 backward."""
    if dtype == "bf16x3f":
        return "bf16x3" if kernel.startswith("mlp_fwd") else "bf16"
    return dtype


# HBM-bound sampling / compositing kernels; ops.py counts their algorithmic bytes per launch
STREAM_KERNELS = ("raygen", "sample_stratified", "sample_pdf", "composite_pdf", "composite_fwd", "composite_bwd")


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); without a torch.distributed environment, N > 1 starts "
                         "torch.distributed.run as a child process (default: WORLD_SIZE, else 1)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--rays", type=int, default=4096, help="rays per GPU per step")
    ap.add_argument("--dtype", default="fp32", choices=list(ALL_DTYPES), help="headline MLP dtype")
    ap.add_argument("--images", type=int, default=100)
    ap.add_argument("--res", type=int, default=800)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-eager-baseline", action="store_true")
    ap.add_argument("--no-second", action="store_true", help="skip the labelled lines of the other MLP dtypes")
    ap.add_argument("--no-render", action="store_true")
    ap.add_argument("--cpu-rays", type=int, default=1024)
    ap.add_argument("--detail-steps", type=int, default=5,
                    help="extra untimed steps that time the sampling/compositing kernels (after the timed region)")
    return ap.parse_args(argv)


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launcher_command(gpus: int, argv, port: int):
    """The torch.distributed.run command that runs this script as ``gpus`` ranks on one node
    (the driver's own form: --nnodes=1, rendezvous on 127.0.0.1)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)


def check_world(gpus, env=os.environ):
    """(world size this process runs at, error or None).  Under torch.distributed.run the world
    is WORLD_SIZE; an explicit --gpus that disagrees with it is an error (the bench would
    otherwise report a rank count nobody asked for)."""
    if "WORLD_SIZE" in env:
        world = int(env["WORLD_SIZE"])
        if gpus is not None and gpus != world:
            return world, f"--gpus {gpus} but WORLD_SIZE={world}: launch with --nproc-per-node {gpus}"
        return world, None
    return (1 if gpus is None else gpus), None


def launch_ranks(gpus: int, argv) -> int:
    """--gpus N > 1 in a plain process: start torch.distributed.run with N ranks as a CHILD
    process (never an exec; this process has made no GPU call), relay rank 0's stdout (the
    JSON line) and return the child's exit status."""
    cmd = launcher_command(gpus, argv, free_port())
    log("launching " + " ".join(cmd))
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, env=env, text=True, bufsize=1)
    for line in proc.stdout:
        sys.stdout.write(line)
        sys.stdout.flush()
    return proc.wait()


def pmc_traffic(kernel, dtype, samples=None):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary
    (profiles/r*/traffic.json, written by tools/pmc_traffic.py from rocprofv3 --pmc
    FETCH_SIZE / WRITE_SIZE passes of this bench), or (None, None).  An MLP kernel's bytes are
    proportional to its samples: with ``samples`` (this run's samples per launch) they are
    scaled from the summary's ``mlp_samples_per_launch`` (the PMC run's; 524,288 = the mean of
    the coarse and the fine launch when each backward is one launch)."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "traffic*.json")), reverse=True):
        with open(path) as f:
            d = json.load(f)
        if d.get("dtype") == dtype and kernel in d.get("kernels", {}):
            t = d["kernels"][kernel]["traffic_bytes"]
            if samples is not None and kernel.startswith("mlp_"):
                t = t * samples / d.get("mlp_samples_per_launch", 524288)
            return t, os.path.relpath(path, ROOT)
    return None, None


def setup_dist():
    """One process per GPU over RCCL ("nccl").  NERF_BENCH_BACKEND=gloo (rehearsal only) lets
    several ranks share the GPUs of a smaller box (device = local rank mod device count)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("NERF_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", init_method="env://", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend, init_method="env://")
        assert dist.get_world_size() == world, (dist.get_world_size(), world)
    return world, rank, torch.device("cuda", local)


def gather_floats(x: float, device):
    """[x of rank 0, x of rank 1, ...] (rank order)."""
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return [x]
    dev = device if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t)
    return [float(p) for p in parts]


def allreduce_standalone(n: int, device, reps: int = 20):
    """Mean ms of one SUM all-reduce of an n-float fp32 buffer (the flat gradient's size) on
    this process group, outside the training step: the link cost the step hides."""
    dev = device if dist.get_backend() == "nccl" else "cpu"
    g = torch.ones(n, dtype=torch.float32, device=dev)
    for _ in range(3):
        dist.all_reduce(g)
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        dist.all_reduce(g)
    if dev != "cpu":
        torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def build(args, device, dtype):
    from src.config import cfg
    cfg.task_arg.mlp_dtype = dtype
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


def next_batch(ds, device):
    from nerf_amd import ops
    rays, rgbs = ds.sample_batch()
    return {"rays": rays[None], "rgbs": rgbs[None], "near": ops.device_scalar(2.0, device),
            "far": ops.device_scalar(6.0, device)}


def train_step(cfg, trainer, opt, ds, device):
    """One training step as Trainer.train runs it: this step's batch was prepared during the
    previous step (its rays and first-chunk stratified samples overlap that step's gradient
    all-reduce); the next one is prepared here the same way."""
    batch = getattr(trainer, "prefetched", None) or trainer.prepare(next_batch(ds, device))
    return trainer.train_step(batch, opt, prefetch=lambda: next_batch(ds, device))


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


def mlp_roofline(k, n, ms, units, dtype):
    """Algorithmic FLOP of one launch (SURVEY.md 8d per-sample figure x samples) / its mean
    HIP-event duration, against the dtype's dense MFMA peak."""
    avg_ms = ms / n
    per = FLOP_PER_SAMPLE[k] * units / n
    ach = per / (avg_ms * 1e-3) / 1e12
    peak = PEAK_TFLOPS[kernel_prec(k, dtype)]
    return {"bound": "mfma", "achieved": round(ach, 2), "peak": peak, "unit": "TFLOP/s",
            "frac": round(ach / peak, 4), "flop_per_launch": per, "samples_per_launch": units // n,
            "avg_launch_ms": round(avg_ms, 4)}


def hbm_roofline(k, n, ms, dtype, samples=None):
    """The same launch against HBM: PMC bytes per launch (the newest committed traffic summary
    for this dtype, profiles/r*/traffic_*.json) / its mean HIP-event duration, against 8 TB/s.
    The bf16 training kernels move their stored tiles at 4.6-5.7 TB/s (the ~6.3 TB/s a copy
    reaches, MI355X_MICROARCH.md): HBM, not the MFMA, bounds them."""
    traffic, src = pmc_traffic(k, dtype, samples)
    if traffic is None:
        return None
    ach = traffic / (ms / n * 1e-3) / 1e9
    return {"bound": "hbm", "traffic": traffic, "achieved": round(ach, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": round(ach / PEAK_HBM_GBS, 4), "traffic_source": src}


def measure_training(args, world, rank, device, dtype):
    """Warmup + exactly args.steps timed steps (barrier + synchronize on both sides, max over
    ranks).  Returns (rays/s, ms/step, roofline, per-kernel table, train-size stream kernels,
    (cfg, net, ds))."""
    from nerf_amd import ops
    cfg, net, trainer, opt, ds = build(args, device, dtype)
    for _ in range(args.warmup):
        train_step(cfg, trainer, opt, ds, device)
    if world > 1:
        dist.barrier()
        trainer.buckets.events = []
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
    dist_info = None
    if world > 1:
        per_rank = gather_floats(elapsed / args.steps * 1e3, device)
        exposed = gather_floats(trainer.buckets.exposed_ms() or 0.0, device)
        trainer.buckets.events = None
        elapsed = max(per_rank) * args.steps / 1e3
        dist_info = {"backend": dist.get_backend(), "world_size": dist.get_world_size(),
                     "ms_per_step_per_rank": [round(x, 3) for x in per_rank],
                     "allreduce_exposed_ms_per_step_per_rank": [round(x, 4) for x in exposed],
                     "allreduce_standalone_ms": round(allreduce_standalone(opt.flat_grad.numel(), device), 4),
                     "allreduce_bytes": opt.flat_grad.numel() * 4,
                     "note": "exposed = compute-stream time in GradBuckets.finish (wait for the per-net "
                             "buckets + 1/W scale), HIP events; standalone = one all-reduce of the flat "
                             "gradient's size outside the step"}
    ktimes = {k: v for k, v in ops.KERNEL_TIMES.summary().items() if k not in STREAM_KERNELS}
    train_stream = detail_times(lambda: [train_step(cfg, trainer, opt, ds, device) for _ in range(args.detail_steps)],
                                dtype) if args.detail_steps > 0 else {}
    value = world * args.rays * args.steps / elapsed
    # dominant kernel: largest total device time among the MLP kernels
    name, (n_launch, ms, units) = max(ktimes.items(), key=lambda kv: kv[1][1])
    esize = 2 if dtype in ("bf16", "bf16x3f") else 4
    traffic, traffic_src = pmc_traffic(name, dtype, units / n_launch)
    store_bytes = STORE_ROWS * esize * units / n_launch
    io_bytes = MLP_IO_BYTES * units / n_launch
    roofline = dict(kernel=name, **mlp_roofline(name, n_launch, ms, units, dtype), traffic=traffic,
                    traffic_unit="HBM bytes per launch (PMC FETCH_SIZE x2 + WRITE_SIZE)", traffic_source=traffic_src,
                    store_bytes_per_launch=store_bytes, mlp_io_bytes_per_launch=io_bytes,
                    traffic_vs_mlp_io=None if traffic is None else round(traffic / io_bytes, 1))
    kt = {k: {"launches": n, "avg_ms": round(m / n, 4), "roofline": mlp_roofline(k, n, m, u, dtype),
              "hbm": hbm_roofline(k, n, m, dtype, u / n)} for k, (n, m, u) in ktimes.items()}
    return value, elapsed / args.steps * 1e3, roofline, kt, train_stream, (cfg, net, ds), dist_info


def render_frame_time(cfg, net, ds, device, world, reps=2):
    """800x800 hierarchical render of test view 0 (perturb 0), rays split over the ranks
    (src/utils/dist_render.py) and gathered; max over ranks."""
    from src.models.nerf.renderer.volume_renderer import Renderer
    from src.utils.dist_render import render_distributed
    r = Renderer(net)
    perturb = cfg.task_arg.perturb
    cfg.task_arg.perturb = 0
    rays, _ = ds.image_rays(0)
    batch = {"rays": rays, "near": torch.tensor([2.0], device=device), "far": torch.tensor([6.0], device=device)}
    net.eval()
    times = []
    keys = ("rgb_map_f", "depth_map_f", "acc_map_f")
    with torch.no_grad():
        render_distributed(r, batch, keys=keys)
        for _ in range(reps):
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            render_distributed(r, batch, keys=keys)
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t0)
        stream = detail_times(lambda: r.render(batch)) if world == 1 else None
    net.train()
    cfg.task_arg.perturb = perturb
    t = min(times)
    if world > 1:
        tt = torch.tensor([t], device=device, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t = float(tt)
    return t, stream


def lego_grid():
    import numpy as np
    z = np.load(os.path.join(ROOT, "tests", "golden", "lego_occupancy_grid.npz"), allow_pickle=False)
    shape = tuple(int(v) for v in z["shape"])
    return torch.from_numpy(np.unpackbits(z["packed"])[: int(np.prod(shape))].reshape(shape).astype(bool))


def max_over_ranks(t: float, device) -> float:
    if dist.is_initialized() and dist.get_world_size() > 1:
        tt = torch.tensor([t], device=device, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t = float(tt)
    return t


def timed_frames(fn, device, reps):
    """(output of the last call, min over reps of the max-over-ranks wall time)."""
    import contextlib
    import io
    with contextlib.redirect_stdout(io.StringIO()):
        fn()
        times = []
        for _ in range(reps):
            if dist.is_initialized():
                dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            o = fn()
            torch.cuda.synchronize()
            times.append(max_over_ranks(time.perf_counter() - t0, device))
    return o, min(times)


def bake_timed(packer, dtype, device, reps):
    """(grid, s): the res-128 bake (occupancy_grid.py:15-80), one voxel slab per rank +
    all-gather at N > 1 (src/utils/dist_render.py bake_distributed)."""
    from nerf_amd import ops
    from src.utils.dist_render import bake_distributed

    def bake():
        return bake_distributed(lambda slab: ops.bake(packer, 128, 1.0, dtype=dtype, slab=slab), 128)
    return timed_frames(bake, device, reps)


def grid_times(cfg, net, ds, device, reps=2):
    """BASELINE config 4: the 128^3 x 8-corner occupancy bake (occupancy_grid.py:15-80) and the
    grid-accelerated 800x800 march (render_accelerated, volume_renderer.py:268-357) of test
    view 0 through the reference's own baked lego grid (tests/golden/lego_occupancy_grid.npz,
    packed bits of logs/lego/occupancy_grid.pt).  Weights are the synthetic seed-0 init; the
    bake is also timed with the coarse alpha bias shifted by +1 so that the threshold bites
    (as the reference-generated res-8 bake golden does).  At N > 1 the frame's rays are dealt
    to the ranks in interleaved blocks and the bake split in voxel slabs."""
    from nerf_amd import ops
    from src.models.nerf.renderer.volume_renderer import Renderer
    from src.utils.dist_render import render_distributed
    out = {}
    with torch.no_grad():
        for tag, shift in (("", 0.0), ("_shifted", 1.0)):
            net.model.alpha_linear.bias += shift
            grid, t = bake_timed(net.model.packer(), cfg.task_arg.mlp_dtype, device, reps)
            out[f"bake_s{tag}"] = round(t, 4)
            out[f"bake_occupied{tag}"] = int(grid.sum())
            net.model.alpha_linear.bias -= shift
        r = Renderer(net)
        r.set_occupancy_grid(lego_grid(), device)
        rays, _ = ds.image_rays(0)
        batch = {"rays": rays, "near": ops.device_scalar(2.0, device), "far": ops.device_scalar(6.0, device)}
        o, t = timed_frames(lambda: render_distributed(r, batch, accelerated=True,
                                                       keys=("rgb_map_f", "depth_map_f", "acc_map_f")), device, reps)
        out["march_s_per_frame"] = round(t, 4)
        out["march_queried_points"] = int(o["n_queried"])
        out["march_evaluated_points"] = int(o["n_evaluated"])
        out["trained"] = trained_grid_times(cfg, device, reps)
    return out


def trained_grid_times(cfg, device, reps=2):
    """Config 4 on a net where the bake threshold bites and rays terminate: the fixture weights
    trained on the procedural scene (tests/golden/trained_v2.npz, tools/train_teacher.py), its
    own res-128 bake (occupancy_grid.py), then the grid march and the hierarchical render of an
    800x800 held-out view (both split over the ranks at N > 1)."""
    import numpy as np
    from nerf_amd import ops
    from src.datasets.nerf.synthetic import view_poses
    from src.models import make_network
    from src.models.nerf.renderer.volume_renderer import Renderer
    from src.utils.camera import focal_for
    from src.utils.dist_render import render_distributed
    z = np.load(os.path.join(ROOT, "tests", "golden", "trained_v2.npz"), allow_pickle=False)
    torch.manual_seed(0)
    net = make_network(cfg)
    net.load_state_dict({k: torch.from_numpy(z[k]) for k in z.files}, strict=True)
    net = net.to(device).eval()
    out = {}
    keys = ("rgb_map_f", "depth_map_f", "acc_map_f")
    with torch.no_grad():
        grid, t = bake_timed(net.model.packer(), cfg.task_arg.mlp_dtype, device, reps)
        out["bake_s"] = round(t, 4)
        out["bake_occupied"] = int(grid.sum())
        r = Renderer(net)
        r.set_occupancy_grid(grid, device)
        pose = view_poses(2, seed=1)[0].to(device)
        pix = torch.arange(800 * 800, device=device)
        rays, _, _ = ops.raygen(pose.reshape(1, 4, 4), 800, 800, focal_for(800), pix=pix)
        batch = {"rays": rays, "near": ops.device_scalar(2.0, device), "far": ops.device_scalar(6.0, device)}
        o, t = timed_frames(lambda: render_distributed(r, batch, accelerated=True, keys=keys), device, reps)
        out["march_s_per_frame"] = round(t, 4)
        out["march_queried_points"] = int(o["n_queried"])
        out["march_evaluated_points"] = int(o["n_evaluated"])
        out["march_rounds"] = int(o.get("rounds", 0))
        perturb = cfg.task_arg.perturb
        cfg.task_arg.perturb = 0
        _, t = timed_frames(lambda: render_distributed(r, batch, keys=keys), device, 1)
        out["hierarchical_render_s"] = round(t, 4)
        cfg.task_arg.perturb = perturb
    return out


def _bench_rays(O, n, dev):
    """Config-1 rays: pose_spherical(30,-30,4), uniform pixel ids of seed 0; gt rgb seed 1."""
    pose = O.pose_spherical(30.0, -30.0, 4.0)
    o, d = O.get_rays(800, 800, O.focal_from_angle(800, 0.6911112070083618), pose)
    idx = torch.randint(0, 800 * 800, (n,), generator=torch.Generator().manual_seed(0))
    rays = torch.cat([o.reshape(-1, 3)[idx], d.reshape(-1, 3)[idx]], 1)
    gt = torch.rand(n, 3, generator=torch.Generator().manual_seed(1))
    return rays.to(dev), gt.to(dev)


def log(msg):
    """Progress on stderr (the JSON line is the only stdout)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def available_cpus():
    """(cores this process may run on, how that was determined): the affinity mask, capped by
    the cgroup CPU quota when one is set (a container's share of a larger host -- running
    more threads than the quota only oversubscribes it)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    basis = "sched_getaffinity"
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
            if q != "max":
                quota = int(q) / int(p)
    except (OSError, ValueError):
        try:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
                q = int(f.read())
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                p = int(f.read())
            if q > 0:
                quota = q / p
        except (OSError, ValueError):
            pass
    if quota is not None and quota < n:
        n, basis = max(1, int(quota)), "cgroup cpu quota"
    # the GPU box grants each GPU a share of its host's cores and states it in OMP_NUM_THREADS
    # (os.cpu_count() there is the whole machine, shared with other jobs)
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and 0 < int(omp) < n:
        n, basis = int(omp), "OMP_NUM_THREADS (the CPU share granted to this GPU)"
    return n, basis


def cpu_model():
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name:"):
                return line.split(":", 1)[1].strip()
    except Exception:  # noqa: BLE001 - reporting only
        pass
    return None


def cpu_baseline(n_rays):
    """Baseline leg: the oracle (tests-only CPU restatement of the reference op graph, torch
    CPU) on a bounded sample -- config 1 of BASELINE.json, one n_rays forward+backward render
    (perturb 0) -- on every host core available to this process."""
    from oracle import nerf_oracle as O
    threads, basis = available_cpus()
    log(f"cpu baseline on {threads} threads ({basis})")
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        state = {k: v.clone().requires_grad_(True) for k, v in O.seeded_network_state(0).items()}
        C, Fn = O.split_params(state, "model"), O.split_params(state, "model_fine")
        rays, gt = _bench_rays(O, n_rays, "cpu")

        def once():
            for v in state.values():
                v.grad = None
            ret = O.render(C, Fn, rays, torch.tensor([2.0]), torch.tensor([6.0]))
            O.loss_fn(ret, gt)[0].backward()

        once()
        t0 = time.perf_counter()
        reps = 0
        while reps < 5 and (reps < 2 or time.perf_counter() - t0 < 20.0):
            once()
            reps += 1
        dt = (time.perf_counter() - t0) / reps
    finally:
        torch.set_num_threads(prev)
    return {"value": round(n_rays / dt, 2), "unit": "rays/s", "cores": threads, "cores_basis": basis,
            "host_cpus": os.cpu_count(), "kind": "port", "cpu_model": cpu_model(), "torch": torch.__version__,
            "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS"),
            "sample": f"config 1: {n_rays}-ray forward+backward render (64+128 samples, perturb 0, seed-0 weights), "
                      f"mean of {reps} after 1 warm-up, oracle restatement on torch CPU"}


def eager_gpu_baseline(device, n_rays, dtype, reps=11):
    """Baseline leg: the reference's per-step op graph (the oracle restatement of
    volume_renderer.render + network.Network + MSE + clip_grad_value_(40) + Adam with one group
    per tensor) run eagerly by PyTorch-ROCm on this GPU -- the "reference per-step PyTorch-ROCm
    rays/s" of the north_star -- with the SAME MLP dtype (bf16 = torch.autocast) and perturb=1,
    n_rays per step."""
    from oracle import nerf_oracle as O
    prm = {k: v.to(device).clone().requires_grad_(True) for k, v in O.seeded_network_state(0).items()}
    C, Fn = O.split_params(prm, "model"), O.split_params(prm, "model_fine")
    opt = torch.optim.Adam([{"params": [p]} for p in prm.values()], lr=5e-4, eps=1e-8)
    rays, gt = _bench_rays(O, n_rays, device)
    near, far = torch.tensor([2.0], device=device), torch.tensor([6.0], device=device)

    def step():
        opt.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=dtype == "bf16"):
            ret = O.render(C, Fn, rays, near, far, perturb=True)
        O.loss_fn({k: v.float() for k, v in ret.items()}, gt)[0].backward()
        torch.nn.utils.clip_grad_value_(list(prm.values()), 40.0)
        opt.step()

    step()
    times = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        step()
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    times.sort()
    dt = times[len(times) // 2]
    return {"value": round(n_rays / dt, 1), "unit": "rays/s", "kind": "pytorch_rocm_eager", "dtype": dtype,
            "ms_per_step": round(dt * 1e3, 2), "ms_per_step_min_max": [round(times[0] * 1e3, 2), round(times[-1] * 1e3, 2)],
            "sample": f"{n_rays}-ray full train step (perturb 1, clip 40 + torch.optim.Adam), median of {reps} "
                      f"after 1 warm-up, reference op graph (oracle restatement) on PyTorch-ROCm {torch.__version__}"}


def main():
    args = parse()
    want, err = check_world(args.gpus)
    if err is not None:
        log(err)
        sys.exit(2)
    if want > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(want, sys.argv[1:]))
    world, rank, device = setup_dist()
    others = [] if args.no_second else [d for d in ALL_DTYPES if d != args.dtype]
    lines = {}
    for dtype in [args.dtype] + others:
        log(f"training {dtype}: {args.warmup} warmup + {args.steps} timed steps")
        value, ms_step, roofline, kt, train_stream, (cfg, net, ds), dist_info = \
            measure_training(args, world, rank, device, dtype)
        render_s, render_stream, grid = None, None, None
        log(f"{dtype}: {value:.0f} rays/s")
        if not args.no_render:
            render_s, render_stream = render_frame_time(cfg, net, ds, device, world)
            log(f"{dtype}: render {render_s:.3f} s/frame")
            grid = grid_times(cfg, net, ds, device)
            log(f"{dtype}: grid {grid}")
        lines[dtype] = {
            "value": round(value, 1), "ms_per_step": round(ms_step, 3), "dtype": dtype,
            "vs_baseline": None, "baseline": None, "roofline": roofline, "kernels": kt,
            "stream_kernels": {"train_step": train_stream, "render_800x800": render_stream},
            "render_s_per_frame": None if render_s is None else round(render_s, 4),
            "render_parallelism": f"tile-split over {world} GPU(s)", "occupancy_grid": grid,
            "distributed": dist_info,
        }
        del net, ds
        torch.cuda.empty_cache()
    # ONE denominator for every tier: the reference's own fp32 step run eagerly by PyTorch-ROCm,
    # measured once per run after all tiers (median of 21 steps, min / max reported).  Eager bf16
    # (autocast) is slower on this stack (host-bound: each bf16 aten::mm in backward costs ~0.55 ms
    # of host time, tools/eager_probe.py), so the fp32 step is the stronger baseline for the bf16
    # tier too; its autocast time is kept beside it for reference.
    if rank == 0 and world == 1 and not args.no_eager_baseline:
        eager = eager_gpu_baseline(device, args.rays, "fp32", reps=21)
        log(f"eager PyTorch-ROCm fp32 {eager['value']} rays/s ({eager['ms_per_step_min_max']} ms min/max)")
        for d in lines:
            lines[d]["baseline"] = eager
            lines[d]["vs_baseline"] = round(lines[d]["value"] / world / eager["value"], 2)
        if "bf16" in lines:
            eb = eager_gpu_baseline(device, args.rays, "bf16", reps=5)
            lines["bf16"]["eager_bf16_autocast"] = {k: eb[k] for k in ("value", "ms_per_step", "ms_per_step_min_max")}
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.cpu_rays)
        log(f"cpu baseline {cpu['value']} rays/s")

    if rank == 0:
        head = lines[args.dtype]
        line = {
            "metric": METRIC, "value": head["value"], "unit": "rays/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": head["ms_per_step"], "higher_is_better": True,
            "scaling": "weak", "vs_baseline": head["vs_baseline"], "dtype": args.dtype,
            "data": "synthetic (100 spherical 800x800 views, random rgb; seed-0 reference init)",
            "config": {"workload": "lego NeRF train step: coarse 64 + fine 128 samples/ray, 4096 rays/GPU, "
                                   "MSE(c)+MSE(f), clip 40 + Adam (BASELINE config 3)",
                       "rays_per_gpu": args.rays, "global_batch_rays": args.rays * world,
                       "samples_per_ray": 64 + 192, "parallelism": f"dp{world}"},
            "roofline": head["roofline"],
            "cpu_baseline": cpu,
        }
        line.update({k: v for k, v in head.items() if k not in line and k not in ("value", "dtype")})
        # north_star "800x800 test view rendered in < 0.5 s on the node", per MLP dtype: the
        # hierarchical render (volume_renderer.render, 64 + 128 samples) and render_accelerated
        # (the grid march, the reference's own fast path once occupancy_grid.pt exists) of the
        # trained fixture's held-out view, both split over the N GPUs of this run
        line["render_800x800_s"] = {
            d: None if lines[d]["occupancy_grid"] is None else {
                "hierarchical": lines[d]["occupancy_grid"]["trained"]["hierarchical_render_s"],
                "accelerated": lines[d]["occupancy_grid"]["trained"]["march_s_per_frame"], "gpus": world}
            for d in lines}
        line["baseline"] = head["baseline"]
        for d in others:
            line[f"{d}_line"] = dict(lines[d], label=f"opt-in {d} MLP (same workload)", metric=METRIC, unit="rays/s")
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
