"""The north_star's speed target, measured: the reference's per-step PyTorch-ROCm rays/s (its
op graph run eagerly on the MI355X -- the oracle restatement of volume_renderer.render +
network.Network + MSE + clip_grad_value_(40) + torch.optim.Adam, BASELINE.md section 4, the
same leg bench.py reports as `baseline`) against this build's training step on the same
4096-ray batch, at the SAME MLP precision and perturb (1) on both sides.

  * fp32 (the reference's precision): this build's step vs the eager fp32 step.  The fp32
    MFMA ceiling bounds this ratio at ~17x (176k rays/s at 157.3 TFLOP/s); the
    test asserts >= 7x (measured 10.8-11.9x in round 2; the eager step is host-launch-bound and
    varies 10.4k-13.7k rays/s between GPU boxes).
  * bf16 (the north_star's ">= 50x at matched PSNR", test_gpu_trained / DESIGN.md 5): this
    build's bf16 step vs the faster of eager fp32 and eager bf16 autocast (autocast is
    host-bound and slower); asserts >= 40x as a regression floor that tolerates a fast host
    (measured 76x).

Run with -s to see the rates."""
import json
import os
import sys
import time

import pytest
import torch

pytestmark = pytest.mark.gpu

RAYS = 4096
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _time(fn, reps, warm=2):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def _build_rate(cuda, dtype):
    """bench.py's timed step: Trainer.train_step (render perturb 1 + MSE + backward + fused clip
    40 + Adam) on bench.py's 4096-ray batch."""
    sys.path.insert(0, ROOT)
    import bench
    from oracle import nerf_oracle as O
    from src.config import cfg
    from src.models import make_network
    from src.train.optimizer import make_optimizer
    from src.train.trainers.make_trainer import make_trainer
    from nerf_amd import ops
    rays, gt = bench._bench_rays(O, RAYS, cuda)
    saved = (cfg.task_arg.mlp_dtype, cfg.task_arg.perturb)
    cfg.task_arg.mlp_dtype, cfg.task_arg.perturb = dtype, 1
    try:
        torch.manual_seed(0)
        net = make_network(cfg)
        trainer = make_trainer(cfg, net)
        opt = make_optimizer(cfg, net)
        batch = {"rays": rays[None], "rgbs": gt[None], "near": ops.device_scalar(2.0, cuda),
                 "far": ops.device_scalar(6.0, cuda)}
        t = _time(lambda: trainer.train_step(batch, opt), 20, warm=5)
    finally:
        cfg.task_arg.mlp_dtype, cfg.task_arg.perturb = saved
    return RAYS / t


@pytest.mark.parametrize("dtype,floor", [("fp32", 7.0), ("bf16", 40.0)])
def test_speedup_vs_pytorch_rocm_eager(cuda, dtype, floor):
    sys.path.insert(0, ROOT)
    import bench
    os.environ.setdefault("NERF_AMD_NO_ARGV", "1")
    eager = bench.eager_gpu_baseline(cuda, RAYS, "fp32", reps=2)["value"]
    if dtype == "bf16":
        eager = max(eager, bench.eager_gpu_baseline(cuda, RAYS, "bf16", reps=2)["value"])
    ours = _build_rate(cuda, dtype)
    res = {"dtype": dtype, "rays": RAYS, "pytorch_rocm_eager_rays_per_s": eager, "build_rays_per_s": ours,
           "speedup": ours / eager}
    print("\nSPEEDUP " + json.dumps(res))
    assert res["speedup"] >= floor, res
