"""The north_star's speed target, measured: the reference's per-step PyTorch-ROCm rays/s (its
op graph run eagerly on the MI355X -- the oracle restatement of volume_renderer.render +
network.Network) against this build's training step on the same
4096-ray batch.  Target: >= 50x (north_star).

The test prints both rates (run with -s to see them) and asserts a conservative 20x floor so
that a regression to an eager-like path cannot pass unnoticed; the measured ratio is
recorded in DESIGN.md / BASELINE.md.  The eager step is forward + backward only (no
optimizer), this build's step includes clip + Adam."""
import json
import os
import time

import pytest
import torch

pytestmark = pytest.mark.gpu

RAYS = 4096


def _rays(O, n, dev):
    pose = O.pose_spherical(30.0, -30.0, 4.0)
    o, d = O.get_rays(800, 800, O.focal_from_angle(800, 0.6911112070083618), pose)
    idx = torch.randint(0, 800 * 800, (n,), generator=torch.Generator().manual_seed(0))
    rays = torch.cat([o.reshape(-1, 3)[idx], d.reshape(-1, 3)[idx]], 1)
    gt = torch.rand(n, 3, generator=torch.Generator().manual_seed(1))
    return rays.to(dev), gt.to(dev)


def _time(fn, reps, warm=2):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def test_speedup_vs_pytorch_rocm_eager(cuda, seeded_state):
    from oracle import nerf_oracle as O
    os.environ.setdefault("NERF_AMD_NO_ARGV", "1")
    rays, gt = _rays(O, RAYS, cuda)
    near, far = torch.tensor([2.0], device=cuda), torch.tensor([6.0], device=cuda)

    # the reference's per-step op graph, eager PyTorch on ROCm (fp32, perturb 0)
    prm = {k: v.to(cuda).clone().requires_grad_(True) for k, v in seeded_state.items()}
    C, Fn = O.split_params(prm, "model"), O.split_params(prm, "model_fine")

    def eager():
        for v in prm.values():
            v.grad = None
        ret = O.render(C, Fn, rays, near, far)
        O.loss_fn(ret, gt)[0].backward()

    t_eager = _time(eager, 3)

    # this build: the training step of bench.py (bf16 MLP, perturb 1, clip + Adam)
    from src.config import cfg
    from src.models import make_network
    from src.train.optimizer import make_optimizer
    from src.train.trainers.make_trainer import make_trainer
    from nerf_amd import ops
    saved = cfg.task_arg.mlp_dtype
    cfg.task_arg.mlp_dtype = "bf16"
    torch.manual_seed(0)
    net = make_network(cfg)
    trainer = make_trainer(cfg, net)
    opt = make_optimizer(cfg, net)
    batch = {"rays": rays[None], "rgbs": gt[None], "near": ops.device_scalar(2.0, cuda),
             "far": ops.device_scalar(6.0, cuda)}
    t_ours = _time(lambda: trainer.train_step(batch, opt), 20, warm=5)
    cfg.task_arg.mlp_dtype = saved

    res = {"rays": RAYS, "pytorch_rocm_eager_rays_per_s": RAYS / t_eager, "build_rays_per_s": RAYS / t_ours,
           "speedup": t_eager / t_ours}
    print("\nSPEEDUP " + json.dumps(res))
    assert res["speedup"] > 20.0, res
