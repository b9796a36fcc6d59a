"""The real data-parallel training step on two ranks (BASELINE config 5's path; reference
src/train/trainers/trainer.py:15-22 DDP construction, :53-62 backward + all-reduce + step).

Two processes share cuda:0 over gloo (RCCL needs one GPU per rank; the collective calls are
the same ``torch.distributed`` ones).  Each rank draws its own 4096-ray batch (rank-distinct
Philox streams) of a synthetic scene, loads the trained fixture weights, and runs the
production step: the fused HIP forward / backward with direct dW into FusedAdam's flat .grad,
the per-net GradBuckets all-reduces fired from inside backward, the fused clip 40 + Adam.
Every rank also computes, with the buckets suspended, the local gradient of EVERY rank's
batch.  Asserted:
  * the bucket-reduced flat gradient equals (sum of the single-process gradients) / world
    bit for bit (the dW is deterministic, and a two-term fp32 sum is order-free);
  * exactly one bucket per net fired from inside backward;
  * after Adam the parameters are bit-identical on both ranks;
  * the prefetching step (the next batch's rays and stratified samples enqueued before the
    step waits for the all-reduce) trains exactly like the plain one (test_prefetch_*).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup(dtype, seed_images=7):
    from src.config import cfg
    from src.datasets.nerf.blender import Dataset
    from src.datasets.nerf.synthetic import view_poses
    from src.models.nerf.network import Network
    from src.train.optimizer import make_optimizer
    from src.train.trainers.make_trainer import make_trainer
    from src.utils.camera import focal_for
    dev = torch.device("cuda", 0)
    cfg.task_arg.perturb = 0
    cfg.task_arg.mlp_dtype = dtype
    cfg.task_arg.train_rays = 4096
    z = np.load(os.path.join(HERE, "golden", "trained_v2.npz"), allow_pickle=False)
    torch.manual_seed(0)
    net = Network()
    net.load_state_dict({k: torch.from_numpy(z[k]) for k in z.files}, strict=True)
    net = net.to(dev)
    trainer = make_trainer(cfg, net)
    opt = make_optimizer(cfg, net)
    g = torch.Generator().manual_seed(seed_images)
    images = torch.rand(4, 128, 128, 3, generator=g).to(dev)
    ds = Dataset.from_arrays(images, view_poses(4, seed=3).to(dev), focal_for(128))
    return cfg, net, trainer, opt, ds, dev


def _batch(rays, rgbs, dev):
    from nerf_amd import ops
    return {"rays": rays[None], "rgbs": rgbs[None], "near": ops.device_scalar(2.0, dev),
            "far": ops.device_scalar(6.0, dev)}


def _worker(rank, world, port, dtype, q, dw_stream=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), NERF_AMD_NO_ARGV="1", NERF_DW_STREAM="1" if dw_stream else "0")
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "nerf-replication_amd")]
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        cfg, net, trainer, opt, ds, dev = _setup(dtype)
        rays, rgbs = ds.sample_batch()
        batch = trainer.prepare(_batch(rays, rgbs, dev))
        # every rank's batch, gathered (host tensors) so that each rank can recompute them all
        all_rays = [torch.empty_like(rays.cpu()) for _ in range(world)]
        all_rgbs = [torch.empty_like(rgbs.cpu()) for _ in range(world)]
        dist.all_gather(all_rays, rays.cpu())
        dist.all_gather(all_rgbs, rgbs.cpu())
        distinct = not torch.equal(all_rays[0], all_rays[1])
        local = []
        with trainer.buckets.suspended():  # single-process gradients: no collective fires
            for r in range(world):
                trainer.forward_backward(_batch(all_rays[r].to(dev), all_rgbs[r].to(dev), dev), opt)
                local.append(opt.flat_grad.clone())
        # the data-parallel step on this rank's own batch
        trainer.forward_backward(batch, opt)
        fired = len(trainer.buckets.works)
        trainer.buckets.finish(opt)
        dp = opt.flat_grad.clone()
        expect = local[0].clone()
        for r in range(1, world):
            expect += local[r]
        expect.mul_(1.0 / world)
        exact = bool(torch.equal(dp, expect))
        maxdiff = float((dp - expect).abs().max())
        scale = float(expect.abs().max())
        opt.clip_value = trainer.clip_value
        opt.step()
        torch.cuda.synchronize()
        params = opt.flat_param.cpu()
        all_params = [torch.empty_like(params) for _ in range(world)]
        dist.all_gather(all_params, params)
        same_params = all(torch.equal(all_params[0], p) for p in all_params[1:])
        q.put((rank, exact, maxdiff, scale, fired, same_params, distinct, None))
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001 - reported to the parent
        import traceback
        q.put((rank, False, None, None, None, False, False, traceback.format_exc()))


@pytest.mark.parametrize("dtype,dw_stream", [("fp32", False), ("bf16", False), ("bf16", True)])
def test_two_rank_dp_step_matches_single_process(dtype, dw_stream):
    """dw_stream: the opt-in NERF_DW_STREAM=1 schedule (every dW on a second stream; a bucket's
    all-reduce is enqueued behind it) reduces the same gradient bit for bit."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, dtype, q, dw_stream)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        res = [q.get(timeout=240) for _ in procs]
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for rank, exact, maxdiff, scale, fired, same, distinct, err in res:
        assert err is None, err
        assert distinct  # each rank drew its own rays
        assert fired == 2  # one bucket per net, started from inside backward
        assert exact, (rank, maxdiff, scale)  # bucketed DP gradient == mean of local gradients, bitwise
        assert same  # identical parameters on every rank after the step
    for p in procs:
        assert p.exitcode == 0


def test_prefetch_step_trains_like_the_plain_step(cuda):
    """Trainer.train_step(prefetch=...) enqueues the next batch's raygen + stratified sampling
    before the optimizer update.  With perturb 1 (training's default, where the stratified
    jitter and the importance-sample uniforms come from the renderer's Philox stream) and the
    same ray stream it must give the same losses and parameters, bit for bit, as the original
    step with no preparation at all (to_cuda -> forward_backward -> apply): prefetching keeps
    the per-step random stream."""
    runs = []
    for use_prefetch in (False, True):
        cfg, net, trainer, opt, ds, dev = _setup("fp32")
        cfg.task_arg.perturb = 1
        losses = []

        def nxt():
            r, c = ds.sample_batch()
            return _batch(r, c, dev)
        try:
            for step in range(3):
                if use_prefetch:
                    batch = trainer.prefetched or trainer.prepare(nxt())
                    _, loss, _ = trainer.train_step(batch, opt, prefetch=nxt)
                    assert trainer.prefetched is not None and "_stratified0" in trainer.prefetched
                else:
                    batch = trainer.to_cuda(nxt())
                    assert "_stratified0" not in batch
                    _, loss, _ = trainer.forward_backward(batch, opt)
                    trainer.apply(opt)
                losses.append(float(loss))
        finally:
            cfg.task_arg.perturb = 0
        torch.cuda.synchronize()
        runs.append((losses, opt.flat_param.detach().cpu().clone()))
    assert runs[0][0] == runs[1][0]
    assert torch.equal(runs[0][1], runs[1][1])
