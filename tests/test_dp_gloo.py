"""CPU, world_size 2 (gloo): the data-parallel step's collective semantics.

Each rank holds a flat gradient (FusedAdam.flat_grad's role); allreduce_grads must leave
every rank with the mean, and broadcast_params must give every rank rank-0's weights
(DistributedDataParallel's construction broadcast, trainer.py:15-22 of the reference).
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      NERF_AMD_NO_ARGV="1")
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "nerf-replication_amd")]
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from src.train.trainers.trainer import allreduce_grads, broadcast_params

    class Opt:
        pass

    opt = Opt()
    opt.flat_grad = torch.arange(10, dtype=torch.float32) * (rank + 1)
    allreduce_grads(opt)
    lin = torch.nn.Linear(4, 3)
    torch.nn.init.constant_(lin.weight, float(rank))
    broadcast_params(lin)
    q.put((rank, opt.flat_grad.tolist(), float(lin.weight.sum())))
    dist.destroy_process_group()


def test_two_rank_gradient_average_and_broadcast():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    expect = [1.5 * i for i in range(10)]
    for rank, grad, wsum in res:
        assert grad == pytest.approx(expect)
        assert wsum == 0.0  # rank 0's weights everywhere
