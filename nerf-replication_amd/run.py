"""Evaluation / benchmark entry point (reference: run.py:1-91).

    python run.py --type evaluate --cfg_file configs/nerf/lego.yaml   # grid-accelerated render + PSNR/SSIM
    python run.py --type network  --cfg_file configs/nerf/lego.yaml   # hierarchical render timing
    python run.py --type dataset  --cfg_file configs/nerf/lego.yaml
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 run.py --type evaluate ...

Under torch.distributed.run every image's rays are dealt to the GPUs in interleaved 256-ray blocks
and gathered after rendering (src/utils/dist_render.py); rank 0 evaluates and prints.
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from src.config import cfg, args  # noqa: E402
from src.config.config import apply_gpus  # noqa: E402


def run_dataset():
    from src.datasets import make_data_loader
    for _ in make_data_loader(cfg, is_train=False):
        pass


def _init_dist():
    """RCCL process group when launched by torch.distributed.run; returns the rank."""
    import torch.distributed as dist
    if int(os.environ.get("WORLD_SIZE", "1")) > 1 and not dist.is_initialized():
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", init_method="env://", device_id=torch.device("cuda", local))
    return dist.get_rank() if dist.is_initialized() else 0


def run_network():
    from src.datasets import make_data_loader
    from src.models import make_network
    from src.models.nerf.renderer import make_renderer
    from src.utils.net_utils import load_network

    from src.utils.dist_render import render_distributed

    rank = _init_dist()
    network = make_network(cfg).cuda()
    load_network(network, cfg.trained_model_dir, epoch=cfg.test.epoch)
    network.eval()
    loader = make_data_loader(cfg, is_train=False)
    renderer = make_renderer(cfg, network)
    total = 0.0
    for batch in loader:
        with torch.no_grad():
            torch.cuda.synchronize()
            t0 = time.time()
            render_distributed(renderer, batch)
            torch.cuda.synchronize()
            total += time.time() - t0
    if rank == 0:
        print(total / len(loader))


def run_evaluate():
    from src.datasets import make_data_loader
    from src.evaluators import make_evaluator
    from src.models import make_network
    from src.models.nerf.renderer import make_renderer
    from src.utils.net_utils import load_network

    from src.utils.dist_render import render_distributed

    rank = _init_dist()
    if rank == 0:
        print(f"trained_model_dir: {cfg.trained_model_dir}")
    network = make_network(cfg).cuda()
    load_network(network, cfg.trained_model_dir, resume=cfg.resume, epoch=cfg.test.epoch)
    network.eval()
    loader = make_data_loader(cfg, is_train=False)
    evaluator = make_evaluator(cfg)
    renderer = make_renderer(cfg, network)
    net_time = []
    if cfg.task_arg.get("accelerated_renderer", False):
        name = os.path.splitext(os.path.basename(args.cfg_file))[0]
        renderer.load_occupancy_grid(os.path.join("logs", name, "occupancy_grid.pt"))
    for batch in loader:
        with torch.no_grad():
            torch.cuda.synchronize()
            t0 = time.time()
            output = render_distributed(renderer, batch, accelerated=True)
            torch.cuda.synchronize()
            net_time.append(time.time() - t0)
        if rank == 0:
            evaluator.evaluate(output, batch)
    if rank == 0:
        evaluator.summarize()
        t = np.mean(net_time[1:]) if len(net_time) > 1 else np.mean(net_time)
        print("net_time: ", t)
        print("fps: ", 1.0 / t)


if __name__ == "__main__":
    apply_gpus(cfg)
    globals()["run_" + args.type]()
