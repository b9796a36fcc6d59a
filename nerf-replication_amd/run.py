"""Evaluation / benchmark entry point (reference: run.py:1-91).

    python run.py --type evaluate --cfg_file configs/nerf/lego.yaml   # grid-accelerated render + PSNR/SSIM
    python run.py --type network  --cfg_file configs/nerf/lego.yaml   # hierarchical render timing
    python run.py --type dataset  --cfg_file configs/nerf/lego.yaml
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


def run_network():
    from src.datasets import make_data_loader
    from src.models import make_network
    from src.models.nerf.renderer import make_renderer
    from src.utils.net_utils import load_network

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
            renderer.render(batch)
            torch.cuda.synchronize()
            total += time.time() - t0
    print(total / len(loader))


def run_evaluate():
    from src.datasets import make_data_loader
    from src.evaluators import make_evaluator
    from src.models import make_network
    from src.models.nerf.renderer import make_renderer
    from src.utils.net_utils import load_network

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
            output = renderer.render_accelerated(batch)
            torch.cuda.synchronize()
            net_time.append(time.time() - t0)
        evaluator.evaluate(output, batch)
    evaluator.summarize()
    t = np.mean(net_time[1:]) if len(net_time) > 1 else np.mean(net_time)
    print("net_time: ", t)
    print("fps: ", 1.0 / t)


if __name__ == "__main__":
    apply_gpus(cfg)
    globals()["run_" + args.type]()
