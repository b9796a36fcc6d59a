"""Occupancy-grid bake / "grid update" (reference: occupancy_grid.py:15-80).

    python occupancy_grid.py --cfg_file configs/nerf/lego.yaml

sigma = relu(coarse raw[3]) at the 8 corners of each of res^3 voxels, occupied if any
corner has sigma > threshold; saved as a bool [res,res,res] tensor to
logs/<cfg name>/occupancy_grid.pt.  On the GPU the corners shared by neighbouring voxels
are evaluated once ((res+1)^3 points instead of 8 res^3, bit-identical because the lego
corner coordinates are exact in fp32) by the density-only fused MLP.  Under
``torch.distributed.run`` each rank bakes one x-slab and the grid is all-gathered.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from src.config import cfg, args  # noqa: E402
from src.config.config import apply_gpus  # noqa: E402


def save_grid(grid: torch.Tensor, path: str) -> None:
    """occupancy_grid.py:72-78: torch.save of the bool [res,res,res] grid on the CPU."""
    if grid.dtype != torch.bool or grid.dim() != 3:
        raise ValueError(f"occupancy grid must be a 3-D bool tensor, got {grid.dtype} {tuple(grid.shape)}")
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    torch.save(grid.cpu(), path)


def main():
    from nerf_amd import ops
    from src.models import make_network
    from src.utils.dist_render import bake_distributed
    from src.utils.net_utils import load_network

    if int(os.environ.get("WORLD_SIZE", "1")) > 1 and not dist.is_initialized():
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        cfg.local_rank = local
        dist.init_process_group("nccl", init_method="env://", device_id=torch.device("cuda", local))
    else:
        apply_gpus(cfg)
    network = make_network(cfg).cuda()
    load_network(network, cfg.trained_model_dir, epoch=cfg.test.epoch)
    network.eval()
    res = int(cfg.task_arg.occupancy_grid_res)
    thr = float(cfg.task_arg.occupancy_grid_threshold)
    b = cfg.train_dataset.scene_bbox
    bbox = (tuple(map(float, b[0])), tuple(map(float, b[1])))
    with torch.no_grad():  # one voxel slab per rank under torchrun, all-gathered
        grid = bake_distributed(lambda slab: ops.bake(network.model.packer(), res, thr, bbox,
                                                      dtype=network.mlp_dtype, slab=slab), res)
    name = os.path.splitext(os.path.basename(args.cfg_file))[0]
    path = os.path.join("logs", name, "occupancy_grid.pt")
    if not dist.is_initialized() or dist.get_rank() == 0:
        print(f"Saving occupancy grid to: {path}")
        save_grid(grid, path)
    if dist.is_initialized():
        dist.destroy_process_group()
    print("Done.")


if __name__ == "__main__":
    main()
