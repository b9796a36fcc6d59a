"""Drop-in ``loss_module`` (reference: src/train/trainers/nerf.py:6-50).

NetworkWrapper(net, train_loader).forward(batch) -> (ret, loss, {loss_c, loss_f, total_loss})
with loss = MSE(rgb_map_c, gt) + MSE(rgb_map_f, gt).  Like the reference it builds its
Renderer from this module path directly (nerf.py:3,10), so the drop-in renderer must live
at src.models.nerf.renderer.volume_renderer.
"""
import torch.nn as nn

from nerf_amd import ops

from src.config import cfg
from src.models.nerf.renderer.volume_renderer import Renderer


class NetworkWrapper(nn.Module):
    def __init__(self, net, train_loader=None):
        super().__init__()
        self.net = net
        self.renderer = Renderer(self.net)
        self.loss_fn = nn.MSELoss()

    def forward(self, batch):
        ret = self.renderer.render(batch)
        gt = batch["rgbs"].reshape(-1, 3) if batch["rgbs"].dim() == 3 else batch["rgbs"]
        if "rgb_map_f" in ret and ret["rgb_map_c"].is_cuda and cfg.task_arg.get("fuse_mse", True):
            # both MSEs and their sum in one launch, the backward in one (ops.mse_pair)
            loss_c, loss_f, total = ops.mse_pair(ret["rgb_map_c"], ret["rgb_map_f"], gt)
            return ret, total, {"loss_c": loss_c, "loss_f": loss_f, "total_loss": total}
        loss_c = self.loss_fn(ret["rgb_map_c"], gt)
        stats = {"loss_c": loss_c}
        if "rgb_map_f" in ret:
            loss_f = self.loss_fn(ret["rgb_map_f"], gt)
            total = loss_c + loss_f
            stats["loss_f"] = loss_f
        else:
            total = loss_c
        stats["total_loss"] = total
        return ret, total, stats
