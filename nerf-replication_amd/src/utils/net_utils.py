"""Checkpoint I/O (reference: src/utils/net_utils.py:288-379, 418-426).

``latest.pth`` / ``{epoch}.pth`` = {"net", "optim", "scheduler", "recorder", "epoch"}; at
most 5 numbered files are kept.  Loads use ``weights_only=True`` (no unpickling of code) and
``map_location="cpu"`` (the reference's load_network needs a GPU for GPU-saved files).
"""
import os
import sys

import torch


def _pths(model_dir):
    return [int(p.split(".")[0]) for p in os.listdir(model_dir) if p != "latest.pth" and p.endswith(".pth")]


def _resolve(model_dir, epoch):
    pths = _pths(model_dir)
    if len(pths) == 0 and "latest.pth" not in os.listdir(model_dir):
        return None
    if epoch == -1:
        pth = "latest" if "latest.pth" in os.listdir(model_dir) else max(pths)
    else:
        pth = epoch
    return os.path.join(model_dir, f"{pth}.pth")


def load_model(net, optim, scheduler, recorder, model_dir, resume=True, epoch=-1):
    if not resume or not os.path.exists(model_dir):
        return 0
    path = _resolve(model_dir, epoch)
    if path is None:
        return 0
    print(f"load model: {path}")
    ck = torch.load(path, map_location="cpu", weights_only=True)
    net.load_state_dict(ck["net"])
    if "optim" in ck:
        optim.load_state_dict(ck["optim"])
        scheduler.load_state_dict(ck["scheduler"])
        recorder.load_state_dict(ck["recorder"])
        return ck["epoch"] + 1
    return 0


def save_model(net, optim, scheduler, recorder, model_dir, epoch, last=False):
    os.makedirs(model_dir, exist_ok=True)
    model = {"net": net.state_dict(), "optim": optim.state_dict(), "scheduler": scheduler.state_dict(),
             "recorder": recorder.state_dict(), "epoch": epoch}
    torch.save(model, os.path.join(model_dir, "latest.pth" if last else f"{epoch}.pth"))
    pths = _pths(model_dir)
    if len(pths) > 5:
        os.remove(os.path.join(model_dir, f"{min(pths)}.pth"))


def load_network(net, model_dir, resume=True, epoch=-1, strict=True):
    if not resume:
        return 0
    if not os.path.exists(model_dir):
        print("pretrained model does not exist")
        return 0
    path = _resolve(model_dir, epoch) if os.path.isdir(model_dir) else model_dir
    if path is None:
        return 0
    print(f"load model: {path}")
    ck = torch.load(path, map_location="cpu", weights_only=True)
    net.load_state_dict(ck["net"], strict=strict)
    return ck["epoch"] + 1 if "epoch" in ck else 0


def save_trained_config(cfg):
    os.makedirs(cfg.trained_config_dir, exist_ok=True)
    with open(os.path.join(cfg.trained_config_dir, "train_cmd.txt"), "w") as f:
        f.write(" ".join(sys.argv))
    with open(os.path.join(cfg.trained_config_dir, "train_config.yaml"), "w") as f:
        f.write(cfg.dump())


def load_pretrain(net, model_dir):
    return load_network(net, model_dir)
