"""Training entry point (reference: train.py:1-135).

    python train.py --cfg_file configs/nerf/lego.yaml [key value ...]
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 train.py \
        --cfg_file configs/nerf/lego.yaml distributed True

One process per GPU; with ``distributed True`` the process group is RCCL ("nccl") and
gradients are averaged once per step (src/train/trainers/trainer.py).  The reference's
always-on autograd anomaly mode (train.py:23, ~20 % cost) is opt-in here
(``detect_anomaly True``).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from src.config import cfg, args  # noqa: E402
from src.config.config import apply_gpus  # noqa: E402


def train(cfg, network):
    from src.datasets import make_data_loader
    from src.evaluators import make_evaluator
    from src.train import make_lr_scheduler, make_optimizer, make_recorder, make_trainer, set_lr_scheduler
    from src.utils.net_utils import load_model, load_pretrain, save_model, save_trained_config

    if cfg.local_rank == 0:
        save_trained_config(cfg)
    train_loader = make_data_loader(cfg, is_train=True, is_distributed=cfg.distributed, max_iter=cfg.ep_iter)
    val_loader = make_data_loader(cfg, is_train=False) if cfg.local_rank == 0 else None
    trainer = make_trainer(cfg, network, train_loader)
    optimizer = make_optimizer(cfg, network)
    scheduler = make_lr_scheduler(cfg, optimizer)
    recorder = make_recorder(cfg)
    evaluator = make_evaluator(cfg)
    begin_epoch = load_model(network, optimizer, scheduler, recorder, cfg.trained_model_dir, resume=cfg.resume)
    if begin_epoch == 0 and cfg.pretrain != "":
        load_pretrain(network, cfg.pretrain)
    set_lr_scheduler(cfg, scheduler)
    for epoch in range(begin_epoch, cfg.train.epoch):
        recorder.epoch = epoch
        trainer.train(epoch, train_loader, optimizer, recorder)
        scheduler.step()
        if (epoch + 1) % cfg.save_ep == 0 and cfg.local_rank == 0:
            save_model(network, optimizer, scheduler, recorder, cfg.trained_model_dir, epoch)
        if (epoch + 1) % cfg.save_latest_ep == 0 and cfg.local_rank == 0:
            save_model(network, optimizer, scheduler, recorder, cfg.trained_model_dir, epoch, last=True)
        if (epoch + 1) % cfg.eval_ep == 0 and cfg.local_rank == 0:
            trainer.val(epoch, val_loader, evaluator, recorder)
    return network


def test(cfg, network):
    from src.datasets import make_data_loader
    from src.evaluators import make_evaluator
    from src.train import make_trainer
    from src.utils.net_utils import load_network

    trainer = make_trainer(cfg, network)
    val_loader = make_data_loader(cfg, is_train=False)
    evaluator = make_evaluator(cfg)
    epoch = load_network(network, cfg.trained_model_dir, resume=cfg.resume, epoch=cfg.test.epoch)
    trainer.val(epoch, val_loader, evaluator)


def main():
    if cfg.get("detect_anomaly", False):
        torch.autograd.set_detect_anomaly(True)
    if cfg.fix_random:
        torch.manual_seed(0)
    if cfg.distributed:
        cfg.local_rank = int(os.environ.get("LOCAL_RANK", os.environ["RANK"])) % torch.cuda.device_count()
        torch.cuda.set_device(cfg.local_rank)
        dist.init_process_group(backend="nccl", init_method="env://")
        dist.barrier()
    else:
        apply_gpus(cfg)
    from src.models import make_network
    network = make_network(cfg)
    if args.test:
        test(cfg, network)
    else:
        train(cfg, network)
    if cfg.distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
