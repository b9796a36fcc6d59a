"""make_trainer (reference: src/train/trainers/make_trainer.py:5-14)."""
from src.models.make_network import load_source

from .trainer import Trainer


def make_trainer(cfg, network, train_loader=None):
    wrapper = load_source(cfg.loss_module, cfg.loss_path).NetworkWrapper(network, train_loader)
    return Trainer(wrapper)
