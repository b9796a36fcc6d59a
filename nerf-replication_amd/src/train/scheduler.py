"""LR schedulers (reference: src/train/scheduler.py:7-27, src/utils/optimizer/lr_scheduler.py:68-79).

ExponentialLR: lr = base_lr * gamma ** (epoch / decay_epochs), stepped once per epoch.
"""
from collections import Counter

import torch


class ExponentialLR(torch.optim.lr_scheduler.LRScheduler):
    def __init__(self, optimizer, decay_epochs, gamma=0.1, last_epoch=-1):
        self.decay_epochs = decay_epochs
        self.gamma = gamma
        super().__init__(optimizer, last_epoch)

    def get_lr(self):
        return [base * self.gamma ** (self.last_epoch / self.decay_epochs) for base in self.base_lrs]


class MultiStepLR(torch.optim.lr_scheduler.LRScheduler):
    def __init__(self, optimizer, milestones, gamma=0.1, last_epoch=-1):
        self.milestones = Counter(milestones)
        self.gamma = gamma
        super().__init__(optimizer, last_epoch)

    def get_lr(self):
        if self.last_epoch not in self.milestones:
            return [g["lr"] for g in self.optimizer.param_groups]
        return [g["lr"] * self.gamma ** self.milestones[self.last_epoch] for g in self.optimizer.param_groups]


def make_lr_scheduler(cfg, optimizer):
    s = cfg.train.scheduler
    if s.type == "multi_step":
        return MultiStepLR(optimizer, milestones=s.milestones, gamma=s.gamma)
    if s.type == "exponential":
        return ExponentialLR(optimizer, decay_epochs=s.decay_epochs, gamma=s.gamma)
    raise NotImplementedError(s.type)


def set_lr_scheduler(cfg, scheduler):
    s = cfg.train.scheduler
    if s.type == "multi_step":
        scheduler.milestones = Counter(s.milestones)
    elif s.type == "exponential":
        scheduler.decay_epochs = s.decay_epochs
    scheduler.gamma = s.gamma
