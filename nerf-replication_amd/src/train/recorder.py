"""Training log recorder (reference: src/train/recorder.py:49-134), console only: smoothed
loss stats, batch/data time and the step counter saved in checkpoints."""
from collections import defaultdict, deque

import torch


class SmoothedValue:
    def __init__(self, window_size=20):
        self.deque = deque(maxlen=window_size)
        self.total = 0.0
        self.count = 0

    def update(self, value):
        self.deque.append(value)
        self.count += 1
        self.total += value

    @property
    def median(self):
        d = sorted(self.deque)
        return d[len(d) // 2] if d else 0.0

    @property
    def avg(self):
        return sum(self.deque) / max(len(self.deque), 1)

    @property
    def global_avg(self):
        return self.total / max(self.count, 1)


class Recorder:
    def __init__(self, cfg=None):
        self.epoch = 0
        self.step = 0
        self.loss_stats = defaultdict(SmoothedValue)
        self.batch_time = SmoothedValue()
        self.data_time = SmoothedValue()

    def update_loss_stats(self, loss_dict):
        for k, v in loss_dict.items():
            self.loss_stats[k].update(float(v.detach()) if torch.is_tensor(v) else float(v))

    def record(self, prefix, step=-1, loss_stats=None, image_stats=None):
        pass

    def state_dict(self):
        return {"step": self.step}

    def load_state_dict(self, sd):
        self.step = sd["step"]

    def __str__(self):
        parts = [f"epoch: {self.epoch}", f"step: {self.step}"]
        parts += [f"{k}: {v.avg:.4f}" for k, v in self.loss_stats.items()]
        parts += [f"data: {self.data_time.avg:.4f}", f"batch: {self.batch_time.avg:.4f}"]
        return "  ".join(parts)


def make_recorder(cfg):
    return Recorder(cfg)
