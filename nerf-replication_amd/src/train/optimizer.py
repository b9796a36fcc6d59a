"""make_optimizer (reference: src/train/optimizer.py:8-28) with a fused gfx950 Adam.

``FusedAdam`` is a torch.optim.Optimizer with torch.optim.Adam's param-group and
state_dict format (one group per tensor, state {step, exp_avg, exp_avg_sq}), so a
reference ``latest.pth["optim"]`` loads and the saved state reloads into torch.optim.Adam.
All parameters, gradients and both moments live in four flat fp32 buffers (params /
.grad / state tensors are views into them): one ``nerf_adam_step`` launch per step (with
the trainer's clip_grad_value_(40) fused in) replaces ~10 ATen kernels per tensor, and the
data-parallel gradient all-reduce is a single RCCL call on ``flat_grad``.
"""
import torch

from nerf_amd import ops


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, clip_value=0.0):
        defaults = dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay, amsgrad=False,
                        maximize=False, foreach=None, capturable=False, differentiable=False, fused=None)
        super().__init__(params, defaults)
        for g in self.param_groups:
            if g["weight_decay"] != 0:
                raise NotImplementedError("FusedAdam: weight_decay != 0 is not on the reference path")
        self.clip_value = float(clip_value)
        plist = self._plist()
        dev = plist[0].device
        total = sum(p.numel() for p in plist)
        self.flat_param = torch.empty(total, device=dev, dtype=torch.float32)
        self.flat_grad = torch.zeros(total, device=dev, dtype=torch.float32)
        self.flat_m = torch.zeros(total, device=dev, dtype=torch.float32)
        self.flat_v = torch.zeros(total, device=dev, dtype=torch.float32)
        self._ranges = []
        off = 0
        with torch.no_grad():
            for p in plist:
                if p.dtype != torch.float32 or p.device != dev:
                    raise TypeError("FusedAdam: parameters must be float32 on one device")
                n = p.numel()
                self.flat_param[off:off + n].copy_(p.detach().reshape(-1))
                p.data = self.flat_param[off:off + n].view_as(p)
                p.grad = self.flat_grad[off:off + n].view_as(p)
                self._ranges.append((off, n))
                st = self.state[p]
                st["step"] = torch.tensor(0.0)
                st["exp_avg"] = self.flat_m[off:off + n].view_as(p)
                st["exp_avg_sq"] = self.flat_v[off:off + n].view_as(p)
                off += n
        self._step = 0

    def _plist(self):
        return [p for g in self.param_groups for p in g["params"]]

    def _rebind(self):
        """Re-point .grad at the flat buffer (after someone set_to_none'd it)."""
        for p, (off, n) in zip(self._plist(), self._ranges):
            if p.grad is None or p.grad.data_ptr() != self.flat_grad[off:off + n].data_ptr():
                if p.grad is not None:
                    self.flat_grad[off:off + n].copy_(p.grad.reshape(-1))
                p.grad = self.flat_grad[off:off + n].view_as(p)

    def zero_grad(self, set_to_none: bool = True):
        self.flat_grad.zero_()
        self._rebind()

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        self._rebind()
        self._step += 1
        # one launch per run of consecutive parameters sharing (lr, betas, eps)
        runs = []
        idx = 0
        for g in self.param_groups:
            key = (float(g["lr"]), tuple(g["betas"]), float(g["eps"]))
            for _ in g["params"]:
                off, n = self._ranges[idx]
                if runs and runs[-1][0] == key and runs[-1][1] + runs[-1][2] == off:
                    runs[-1][2] += n
                else:
                    runs.append([key, off, n])
                idx += 1
        for (lr, betas, eps), off, n in runs:
            sl = slice(off, off + n)
            ops.adam_step(self.flat_param[sl], self.flat_grad[sl], self.flat_m[sl], self.flat_v[sl], lr, self._step,
                          betas, eps, self.clip_value)
        ops.params_updated()
        return loss

    def state_dict(self):
        for p in self._plist():
            self.state[p]["step"] = torch.tensor(float(self._step))
        return super().state_dict()

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        with torch.no_grad():
            for p, (off, n) in zip(self._plist(), self._ranges):
                st = self.state[p]
                for key, flat in (("exp_avg", self.flat_m), ("exp_avg_sq", self.flat_v)):
                    if key in st:
                        flat[off:off + n].copy_(st[key].reshape(-1).to(flat.device, torch.float32))
                    st[key] = flat[off:off + n].view_as(p)
                if "step" in st:
                    self._step = int(float(st["step"]))
                st["step"] = torch.tensor(float(self._step))


def make_optimizer(cfg, net, clip_value=40.0):
    """One param group per tensor, like the reference (optimizer.py:12-22)."""
    lr, wd, eps = cfg.train.lr, cfg.train.weight_decay, cfg.train.eps
    params = [{"params": [p], "lr": lr, "weight_decay": wd, "eps": eps}
              for _, p in net.named_parameters() if p.requires_grad]
    if "adam" not in cfg.train.optim:
        raise NotImplementedError(f"optimizer {cfg.train.optim!r}: only adam is on the lego path")
    return FusedAdam(params, lr, weight_decay=wd, eps=eps, clip_value=clip_value)
