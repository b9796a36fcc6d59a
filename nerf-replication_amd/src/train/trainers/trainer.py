"""Trainer (reference: src/train/trainers/trainer.py:11-130), data-parallel on RCCL.

The reference wraps the loss module in DistributedDataParallel (trainer.py:15-22).  Here
every rank draws its own rays (rank-distinct Philox streams), and the gradient -- one flat
fp32 buffer owned by FusedAdam (1,191,688 values, 4.77 MB) -- is averaged across ranks in
two buckets, one per NeRF: each net's MLP backward reports its finished flat gradient
(PackedMLP.grad_ready) and that bucket's all-reduce starts at once on the collective
stream, so the fine net's reduction (its backward runs first) overlaps the coarse net's
backward.  The next batch's ray generation and stratified sampling (which read no
parameter) are enqueued before the step waits for the reduction, so they run while it is in
flight (``train_step(..., prefetch=)``).  Initial weights are broadcast from rank 0, as DDP
does at construction.  The clip_grad_value_(40) of trainer.py:61 is fused into the Adam
launch.
"""
import contextlib
import datetime
import time

import torch
import torch.distributed as dist

from src.config import cfg


def dist_world():
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def broadcast_params(module: torch.nn.Module) -> None:
    if dist_world() > 1:
        with torch.no_grad():
            for p in module.parameters():
                dist.broadcast(p.data, src=0)


def allreduce_grads(optimizer) -> None:
    """Average the flat gradient across ranks (one collective per step)."""
    if dist_world() > 1:
        g = optimizer.flat_grad
        dist.all_reduce(g, op=dist.ReduceOp.SUM)
        g.mul_(1.0 / dist_world())


class GradBuckets:
    """Per-net all-reduce buckets started from inside backward.

    ``attach(packers)`` installs a grad_ready hook on every NeRF's PackedMLP; a hook fires
    when that net's dW has been enqueued into its slice of the flat gradient and starts an
    async SUM all-reduce of the slice.  ``finish(optimizer)`` waits for the started buckets,
    all-reduces whatever did not report (a net whose grads are not flat views, or that did
    not run), and divides by the world size."""

    def __init__(self):
        self.works = []
        self.done = []
        self.packers = []
        self.events = None  # a list: finish() appends (start, end) HIP events on the compute stream

    def exposed_ms(self):
        """Mean compute-stream time per step spent in finish() (waiting for the buckets + the
        1/W scale): the part of the all-reduce the backward did not hide."""
        if not self.events:
            return None
        torch.cuda.synchronize()
        return sum(a.elapsed_time(b) for a, b in self.events) / len(self.events)

    def attach(self, packers):
        self.packers = list(packers)
        for pk in self.packers:
            pk.grad_ready = self._hook

    @contextlib.contextmanager
    def suspended(self):
        """No bucket fires inside (a local, un-reduced backward)."""
        hooks = [pk.grad_ready for pk in self.packers]
        for pk in self.packers:
            pk.grad_ready = None
        try:
            yield
        finally:
            for pk, h in zip(self.packers, hooks):
                pk.grad_ready = h

    def begin(self) -> None:
        """Start of a step: forget forwards whose backward never ran (an aborted step), so a
        net's bucket fires after exactly this step's last chunk."""
        for pk in self.packers:
            pk.pending = 0

    def _hook(self, flat):
        if flat is None or dist_world() == 1:
            return
        self.works.append(dist.all_reduce(flat, op=dist.ReduceOp.SUM, async_op=True))
        self.done.append((flat.data_ptr(), flat.numel()))

    def finish(self, optimizer) -> None:
        world = dist_world()
        if world == 1:
            return
        ev = None
        if self.events is not None and optimizer.flat_grad.is_cuda:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        for w in self.works:
            w.wait()
        g = optimizer.flat_grad
        base = g.data_ptr()
        covered = sorted(((p - base) // 4, n) for p, n in self.done)
        pos = 0
        for off, n in covered + [(g.numel(), 0)]:
            if off > pos:  # a range nobody reported: reduce it now
                dist.all_reduce(g[pos:off], op=dist.ReduceOp.SUM)
            pos = max(pos, off + n)
        g.mul_(1.0 / world)
        if ev is not None:
            ev[1].record()
            self.events.append(ev)
        self.works, self.done = [], []


class Trainer:
    def __init__(self, network):
        device = torch.device("cuda", cfg.local_rank) if torch.cuda.is_available() else torch.device("cpu")
        self.network = network.to(device)
        broadcast_params(self.network)
        self.local_rank = cfg.local_rank
        self.device = device
        self.global_step = 0
        self.clip_value = 40.0
        self.prefetched = None
        self.buckets = GradBuckets()
        self.buckets.packers = [m.packer() for m in self.network.modules() if hasattr(m, "packer")]
        if dist_world() > 1:
            self.buckets.attach(self.buckets.packers)

    def reduce_loss_stats(self, loss_stats):
        return {k: torch.mean(v) for k, v in loss_stats.items()}

    def to_cuda(self, batch):
        if batch is None:
            return None
        out = {}
        for k, v in batch.items():
            if torch.is_tensor(v):
                out[k] = v.to(self.device, non_blocking=True)
            elif isinstance(v, (list, tuple)):
                out[k] = [b.to(self.device) if torch.is_tensor(b) else b for b in v]
            else:
                out[k] = v
        return out

    def prepare(self, batch):
        """Device copy of a batch with its first render chunk's stratified samples computed
        (Renderer.prepare): work that reads no parameter, so it may run before the previous
        step's optimizer update."""
        batch = self.to_cuda(batch)
        renderer = getattr(self.network, "renderer", None)
        if batch is not None and renderer is not None and hasattr(renderer, "prepare"):
            renderer.prepare(batch)
        return batch

    def forward_backward(self, batch, optimizer):
        """render -> loss -> backward, dW straight into FusedAdam's flat .grad; the per-net
        all-reduce buckets start inside (trainer.py:53-60 of the reference)."""
        from nerf_amd import ops
        self.buckets.begin()
        output, loss, loss_stats = self.network(batch)
        if loss.dim() > 0:  # (a 0-d loss is its own mean: no extra launch)
            loss = loss.mean()
        optimizer.zero_grad()
        with ops.direct_grad():
            loss.backward()
        return output, loss, loss_stats

    def apply(self, optimizer):
        """Wait for the gradient buckets, then fused clip_grad_value_(40) + Adam (:61-62)."""
        self.buckets.finish(optimizer)
        optimizer.clip_value = self.clip_value
        optimizer.step()

    def train_step(self, batch, optimizer, prefetch=None):
        """One step.  ``prefetch`` (optional) returns the next batch: it is called after the
        backward has been enqueued and before the step waits for the gradient all-reduce, and
        the prepared batch (its rays and first chunk's stratified samples enqueued on the
        compute stream, overlapping the reduction) is left in ``self.prefetched``."""
        output, loss, loss_stats = self.forward_backward(batch, optimizer)
        self.prefetched = self.prepare(prefetch()) if prefetch is not None else None
        self.apply(optimizer)
        return output, loss, loss_stats

    def train(self, epoch, data_loader, optimizer, recorder):
        max_iter = len(data_loader)
        self.network.train()
        end = time.time()
        it = iter(data_loader)
        batch = next(it, None)
        if batch is not None:
            batch = self.prepare(batch)
        iteration = 0
        while batch is not None:
            data_time = time.time() - end
            iteration += 1
            batch["step"] = self.global_step
            _, loss, loss_stats = self.train_step(batch, optimizer, prefetch=lambda: next(it, None))
            batch = self.prefetched
            self.global_step += 1
            if self.local_rank > 0:
                continue
            recorder.step += 1
            if iteration % cfg.log_interval == 0 or iteration == (max_iter - 1):
                recorder.update_loss_stats(self.reduce_loss_stats(loss_stats))
                batch_time = time.time() - end
                recorder.batch_time.update(batch_time / cfg.log_interval)
                recorder.data_time.update(data_time)
                end = time.time()
                eta = recorder.batch_time.global_avg * (max_iter - iteration)
                lr = optimizer.param_groups[0]["lr"]
                mem = torch.cuda.max_memory_allocated() / 1024.0 / 1024.0 if torch.cuda.is_available() else 0.0
                print("  ".join([f"eta: {datetime.timedelta(seconds=int(eta))}", str(recorder), f"lr: {lr:.6f}",
                                 f"max_mem: {mem:.0f}"]))
                recorder.record("train")

    def val(self, epoch, data_loader, evaluator=None, recorder=None):
        self.network.eval()
        val_loss_stats = {}
        n = 0
        for batch in data_loader:
            batch = self.to_cuda(batch)
            with torch.no_grad():
                output, loss, loss_stats = self.network(batch)
                if evaluator is not None:
                    evaluator.evaluate(output, batch)
            for k, v in self.reduce_loss_stats(loss_stats).items():
                val_loss_stats[k] = val_loss_stats.get(k, 0.0) + float(v)
            n += 1
        print([f"{k}: {v / max(n, 1):.4f}" for k, v in val_loss_stats.items()])
        result = evaluator.summarize() if evaluator is not None else {}
        if recorder:
            recorder.record("val", epoch, val_loss_stats, result)
        return result
