"""Inference-forward time per precision at 524,288 samples (median of 3 rounds x 5 launches; HIP events)."""
import os, sys, json, torch
sys.path.insert(0, os.path.join(os.getcwd(), "nerf-replication_amd"))
from nerf_amd import ops
dev = torch.device("cuda:0")
torch.manual_seed(0)
shapes = [(256, 63), (256,)] + [(256, 256), (256,)] * 4 + [(256, 319), (256,)] + [(256, 256), (256,)] * 2 + \
         [(128, 283), (128,), (256, 256), (256,), (1, 256), (1,), (3, 128), (3,)]
params = [(torch.rand(s, device=dev) - 0.5) * (0.2 if len(s) == 2 else 0.1) for s in shapes]
packer = ops.PackedMLP(params)
M = 524288
pts = (torch.rand(M, 3, device=dev) - 0.5) * 3
vd = torch.nn.functional.normalize(torch.randn(M // 64, 3, device=dev), dim=-1)
out = {}
with torch.no_grad():
    for r in range(4):
        for dt in ("fp32", "bf16x6", "bf16x3"):
            ops.mlp(packer, pts, vd, 64, dtype=dt); torch.cuda.synchronize()
            a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(5): ops.mlp(packer, pts, vd, 64, dtype=dt)
            e.record(); torch.cuda.synchronize()
            if r: out.setdefault(dt, []).append(a.elapsed_time(e) / 5)
print(json.dumps({k: sorted(v)[len(v)//2] for k, v in out.items()}))
