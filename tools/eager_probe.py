import os, sys, time, torch
sys.path[:0]=['/root/repo','/root/repo/nerf-replication_amd']
os.environ.setdefault("NERF_AMD_NO_ARGV","1")
import bench
from oracle import nerf_oracle as O
dev=torch.device('cuda:0')
for dt in ('fp32','bf16'):
    print(dt, bench.eager_gpu_baseline(dev, 4096, dt, reps=2), flush=True)
# profile one bf16 autocast step
prm = {k: v.to(dev).clone().requires_grad_(True) for k, v in O.seeded_network_state(0).items()}
C, Fn = O.split_params(prm, "model"), O.split_params(prm, "model_fine")
rays, gt = bench._bench_rays(O, 4096, dev)
near, far = torch.tensor([2.0], device=dev), torch.tensor([6.0], device=dev)
from torch.profiler import profile, ProfilerActivity
def step():
    with torch.autocast("cuda", dtype=torch.bfloat16):
        ret = O.render(C, Fn, rays, near, far, perturb=True)
    O.loss_fn({k: v.float() for k, v in ret.items()}, gt)[0].backward()
step(); torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as p:
    step(); torch.cuda.synchronize()
print(p.key_averages().table(sort_by="cuda_time_total", row_limit=15))
