"""Training on the GPU against the reference's arithmetic, over several optimizer steps.

* ``test_trajectory_fp32_vs_oracle``: 10 steps of the production training step
  (Trainer.train_step: kernels, direct dW into FusedAdam's flat .grad, fused clip 40 + Adam)
  from the trained fixture weights, 64 rays of the config-3 batch per step, perturb 0.  At
  every step the GPU's loss is held to 1e-4 of the oracle's (tests-only CPU restatement of
  volume_renderer.render + network) evaluated at the GPU's current parameters, and the
  free-running oracle trajectory (clip_grad_value_(40) + torch.optim.Adam, one group per
  tensor; trainer.py:60-62, optimizer.py:8-28) is run beside it: its loss stays within 1e-4
  of the GPU's for the first 6 steps.  After that the two trajectories separate the way any
  two fp32 evaluations of the reference do: Adam turns last-ulp gradient differences of
  cancelling entries into +-lr steps, and an importance sample whose u sits within an ulp of
  a CDF entry changes bins (volume_renderer.py:117) -- recorded, not asserted.
* ``test_psnr_fp32_vs_bf16_training``: the same training run (seed-0 init, procedural scene,
  identical ray streams) with the fp32, the bf16 and the bf16x3 MLP; held-out PSNR curve of each
  (BASELINE config 3's "PSNR curve").  The two runs are different trajectories, so their PSNR
  difference is training noise (checkpoint differences of +-0.6 dB, either sign), so only the
  mean difference over the curve is bounded (0.5 dB); the north_star's 0.05 dB is about
  rendering the SAME weights, held in test_gpu_trained.py::test_heldout_view_psnr.
"""
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
os.environ.setdefault("NERF_AMD_NO_ARGV", "1")
HERE = os.path.dirname(os.path.abspath(__file__))


def _trained():
    z = np.load(os.path.join(HERE, "golden", "trained_v2.npz"), allow_pickle=False)
    return {k: torch.from_numpy(z[k]) for k in z.files}


def test_trajectory_fp32_vs_oracle(cuda):
    from oracle import nerf_oracle as O
    from nerf_amd import ops
    from src.config import cfg
    from src.models.nerf.network import Network
    from src.train.optimizer import make_optimizer
    from src.train.trainers.make_trainer import make_trainer
    g2 = np.load(os.path.join(HERE, "golden", "golden_v2.npz"), allow_pickle=False)
    rays_all = torch.from_numpy(g2["rays4096"])
    gt_all = torch.from_numpy(g2["grad4096_gt"]).reshape(-1, 3)
    state = _trained()
    cfg.task_arg.perturb = 0
    cfg.task_arg.mlp_dtype = "fp32"
    torch.manual_seed(0)
    net = Network()
    net.load_state_dict(state, strict=True)
    net = net.to(cuda)
    trainer = make_trainer(cfg, net)
    opt = make_optimizer(cfg, net)
    prm = {k: v.clone().requires_grad_(True) for k, v in state.items()}
    C, Fn = O.split_params(prm, "model"), O.split_params(prm, "model_fine")
    adam = torch.optim.Adam([{"params": [p]} for p in prm.values()], lr=float(cfg.train.lr), eps=float(cfg.train.eps))
    near, far = torch.tensor([2.0]), torch.tensor([6.0])
    forced, free = [], []
    for step in range(10):
        sl = slice(64 * step, 64 * (step + 1))
        rays, gt = rays_all[sl], gt_all[sl]
        # the reference's loss at the parameters the GPU trajectory has reached
        cur = {k: v.detach().cpu() for k, v in net.state_dict().items()}
        with torch.no_grad():
            at_gpu = O.loss_fn(O.render(O.split_params(cur, "model"), O.split_params(cur, "model_fine"), rays, near,
                                        far), gt)[0]
        batch = {"rays": rays.to(cuda)[None], "rgbs": gt.to(cuda)[None], "near": ops.device_scalar(2.0, cuda),
                 "far": ops.device_scalar(6.0, cuda)}
        _, loss, _ = trainer.train_step(batch, opt)
        adam.zero_grad()
        loss_ref = O.loss_fn(O.render(C, Fn, rays, near, far), gt)[0]
        loss_ref.backward()
        torch.nn.utils.clip_grad_value_(list(prm.values()), 40.0)
        adam.step()
        forced.append((float(loss), float(at_gpu)))
        free.append((float(loss), float(loss_ref)))
    print("\nper-step loss (gpu, oracle at gpu params):", json.dumps(forced))
    print("free-running (gpu, oracle + torch Adam):", json.dumps(free))
    for a, b in forced:
        assert abs(a - b) < 1e-4, forced
    for a, b in free[:6]:
        assert abs(a - b) < 1e-4, free


@pytest.mark.parametrize("steps,every", [(int(os.environ.get("NERF_PSNR_STEPS", "2000")), 250)])
def test_psnr_fp32_vs_bf16_training(cuda, steps, every):
    from nerf_amd import ops
    from src.config import cfg
    from src.datasets.nerf.blender import Dataset
    from src.datasets.nerf.synthetic import camera_rays, make_scene, psnr, shade, view_poses
    from src.models import make_network
    from src.models.nerf.renderer.volume_renderer import Renderer
    from src.train.optimizer import make_optimizer
    from src.train.trainers.make_trainer import make_trainer
    from src.utils.camera import focal_for
    imgs, poses, focal = make_scene(100, 100, 100, cuda, seed=0)
    ev = view_poses(4, seed=1).to(cuda)
    f_ev = focal_for(100)
    gts, evrays = [], []
    for k in range(ev.shape[0]):
        o, d = camera_rays(ev[k], 100, 100, f_ev)
        gts.append(shade(o, d))
        evrays.append(torch.cat([o, d], -1))

    def heldout(net):
        cfg.task_arg.perturb = 0
        net.eval()
        r = Renderer(net)
        ps = []
        with torch.no_grad():
            for rr, gt in zip(evrays, gts):
                out = r.render({"rays": rr, "near": torch.tensor([2.0], device=cuda),
                                "far": torch.tensor([6.0], device=cuda)})
                ps.append(psnr(out["rgb_map_f"], gt))
        net.train()
        cfg.task_arg.perturb = 1
        return float(np.mean(ps))

    curve = {}
    low = ("bf16", "bf16x3")
    for dtype in ("fp32",) + low:
        cfg.task_arg.mlp_dtype = dtype
        cfg.task_arg.perturb = 1
        torch.manual_seed(0)
        net = make_network(cfg)
        trainer = make_trainer(cfg, net)
        opt = make_optimizer(cfg, net)
        ds = Dataset.from_arrays(imgs, poses, focal)  # same seed -> same ray stream for both dtypes
        curve[dtype] = []
        for step in range(1, steps + 1):
            rays, rgbs = ds.sample_batch()
            trainer.train_step({"rays": rays[None], "rgbs": rgbs[None], "near": ops.device_scalar(2.0, cuda),
                                "far": ops.device_scalar(6.0, cuda)}, opt)
            if step % every == 0:
                curve[dtype].append((step, heldout(net)))
    cfg.task_arg.mlp_dtype = "fp32"
    cfg.task_arg.perturb = 0
    summary = {"steps": steps, "rays_per_step": int(cfg.task_arg.train_rays), "heldout_views": 4, "res": 100}
    for dt in ("fp32",) + low:
        summary[f"psnr_curve_{dt}"] = curve[dt]
    for dt in low:  # keys without a suffix: bf16 (round-2 record format)
        sfx = "" if dt == "bf16" else f"_{dt}"
        summary["final_delta_db" + sfx] = curve[dt][-1][1] - curve["fp32"][-1][1]
        summary["mean_delta_db" + sfx] = float(np.mean([b[1] - a[1] for a, b in zip(curve["fp32"], curve[dt])]))
    print("\nPSNR " + json.dumps(summary))
    out_dir = os.path.join(os.path.dirname(HERE), "gpurun_out")
    if os.path.isdir(out_dir):
        with open(os.path.join(out_dir, "psnr_fp32_vs_bf16.json"), "w") as f:
            json.dump(summary, f, indent=1)
    # both runs learn the scene; their curves agree to within the run-to-run noise (checkpoint
    # differences of +-0.6 dB, either sign, were measured: profiles/r2/psnr_fp32_vs_bf16.json)
    for dt in ("fp32",) + low:
        assert curve[dt][-1][1] > curve[dt][0][1] + 3.0, summary
    # The mean over 8 checkpoints (every 250 steps; rounds 2-4 used 4, every 500) of the shipped
    # default configuration.  The 4-checkpoint bf16 mean moved with any bit-level change of its
    # trajectory: -0.33 / +0.18 (round 2), -0.47 (round 3), +0.05 (round 4 default), and -0.53
    # with the opt-in chunked backward (off by default, not what this test runs); the 200k-step
    # config-3 runs put bf16 +0.23 dB from fp32, inside its own 0.47 dB seed-to-seed spread.
    assert abs(summary["mean_delta_db"]) <= 0.5, summary
    assert abs(summary["mean_delta_db_bf16x3"]) <= 0.5, summary


@pytest.mark.parametrize("dtype", ["fp32", "bf16x3f", "bf16"])
def test_backward_scheduling_knobs(cuda, dtype):
    """The MLP backward's opt-in schedules (nerf_amd/ops.py) on the production step's
    forward_backward (4096 rays of the config-3 batch, trained weights, direct dW into the flat
    .grad): the dW stream (NERF_DW_STREAM, every dW on a second stream after its dX) gives the
    one-stream gradient bit for bit; the chunked backward (BWD_CHUNK, dX + dW per 262,144
    samples) the same gradient up to the order of the dW partial sums (relative 1e-5 of each
    tensor's largest entry; measured ~5e-7, tools/mlp_bench.py --chunks)."""
    from nerf_amd import ops
    from src.config import cfg
    from src.models.nerf.network import Network
    from src.train.optimizer import make_optimizer
    from src.train.trainers.make_trainer import make_trainer
    g2 = np.load(os.path.join(HERE, "golden", "golden_v2.npz"), allow_pickle=False)
    rays = torch.from_numpy(g2["rays4096"]).to(cuda)
    gt = torch.from_numpy(g2["grad4096_gt"]).reshape(-1, 3).to(cuda)
    cfg.task_arg.perturb = 0
    cfg.task_arg.mlp_dtype = dtype
    torch.manual_seed(0)
    net = Network()
    net.load_state_dict(_trained(), strict=True)
    net = net.to(cuda)
    trainer = make_trainer(cfg, net)
    opt = make_optimizer(cfg, net)
    batch = {"rays": rays[None], "rgbs": gt[None], "near": ops.device_scalar(2.0, cuda),
             "far": ops.device_scalar(6.0, cuda)}
    saved = (dict(ops.BWD_CHUNK), ops.DW_STREAM)
    code = ops.pack_code(ops.dtype_code(dtype), 1)
    grads = {}
    try:
        for name, chunk, stream in (("one", None, False), ("stream", None, True), ("chunk", 262144, False),
                                    ("chunk+stream", 262144, True)):
            ops.BWD_CHUNK = {code: chunk} if chunk else {}
            ops.DW_STREAM = stream
            trainer.forward_backward(dict(batch), opt)
            torch.cuda.synchronize()
            grads[name] = opt.flat_grad.clone()
    finally:
        ops.BWD_CHUNK, ops.DW_STREAM = saved
        cfg.task_arg.mlp_dtype = "fp32"
    assert torch.equal(grads["one"], grads["stream"])
    assert torch.equal(grads["chunk"], grads["chunk+stream"])
    for off, n in opt._ranges:  # per tensor of the flat gradient
        a, b = grads["one"][off:off + n], grads["chunk"][off:off + n]
        assert float((a - b).abs().max()) <= 1e-5 * float(a.abs().max()) + 1e-12, (dtype, off, n)
