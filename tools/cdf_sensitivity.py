"""Calibration of the selective coarse pass (round 6): how far the split-bf16 coarse net moves the CDF of
volume_renderer.py:82-134, against the fp32 coarse net, on the trained net's 800x800 held-out frame (GPU; test
infrastructure: reads tests/golden/, imports nothing from oracle/).

    python tools/cdf_sensitivity.py [--dtype bf16x3] [--out gpurun_out/r6/cdf_sensitivity.json]

For every ray of the frame (64 stratified samples at perturb 0): coarse raw at fp32 and at the tier, weights
(nerf_composite_fwd), then the CDF and the importance samples' bins (nerf_sample_pdf, debug outputs).  Reports
  * the CDF moves: max |dcdf| / (min(c, 1 - c) + abs_tol) and quantiles (the rel_tol the fragile flag needs),
  * the rays whose bins differ (and, separately, whose samples moved by > 1e-3: bins or the den switch) and
    how many of the bin moves the fragile flag (nerf_composite_pdf_fragile on the tier's coarse raw, den rule off)
    missed, at several rel_tol / abs_tol,
  * the flagged fraction at each rel_tol (the fp32 re-evaluation the selective render pays).
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "nerf-replication_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
os.environ.setdefault("NERF_AMD_NO_ARGV", "1")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16x3")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "r6", "cdf_sensitivity.json"))
    args = ap.parse_args()
    from fullframe_outliers import frame_rays
    from nerf_amd import ops
    from src.config import cfg
    from src.models.nerf.network import Network
    from src.models.nerf.renderer.volume_renderer import FRAGILE_ABS_TOL
    dev = torch.device("cuda:0")
    g4 = np.load(os.path.join(ROOT, "tests/golden/golden_v4.npz"), allow_pickle=False)
    z = np.load(os.path.join(ROOT, "tests/golden/trained_v2.npz"), allow_pickle=False)
    cfg.task_arg.perturb = 0
    torch.manual_seed(0)
    net = Network()
    net.load_state_dict({k: torch.from_numpy(z[k]) for k in z.files}, strict=True)
    net = net.to(dev).eval()
    rays = frame_rays(g4, dev)
    near, far = torch.tensor([2.0], device=dev), torch.tensor([6.0], device=dev)
    n_s, n_i = 64, 128
    rels = [1e-5, 3e-5, 1e-4, 3e-4, 1e-3]
    abs_tols = [0.0, 3e-8, 1.2e-7]
    stats = {"dtype": args.dtype, "rays": int(rays.shape[0]), "abs_tol": FRAGILE_ABS_TOL, "ratio_max": 0.0,
             "bins_moved_rays": 0, "missed": {f"{r}/{a}": 0 for r in rels for a in abs_tols},
             "flagged": {f"{r}/{a}": 0 for r in rels for a in abs_tols}}
    ratios = []
    with torch.no_grad():
        for i in range(0, rays.shape[0], 65536):
            rc = rays[i:i + 65536]
            zc, pts, vd = ops.sample_stratified(rc, near, far, n_s, False)
            out = {}
            for dt in ("fp32", args.dtype):
                raw = net(pts, vd, "coarse", dtype=dt)
                _, _, _, w = ops.composite(raw, zc, rc[:, 3:6], False)
                out[dt] = (raw, ops.sample_pdf(zc, w, n_i, det=True, rays=rc, debug=True))
            cf, cb = out["fp32"][1]["cdf"], out[args.dtype][1]["cdf"]
            d = (cb - cf).abs()
            ratio = (d / (torch.minimum(cf, 1 - cf).clamp_min(0) + FRAGILE_ABS_TOL))[:, 1:]  # (cdf[0] = 0 exact)
            stats["ratio_max"] = max(stats["ratio_max"], float(ratio.max()))
            ratios.append(ratio.flatten()[torch.randperm(ratio.numel(), device=dev)[:200000]].cpu())
            moved = (out["fp32"][1]["inds"] != out[args.dtype][1]["inds"]).any(1)
            # (the den switch: samples of an unchanged bin that still moved by more than a bin-relative 1e-3)
            ds = (out["fp32"][1]["samples"] - out[args.dtype][1]["samples"]).abs().amax(1)
            moved = moved | (ds > 1e-3)
            stats["bins_moved_rays"] += int(moved.sum())
            binmoved = (out["fp32"][1]["inds"] != out[args.dtype][1]["inds"]).any(1)
            stats["bin_moved_rays"] = stats.get("bin_moved_rays", 0) + int(binmoved.sum())
            for r in rels:
                for a in abs_tols:
                    _, _, _, _, frag = ops.composite_sample_pdf_fragile(out[args.dtype][0], zc, rc, False, n_i, r, a)
                    f = frag.bool()
                    stats["flagged"][f"{r}/{a}"] += int(f.sum())
                    stats["missed"][f"{r}/{a}"] += int((binmoved & ~f).sum())
    q = torch.cat(ratios)
    stats["ratio_quantiles"] = {str(p): float(torch.quantile(q, p)) for p in (0.5, 0.9, 0.99, 0.999)}
    stats["flagged_fraction"] = {k: v / stats["rays"] for k, v in stats["flagged"].items()}
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    json.dump(stats, open(args.out, "w"), indent=1)
    print(json.dumps(stats), flush=True)


if __name__ == "__main__":
    main()
