"""One ray's importance sampling under the fp32 and the split-bf16 coarse net (round 6 diagnostic of the selective
coarse pass; GPU, test infrastructure, reads tests/golden/).

    python tools/fragile_ray.py [--pixel 291410] [--dtype bf16x3]

Prints, for every importance sample whose bin differs between the two coarse nets: u, the bracketing CDF entries
under both, their move, and min(c, 1 - c); and the fragile flag of nerf_composite_pdf_fragile at several rel_tol.
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
    ap.add_argument("--pixel", type=int, default=291410)
    ap.add_argument("--dtype", default="bf16x3")
    args = ap.parse_args()
    from fullframe_outliers import frame_rays
    from nerf_amd import ops
    from src.config import cfg
    from src.models.nerf.network import Network
    dev = torch.device("cuda:0")
    g4 = np.load(os.path.join(ROOT, "tests/golden/golden_v4.npz"), allow_pickle=False)
    z = np.load(os.path.join(ROOT, "tests/golden/trained_v2.npz"), allow_pickle=False)
    cfg.task_arg.perturb = 0
    torch.manual_seed(0)
    net = Network()
    net.load_state_dict({k: torch.from_numpy(z[k]) for k in z.files}, strict=True)
    net = net.to(dev).eval()
    rc = frame_rays(g4, dev)[args.pixel:args.pixel + 1]
    near, far = torch.tensor([2.0], device=dev), torch.tensor([6.0], device=dev)
    with torch.no_grad():
        zc, pts, vd = ops.sample_stratified(rc, near, far, 64, False)
        res = {}
        for dt in ("fp32", args.dtype):
            raw = net(pts, vd, "coarse", dtype=dt)
            _, _, _, w = ops.composite(raw, zc, rc[:, 3:6], False)
            res[dt] = (raw, w, ops.sample_pdf(zc, w, 128, det=True, rays=rc, debug=True))
        flags = {}
        for rel in (1e-5, 1e-4, 1e-3, 1e-2, 1e-1):
            flags[str(rel)] = int(ops.composite_sample_pdf_fragile(res[args.dtype][0], zc, rc, False, 128, rel,
                                                                   1.2e-7)[4][0])
    cf, cb = res["fp32"][2]["cdf"][0].double().cpu(), res[args.dtype][2]["cdf"][0].double().cpu()
    i_f, i_b = res["fp32"][2]["inds"][0].cpu(), res[args.dtype][2]["inds"][0].cpu()
    u = torch.linspace(0, 1, 128).double()
    moves = []
    for i in torch.nonzero(i_f != i_b).flatten().tolist():
        ks = sorted({int(i_f[i]) - 1, int(i_f[i]), int(i_b[i]) - 1, int(i_b[i])})
        moves.append({"i": i, "u": float(u[i]), "ind_fp32": int(i_f[i]), "ind_tier": int(i_b[i]),
                      "entries": {k: {"fp32": float(cf[k]), "tier": float(cb[k]), "move": float(cb[k] - cf[k]),
                                      "min_c_1mc": float(min(cf[k], 1 - cf[k]))} for k in ks if 0 <= k < cf.numel()}})
    wf, wb = res["fp32"][1][0].double().cpu(), res[args.dtype][1][0].double().cpu()
    out = {"pixel": args.pixel, "moves": moves, "flag_at_rel_tol": flags,
           "max_cdf_move": float((cb - cf).abs().max()), "acc_fp32": float(wf.sum()),
           "max_weight_move": float((wb - wf).abs().max())}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
