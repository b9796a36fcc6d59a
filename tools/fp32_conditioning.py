"""How far the fp32 contract (rgb / depth within 1e-4 of the reference) is a property of fp32
arithmetic itself, on the trained-net goldens (tests/golden/golden_v2.npz, golden_v3.npz, written
by the reference).  CPU only; test infrastructure (imports the oracle).

    python tools/fp32_conditioning.py [--mode fp64|bf16x6|bf16x3]

Renders the goldens' rays with the oracle whose MLP is replaced by
  fp64    every layer in float64 (exact up to fp64 rounding), rounded to fp32 per layer output
  bf16x6  every operand split exactly into three bf16 (x = hi + mid + lo), the six cross products
          hh, hm, mh, hl, lh, mm (dropped terms < 2^-24 relative), accumulated in fp64
  bf16x3  hi + lo split, products hh + hl + lh (the kernels' bf16x3 tier)
and prints the largest |ours - reference| per golden and, for the view100 rays that move by more
than 1e-3, the coarse CDF's steps next to sample_pdf's den < 1e-5 switch
(volume_renderer.py:120-126): the reference output is discontinuous there at the ulp level.
"""
import argparse
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import nerf_oracle as O  # noqa: E402


def bf(x):
    return x.to(torch.bfloat16).to(torch.float32)


def split3(x):
    h = bf(x)
    r = x - h
    m = bf(r)
    return h, m, bf(r - m)


def make_lin(mode):
    def lin(x, w, b):
        if mode == "fp64":
            return (F.linear(x.double(), w.double()) + b.double()).float()
        xs, ws = split3(x), split3(w)
        pairs = [(0, 0), (0, 1), (1, 0), (0, 2), (2, 0), (1, 1)] if mode == "bf16x6" else [(0, 0), (0, 1), (1, 0)]
        return (sum(F.linear(xs[i].double(), ws[j].double()) for i, j in pairs) + b.double()).float()
    return lin


def make_mlp(lin):
    def mlp(p, x63, d27):
        h = x63
        for i in range(8):
            h = F.relu(lin(h, *p[f"pts_linears.{i}"]))
            if i == 4:
                h = torch.cat([x63, h], -1)
        alpha = lin(h, *p["alpha_linear"])
        feat = lin(h, *p["feature_linear"])
        hv = F.relu(lin(torch.cat([feat, d27], -1), *p["views_linears.0"]))
        return torch.cat([lin(hv, *p["rgb_linear"]), alpha], -1)
    return mlp


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="fp64", choices=["fp64", "bf16x6", "bf16x3"])
    args = ap.parse_args()
    torch.set_num_threads(os.cpu_count() or 1)
    z = np.load(os.path.join(ROOT, "tests/golden/trained_v2.npz"))
    st = {k: torch.from_numpy(z[k]) for k in z.files}
    g2 = np.load(os.path.join(ROOT, "tests/golden/golden_v2.npz"))
    g3 = np.load(os.path.join(ROOT, "tests/golden/golden_v3.npz"))
    C, Fn = O.split_params(st, "model"), O.split_params(st, "model_fine")
    near, far = torch.tensor([2.0]), torch.tensor([6.0])
    fp32_mlp = O.mlp
    O.mlp = make_mlp(make_lin(args.mode))
    for k in g3["frames"].tolist():
        out = O.render(C, Fn, torch.from_numpy(g3[f"video_rays_{k}"]), near, far)
        print(f"video frame {k:3d} rgb_map_f max err {np.abs(out['rgb_map_f'].numpy() - g3[f'video_rgb_{k}']).max():.3g}")
    out = O.render(C, Fn, torch.from_numpy(g2["rays"]), near, far)
    for kk in ("rgb_map_f", "depth_map_f", "acc_map_f", "rgb_map_c", "depth_map_c"):
        print(f"render0 {kk} max err {np.abs(out[kk].numpy() - g2['render0_' + kk]).max():.3g}")
    rays = torch.from_numpy(g2["view100_rays"])
    mine = O.render(C, Fn, rays, near, far, keep=True)
    e = np.abs(mine["rgb_map_f"].numpy() - g2["view100_rgb_map_f"]).max(-1)
    print(f"view100 rgb_map_f max err {e.max():.3g}, values over 1e-4: {(e > 1e-4).sum()}")
    bad = np.nonzero(e > 1e-3)[0].tolist()
    if bad:
        O.mlp = fp32_mlp
        ref = O.render(C, Fn, rays[bad], near, far, keep=True)
        for i, r in enumerate(bad):
            den_ref = (ref["cdf"][i, 1:] - ref["cdf"][i, :-1])
            den_ours = (mine["cdf"][r, 1:] - mine["cdf"][r, :-1])
            flips = int(((den_ref < 1e-5) != (den_ours < 1e-5)).sum())
            print(f"  ray {r}: rgb err {e[r]:.3g}; coarse weight sum {float(ref['weights_c'][i].sum()):.3g}; "
                  f"CDF steps within 1e-7 of the 1e-5 switch: {int(((den_ref - 1e-5).abs() < 1e-7).sum())}; "
                  f"steps that switch differently: {flips}; largest fine-sample move "
                  f"{float((ref['z_samples'][i] - mine['z_samples'][r]).abs().max()):.3g}")


if __name__ == "__main__":
    main()
