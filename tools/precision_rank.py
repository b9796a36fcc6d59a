"""Rank the NeRF MLP's layers by how much bf16 rounding of each one moves the rendered outputs.

CPU emulation (test infrastructure: it uses the oracle's render with a per-layer precision
MLP) of the kernel's precision tiers on the trained-net goldens (tests/golden/golden_v2.npz,
written by the reference):
  'b'  bf16: the layer's weights and its input activations rounded to bf16 (RNE, as
       v_cvt_pk_bf16_f32), products exact, fp32 accumulation, fp32 bias
  'x'  bf16x3 / fp32: the layer's product in fp32 (bf16x3 is within ~1e-5 of it)
  'w'  weights split hi + lo, activations bf16 (two bf16 MFMAs per product)
  'a'  activations split, weights bf16 (two bf16 MFMAs)
  'h'  fp16: weights and input activations rounded to fp16
Layers: L0..L7 (pts_linears), F (feature_linear), A (alpha_linear), V (views_linears),
R (rgb_linear).  Reference: src/models/nerf/network.py:49-74.

  python tools/precision_rank.py [--greedy] [--cfg bbbbbbbbbbbb]
prints the largest |ours - reference| over render0 / render1 / cfg3sub / view100 per
configuration.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import nerf_oracle as O  # noqa: E402

LAYERS = ["L0", "L1", "L2", "L3", "L4", "L5", "L6", "L7", "F", "A", "V", "R"]
# MFMA tile products per layer (out tiles x in tiles, mlp_tables.h): the cost of each layer
TILES = {"L0": 16, "L1": 64, "L2": 64, "L3": 64, "L4": 64, "L5": 80, "L6": 64, "L7": 64, "F": 64, "A": 8,
         "V": 36, "R": 4}
MFMAS = {"b": 1, "x": 3, "w": 2, "a": 2, "h": 1}


def bf(x):
    return x.to(torch.bfloat16).to(torch.float32)


def lin(mode, x, w, b):
    if mode == "x":
        return F.linear(x, w, b)
    if mode == "h":  # fp16 operands (v_mfma_f32_32x32x16_f16)
        xh, wh = x.to(torch.float16).double(), w.to(torch.float16).double()
        return (F.linear(xh, wh) + b.double()).float()
    xw = bf(x) if mode in "bw" else x
    ww = bf(w) if mode in "ba" else w
    # products of bf16 values are exact in fp32; the accumulation is fp32 (double here, then
    # rounded: the MFMA's fp32 accumulation error is far below the bf16 rounding studied)
    return (F.linear(xw.double(), ww.double()) + b.double()).float()


GRAD_SCALE = 2.0 ** 24  # fp16 backward: dz is stored as fp16(dz * GRAD_SCALE)


def rnd(mode, x, scale=1.0):
    if mode == "b":
        return bf(x)
    if mode == "h":
        return (x * scale).to(torch.float16).to(torch.float32) / scale
    return x


class EmuLinear(torch.autograd.Function):
    """A layer whose backward stores its output gradient (dz) rounded per `bmode` and
    multiplies with the weights / stored input activations rounded the same way (the dX and
    dW kernels), fp32(-exact) accumulation.  dbias = the sum of the stored dz."""

    @staticmethod
    def forward(ctx, x, w, b, fmode, bmode):
        ctx.bmode = bmode
        ctx.save_for_backward(x, w)
        return lin(fmode, x, w, b)

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        m = ctx.bmode
        if m == "x":
            gz, wr, xr = gy, w, x
        else:
            gz = rnd(m, gy, GRAD_SCALE)
            wr, xr = rnd(m, w), rnd(m, x)
        gx = (gz.double() @ wr.double()).float()
        gw = (gz.double().t() @ xr.double()).float()
        return gx, gw, gz.sum(0), None, None


def make_mlp(cfg, bcfg=None):
    m = dict(zip(LAYERS, cfg))
    mb = dict(zip(LAYERS, bcfg)) if bcfg else None

    def L(name, x, w, b):
        if mb is None:
            return lin(m[name], x, w, b)
        return EmuLinear.apply(x, w, b, m[name], mb[name])

    def mlp(p, x63, d27):
        h = x63
        for i in range(8):
            h = F.relu(L(f"L{i}", h, *p[f"pts_linears.{i}"]))
            if i == 4:
                h = torch.cat([x63, h], -1)
        alpha = L("A", h, *p["alpha_linear"])
        feat = L("F", h, *p["feature_linear"])
        hv = F.relu(L("V", torch.cat([feat, d27], -1), *p["views_linears.0"]))
        rgb = L("R", hv, *p["rgb_linear"])
        return torch.cat([rgb, alpha], -1)
    return mlp


def grad_errors(fcfg, bcfg, g2, state, tag="grad64"):
    """Largest gradient error relative to each tensor's largest entry (the test's metric,
    tests/test_gpu_trained.py::_grad_check) for forward modes fcfg / backward modes bcfg
    ("coarse/fine" strings)."""
    fc, ff = fcfg.split("/") if "/" in fcfg else (fcfg, fcfg)
    bc, bfm = bcfg.split("/") if "/" in bcfg else (bcfg, bcfg)
    params = {k: v.clone().requires_grad_(True) for k, v in state.items()}
    pc, pf = O.split_params(params, "model"), O.split_params(params, "model_fine")
    mc, mf = make_mlp(fc, bc), make_mlp(ff, bfm)
    orig = O.mlp
    O.mlp = lambda p, x63, d27: (mc if p is pc else mf)(p, x63, d27)
    try:
        rays = torch.from_numpy(g2["rays" if tag == "grad64" else "rays4096"])
        out = O.render(pc, pf, rays, 2.0, 6.0)
        loss, _, _ = O.loss_fn(out, torch.from_numpy(g2[f"{tag}_gt"]))
        loss.backward()
    finally:
        O.mlp = orig
    worst, wn, worst_norm = 0.0, None, 0.0
    num = den = 0.0
    for i, name in enumerate(g2[f"{tag}_names"]):
        g = params[str(name)].grad.reshape(-1).double()
        sel = g[torch.from_numpy(g2[f"{tag}_sel_idx"][i])].numpy()
        scale = float(g2[f"{tag}_absmax"][i]) + 1e-30
        num += float((((sel - g2[f"{tag}_sel_val"][i]) / scale) ** 2).sum())
        den += float(((g2[f"{tag}_sel_val"][i] / scale) ** 2).sum())
        e = float(np.abs(sel - g2[f"{tag}_sel_val"][i]).max())
        if e < 1e-8:
            e = 0.0
        if e / scale > worst:
            worst, wn = e / scale, str(name)
        nr = abs(float(torch.linalg.vector_norm(g)) - g2[f"{tag}_norms"][i]) / (g2[f"{tag}_norms"][i] + 1e-30)
        worst_norm = max(worst_norm, nr)
    print(f"  sampled-entry relative L2 error (each tensor over its largest entry): {np.sqrt(num / den):.2e}")
    return worst, wn, worst_norm


def load():
    g2 = np.load(os.path.join(ROOT, "tests", "golden", "golden_v2.npz"), allow_pickle=False)
    st = np.load(os.path.join(ROOT, "tests", "golden", "trained_v2.npz"), allow_pickle=False)
    state = {k: torch.from_numpy(st[k]) for k in st.files}
    return g2, O.split_params(state, "model"), O.split_params(state, "model_fine")


def evaluate(cfg, g2, pc, pf, sets=("render0", "render1", "cfg3sub", "view100")):
    """cfg: 12 layer modes for both nets, or "coarse/fine" (12 + 12)"""
    cc, cf = cfg.split("/") if "/" in cfg else (cfg, cfg)
    mc, mf = make_mlp(cc), make_mlp(cf)
    orig = O.mlp
    O.mlp = lambda p, x63, d27: (mc if p is pc else mf)(p, x63, d27)
    worst = {}
    try:
        with torch.no_grad():
            for s in sets:
                if s == "render0":
                    out = O.render(pc, pf, torch.from_numpy(g2["rays"]), 2.0, 6.0)
                elif s == "render1":
                    out = O.render(pc, pf, torch.from_numpy(g2["rays"]), 2.0, 6.0, perturb=True,
                                   t_rand=torch.from_numpy(g2["render1_t_rand"]), u=torch.from_numpy(g2["render1_u"]))
                elif s == "cfg3sub":
                    out = O.render(pc, pf, torch.from_numpy(g2["rays4096"][::16].copy()), 2.0, 6.0)
                else:
                    out = O.render(pc, pf, torch.from_numpy(g2["view100_rays"]), 2.0, 6.0)
                keys = ["rgb_map_f"] if s == "view100" else \
                    ["rgb_map_c", "depth_map_c", "acc_map_c", "rgb_map_f", "depth_map_f", "acc_map_f"]
                for k in keys:
                    e = float(np.abs(out[k].numpy() - g2[f"{s}_{k}"]).max())
                    worst[f"{s}:{k}"] = e
    finally:
        O.mlp = orig
    return worst


def cost(cfg):
    """MFMA cost relative to all-bf16 (coarse 64 + fine 192 samples per ray)"""
    cc, cf = cfg.split("/") if "/" in cfg else (cfg, cfg)
    one = lambda c: sum(TILES[l] * MFMAS[m] for l, m in zip(LAYERS, c)) / sum(TILES.values())
    return (64 * one(cc) + 192 * one(cf)) / 256


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", action="append", default=[])
    ap.add_argument("--single", action="store_true", help="all-bf16 with one layer upgraded, and the reverse")
    ap.add_argument("--greedy", action="store_true")
    ap.add_argument("--sets", default="render0,render1,cfg3sub,view100")
    ap.add_argument("--out", default=None)
    ap.add_argument("--grad", action="append", default=[], help="fwdcfg:bwdcfg, e.g. x*12/h*12:b*12/h*12")
    args = ap.parse_args()
    torch.set_num_threads(os.cpu_count())
    g2, pc, pf = load()
    sets = tuple(args.sets.split(","))
    rows = []

    def run(cfg):
        w = evaluate(cfg, g2, pc, pf, sets)
        k = max(w, key=w.get)
        rows.append({"cfg": cfg, "cost": cost(cfg), "max": w[k], "where": k, "all": w})
        print(f"{cfg}  cost {cost(cfg):.3f}x bf16  max {w[k]:.2e}  ({k})", flush=True)
        return w[k]

    for c in args.cfg:
        run(c)
    if args.grad:
        st = np.load(os.path.join(ROOT, "tests", "golden", "trained_v2.npz"), allow_pickle=False)
        state = {k: torch.from_numpy(st[k]) for k in st.files}
        for spec in args.grad:
            fc, bc = spec.split(":")
            for tag in ("grad64", "grad4096"):
                w, wn, wnorm = grad_errors(fc, bc, g2, state, tag)
                print(f"grad {spec} {tag}: max rel {w:.2e} ({wn}), norm rel {wnorm:.2e}", flush=True)
                rows.append({"grad": spec, "tag": tag, "max_rel": w, "where": wn, "norm_rel": wnorm})
    if args.single:
        run("b" * 12)
        run("x" * 12)
        for i, l in enumerate(LAYERS):
            run("b" * i + "x" + "b" * (11 - i))
        for i, l in enumerate(LAYERS):
            run("x" * i + "b" + "x" * (11 - i))
    if args.greedy:
        cfg = list("b" * 12)
        best = run("".join(cfg))
        while best > 2e-3 and "b" in cfg:
            cands = []
            for i in range(12):
                for m in ("w", "a", "x"):
                    if MFMAS[m] <= MFMAS[cfg[i]]:
                        continue
                    c = cfg.copy()
                    c[i] = m
                    e = run("".join(c))
                    cands.append(((e - best) / (cost(c) - cost(cfg)), e, c))
            cands.sort(key=lambda t: t[0])
            _, best, cfg = cands[0]
            print("greedy ->", "".join(cfg), f"{best:.2e}", flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
