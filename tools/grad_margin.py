"""Margin of the fp32 gradient parity test (tests/test_gpu_trained.py::test_loss_gradients_fp32)
for one build of libnerf_amd.so: per tensor, max |grad - reference| / (largest reference entry)
and the norm's relative error, for the 64-ray and the 4096-ray loss.  Prints one JSON line.

    python tools/grad_margin.py [--lib variants/x.so] [--dtype fp32]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "nerf-replication_amd")):
    sys.path.insert(0, p)
os.environ.setdefault("NERF_AMD_NO_ARGV", "1")

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=None)
    ap.add_argument("--dtype", default="fp32")
    args = ap.parse_args()
    from nerf_amd import _lib
    if args.lib:
        _lib.LIB_PATH = os.path.abspath(args.lib)
    from src.config import cfg
    from src.models.nerf.network import Network
    from src.train.trainers.nerf import NetworkWrapper
    dev = torch.device("cuda:0")
    g2 = np.load(os.path.join(ROOT, "tests", "golden", "golden_v2.npz"), allow_pickle=False)
    z = np.load(os.path.join(ROOT, "tests", "golden", "trained_v2.npz"), allow_pickle=False)
    cfg.task_arg.perturb = 0
    net = Network()
    net.load_state_dict({k: torch.from_numpy(z[k]) for k in z.files}, strict=True)
    net = net.to(dev)
    net.mlp_dtype = args.dtype
    wrapper = NetworkWrapper(net)
    out = {"lib": os.path.basename(args.lib or "libnerf_amd.so"), "dtype": args.dtype}
    for tag, key in (("grad64", "rays"), ("grad4096", "rays4096")):
        net.zero_grad()
        batch = {"rays": torch.from_numpy(g2[key]).to(dev)[None], "near": torch.tensor([2.0], device=dev),
                 "far": torch.tensor([6.0], device=dev), "rgbs": torch.from_numpy(g2[f"{tag}_gt"]).to(dev)}
        _, loss, stats = wrapper(batch)
        loss.backward()
        params = dict(net.named_parameters())
        worst = []
        for i, name in enumerate(g2[f"{tag}_names"]):
            g = params[str(name)].grad.reshape(-1).double().cpu()
            sel = g[torch.from_numpy(g2[f"{tag}_sel_idx"][i])].numpy()
            scale = float(g2[f"{tag}_absmax"][i]) + 1e-30
            err = float(np.abs(sel - g2[f"{tag}_sel_val"][i]).max())
            nrel = abs(float(torch.linalg.vector_norm(g)) - float(g2[f"{tag}_norms"][i])) / (float(g2[f"{tag}_norms"][i]) + 1e-30)
            worst.append((err / scale if err >= 1e-8 else 0.0, nrel, str(name)))
        worst.sort(reverse=True)
        out[tag] = {"loss_rel": [float(stats["loss_c"]) / float(g2[f"{tag}_loss"][0]) - 1,
                                 float(stats["loss_f"]) / float(g2[f"{tag}_loss"][1]) - 1],
                    "worst_sel": [[round(w[0], 7), w[2]] for w in worst[:5]],
                    "worst_norm": max(w[1] for w in worst)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
