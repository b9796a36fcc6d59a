"""Compare config-3 PSNR curves of two MLP precisions (tools/psnr_curve.py outputs).

    python tools/psnr_compare.py profiles/r3/psnr_curve_200k_fp32.json profiles/r3/psnr_curve_200k_bf16.json

Prints per-checkpoint deltas (b - a), their mean, the mean over the last third and the best / final
values of each curve (held-out PSNR of one training run per precision: checkpoint-to-checkpoint
noise of a run at lr 5e-4 with perturbed samples is about +-1 dB, so means are what compare)."""
import json
import sys

import numpy as np


def curve(path):
    d = json.load(open(path))
    key = [k for k in d if k.startswith("psnr_curve_")][0]
    return key[len("psnr_curve_"):], {int(s): float(p) for s, p in d[key]}, d


def main(pa, pb):
    na, a, _ = curve(pa)
    nb, b, _ = curve(pb)
    steps = sorted(set(a) & set(b))
    delta = [b[s] - a[s] for s in steps]
    third = max(1, len(steps) // 3)
    out = {"a": na, "b": nb, "checkpoints": len(steps), "last_step": steps[-1] if steps else None,
           "mean_delta_db": round(float(np.mean(delta)), 3),
           "mean_delta_db_last_third": round(float(np.mean(delta[-third:])), 3),
           "mean_a_last_third": round(float(np.mean([a[s] for s in steps[-third:]])), 3),
           "mean_b_last_third": round(float(np.mean([b[s] for s in steps[-third:]])), 3),
           f"best_{na}": max(a.values()), f"best_{nb}": max(b.values()),
           f"final_{na}": a[steps[-1]], f"final_{nb}": b[steps[-1]],
           "delta_db": [round(x, 3) for x in delta]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
