"""Stage isolation for the render_video golden frames (tests/golden/golden_v3.npz): render the
reference's rays with the fp32 path, then for the worst rays feed each HIP stage the oracle's
own inputs (coarse MLP on the oracle's points, composite on the oracle's raw, sample_pdf on the
oracle's weights, fine MLP on the oracle's fine points) and report each stage's output error
and what it does to rgb_map_f when spliced into the oracle.  Diagnostic only (tests-side code:
imports the oracle)."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "nerf-replication_amd")]
os.environ.setdefault("NERF_AMD_NO_ARGV", "1")

from nerf_amd import ops  # noqa: E402
from oracle import nerf_oracle as O  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    z = np.load(os.path.join(ROOT, "tests/golden/trained_v2.npz"))
    st = {k: torch.from_numpy(z[k]) for k in z.files}
    g3 = np.load(os.path.join(ROOT, "tests/golden/golden_v3.npz"))
    from src.config import cfg
    from src.models.nerf.network import Network
    from src.models.nerf.renderer.volume_renderer import Renderer
    cfg.task_arg.perturb = 0
    torch.manual_seed(0)
    net = Network()
    net.load_state_dict(st, strict=True)
    net = net.to(dev)
    r = Renderer(net)
    C, Fn = O.split_params(st, "model"), O.split_params(st, "model_fine")
    near, far = torch.tensor([2.0]), torch.tensor([6.0])
    rep = {}
    for k in g3["frames"].tolist():
        rays = torch.from_numpy(g3[f"video_rays_{k}"])
        ref = g3[f"video_rgb_{k}"]
        with torch.no_grad():
            out = r.render({"rays": rays.to(dev), "near": near.to(dev), "far": far.to(dev)})
        got = out["rgb_map_f"].cpu().numpy()
        err = np.abs(got - ref).max(1)
        worst = np.argsort(-err)[:4]
        rows = []
        for i in worst.tolist():
            ry = rays[i:i + 1]
            o = O.render(C, Fn, ry, near, far, keep=True)
            d = ry[:, 3:6]
            vd = d / torch.norm(d, dim=-1, keepdim=True)
            pts_c = ry[:, None, :3] + d[:, None] * o["z_vals"][..., None]
            pts_f = ry[:, None, :3] + d[:, None] * o["z_vals_f"][..., None]
            with torch.no_grad():
                raw_c = ops.mlp(net.model.packer(), pts_c.to(dev), vd.to(dev), 64).reshape(1, 64, 4).cpu()
                raw_f = ops.mlp(net.model_fine.packer(), pts_f.to(dev), vd.to(dev), 192).reshape(1, 192, 4).cpu()
                rgb_cg, _, _, w_cg = ops.composite(o["raw_c"].to(dev), o["z_vals"].to(dev), d.to(dev))
                pdf = ops.sample_pdf(o["z_vals"].to(dev), o["weights_c"].to(dev), 128, det=True, debug=True)
                rgb_fg, dep_fg, _, _ = ops.composite(o["raw_f"].to(dev), o["z_vals_f"].to(dev), d.to(dev))
            # splice our coarse raw into the oracle: the effect on rgb_f through the CDF
            rgb_c2, _, _, w_c2 = O.composite(raw_c, o["z_vals"], d)
            zmid = 0.5 * (o["z_vals"][..., 1:] + o["z_vals"][..., :-1])
            pdf2 = O.sample_pdf(zmid, w_c2[..., 1:-1], 128, det=True)
            zf2, _ = torch.sort(torch.cat([o["z_vals"], pdf2.samples], -1), -1)
            pf2 = ry[:, None, :3] + d[:, None] * zf2[..., None]
            rf2 = O.network_forward(Fn, pf2, vd)
            rgb_f_spliced_c = O.composite(rf2, zf2, d)[0]
            # splice our fine raw into the oracle
            rgb_f_spliced_f = O.composite(raw_f, o["z_vals_f"], d)[0]
            sig = lambda a: a[..., 3]  # noqa: E731
            rows.append({
                "ray": i, "err_rgb_f": float(err[i]), "got": got[i].tolist(), "ref": ref[i].tolist(),
                "coarse_raw_maxabs": float((raw_c - o["raw_c"]).abs().max()),
                "coarse_sigma_maxrel": float(((sig(raw_c) - sig(o["raw_c"])).abs() / sig(o["raw_c"]).abs().clamp_min(1e-3)).max()),
                "fine_raw_maxabs": float((raw_f - o["raw_f"]).abs().max()),
                "composite_c_w_maxabs": float((w_cg.cpu() - o["weights_c"]).abs().max()),
                "composite_f_rgb_err": float((rgb_fg.cpu() - o["rgb_map_f"]).abs().max()),
                "pdf_zfine_maxabs": float((pdf["z_fine"].cpu() - o["z_vals_f"]).abs().max()),
                "pdf_inds_equal": bool(torch.equal(pdf["inds"].cpu().long(), o["inds"])),
                "oracle_with_our_coarse_raw_rgb_f_err": float((rgb_f_spliced_c - o["rgb_map_f"]).abs().max()),
                "oracle_with_our_fine_raw_rgb_f_err": float((rgb_f_spliced_f - o["rgb_map_f"]).abs().max()),
                "oracle_vs_ref": float(np.abs(o["rgb_map_f"].numpy() - ref[i]).max()),
            })
        rep[k] = {"max_err": float(err.max()), "n_over_1e-4": int((np.abs(got - ref) > 1e-4).sum()), "worst": rows}
        print(k, json.dumps(rep[k]["worst"][0]), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "diag_video.json"), "w") as f:
        json.dump(rep, f, indent=1)


if __name__ == "__main__":
    main()
