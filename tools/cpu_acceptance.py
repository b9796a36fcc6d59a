"""BASELINE.md section 4 acceptance of the CPU restatement (build container only: it imports
the reference from /root/reference the way tests/golden/make_golden.py does).

Times, interleaved on the same host and thread count, config 1 (1024 rays, perturb 0,
seed-0 weights, forward + backward; and the full step with clip 40 + Adam) through
  * the reference itself (make_renderer / make_network from /root/reference), and
  * the oracle restatement (oracle/nerf_oracle.py, which bench.py's cpu_baseline times),
and writes profiles/r2/cpu_acceptance.json with both rates, their ratio, and the survey's
probed 528.8 / 487.6 rays/s for comparison.

    python tools/cpu_acceptance.py [--threads 8] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--rays", type=int, default=1024)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r2", "cpu_acceptance.json"))
    args = ap.parse_args()
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    sys.path.insert(0, ROOT)
    import make_golden  # noqa: E402  (reference import recipe)
    cfg, make_network, make_renderer = make_golden._import_reference()  # cwd = /root/reference
    import torch
    from oracle import nerf_oracle as O
    torch.set_num_threads(args.threads)

    pose = O.pose_spherical(30.0, -30.0, 4.0)
    o, d = O.get_rays(800, 800, O.focal_from_angle(800, 0.6911112070083618), pose)
    idx = torch.randint(0, 800 * 800, (args.rays,), generator=torch.Generator().manual_seed(0))
    rays = torch.cat([o.reshape(-1, 3)[idx], d.reshape(-1, 3)[idx]], 1)
    gt = torch.rand(args.rays, 3, generator=torch.Generator().manual_seed(1))
    near, far = torch.tensor([2.0]), torch.tensor([6.0])

    torch.manual_seed(0)
    ref_net = make_network(cfg)
    ref_r = make_renderer(cfg, ref_net)
    ref_opt = torch.optim.Adam([{"params": [p]} for p in ref_net.parameters()], lr=5e-4, eps=1e-8)
    state = {k: v.clone().requires_grad_(True) for k, v in O.seeded_network_state(0).items()}
    C, Fn = O.split_params(state, "model"), O.split_params(state, "model_fine")
    or_opt = torch.optim.Adam([{"params": [p]} for p in state.values()], lr=5e-4, eps=1e-8)
    import contextlib
    import io

    def ref_step(full):
        ref_opt.zero_grad()
        with contextlib.redirect_stdout(io.StringIO()):  # the reference prints "Render time"
            ret = ref_r.render({"rays": rays[None], "near": near, "far": far})
        loss = torch.nn.functional.mse_loss(ret["rgb_map_c"], gt) + torch.nn.functional.mse_loss(ret["rgb_map_f"], gt)
        loss.backward()
        if full:
            torch.nn.utils.clip_grad_value_(list(ref_net.parameters()), 40.0)
            ref_opt.step()

    def oracle_step(full):
        or_opt.zero_grad()
        ret = O.render(C, Fn, rays, near, far)
        O.loss_fn(ret, gt)[0].backward()
        if full:
            torch.nn.utils.clip_grad_value_(list(state.values()), 40.0)
            or_opt.step()

    res = {}
    for full in (False, True):
        tag = "full_step" if full else "fwd_bwd"
        times = {"reference": [], "oracle": []}
        ref_step(full)
        oracle_step(full)
        for _ in range(args.reps):  # interleaved: host noise hits both alike
            for name, fn in (("reference", ref_step), ("oracle", oracle_step)):
                t0 = time.perf_counter()
                fn(full)
                times[name].append(time.perf_counter() - t0)
        rr = args.rays / (sum(times["reference"]) / args.reps)
        ro = args.rays / (sum(times["oracle"]) / args.reps)
        res[tag] = {"reference_rays_per_s": round(rr, 1), "oracle_rays_per_s": round(ro, 1),
                    "oracle_over_reference": round(ro / rr, 3), "within_15pct": abs(ro / rr - 1) <= 0.15,
                    "survey_probe_rays_per_s": 528.8 if not full else 487.6}
        print(tag, json.dumps(res[tag]), flush=True)
    out = {"threads": args.threads, "rays": args.rays, "reps": args.reps, "torch": torch.__version__,
           "cpu_count": os.cpu_count(), "results": res,
           "note": "anomaly mode off on both; the reference's set_detect_anomaly(True) (train.py:23) is a "
                   "train.py setting, not part of render"}
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", args.out)


if __name__ == "__main__":
    main()
