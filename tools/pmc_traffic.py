"""Per-launch HBM traffic of the MLP, sampling and compositing kernels from rocprofv3 --pmc CSVs.

    rocprofv3 --pmc FETCH_SIZE -d <dir_f> -o fetch --output-format csv -- python3 bench.py ...
    rocprofv3 --pmc WRITE_SIZE -d <dir_w> -o write --output-format csv -- python3 bench.py ...
    python tools/pmc_traffic.py <fetch csv> <write csv> bf16 > profiles/rN/traffic.json

FETCH_SIZE / WRITE_SIZE are in KiB.  On gfx950 FETCH_SIZE reports half the bytes of a
wide (16 B/lane) coalesced read, so it is doubled (MI355X_MICROARCH.md, HBM); WRITE_SIZE
is exact for 16 B/lane stores and float atomics.  Infinity-Cache hits are counted too.
"""
import collections
import csv
import json
import sys

LABELS = {
    "fwd_kernel<nerf::mlp::PBF16, true, false,": "mlp_fwd_train",
    "fwd_kernel<nerf::mlp::PF32, true, false,": "mlp_fwd_train",
    "fwd_kernel<nerf::mlp::PBF16, false, false,": "mlp_fwd",
    "fwd_kernel<nerf::mlp::PF32, false, false,": "mlp_fwd",
    "dx_kernel<nerf::mlp::PBF16>": "mlp_bwd_dx",
    "dx_kernel<nerf::mlp::PF32>": "mlp_bwd_dx",
    "dw_kernel<nerf::mlp::PBF16>": "mlp_bwd_dw",
    "dw_kernel<nerf::mlp::PF32>": "mlp_bwd_dw",
    "fwd_kernel<nerf::mlp::PBF3, true, false,": "mlp_fwd_train",
    "fwd_kernel<nerf::mlp::PBF3, false, false,": "mlp_fwd",
    "dx_kernel<nerf::mlp::PBF3>": "mlp_bwd_dx",
    "dx_kernel<nerf::mlp::PF32W>": "mlp_bwd_dx",  # (the wide dX, round 6)
    "dx_kernel<nerf::mlp::PBF3W>": "mlp_bwd_dx",
    "dx_kernel<nerf::mlp::PBF16W>": "mlp_bwd_dx",
    "dw_kernel<nerf::mlp::PBF3>": "mlp_bwd_dw",
    "fwd_kernel<nerf::mlp::PBF3W, true, false,": "mlp_fwd_train",  # (the wide bf16x3 forward, round 6)
    "fwd_kernel<nerf::mlp::PBF3W, false, false,": "mlp_fwd",
    "fwd_kernel<nerf::mlp::PF32W, true, false,": "mlp_fwd_train",  # (the wide fp32 training forward, round 6)
    "raygen_kernel(": "raygen",
    "stratified_kernel(": "sample_stratified",
    "sample_pdf_kernel(": "sample_pdf",
    "composite_pdf_kernel(": "composite_pdf",
    "composite_kernel<1, false>": "composite_fwd",
    "composite_kernel<3, false>": "composite_fwd",
    "composite_kernel<1, true>": "composite_bwd",
    "composite_kernel<3, true>": "composite_bwd",
}


def per_kernel(path, counter):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        for pat, label in LABELS.items():
            if pat in r["Kernel_Name"]:
                d[label].append(float(r["Counter_Value"]) * 1024.0)
    return {k: sum(v) / len(v) for k, v in d.items()}, {k: len(v) for k, v in d.items()}


def main(fetch_csv, write_csv, dtype, mlp_samples=524288):
    f, nf = per_kernel(fetch_csv, "FETCH_SIZE")
    w, _ = per_kernel(write_csv, "WRITE_SIZE")
    out = {}
    for k in sorted(set(f) | set(w)):
        rd = 2.0 * f.get(k, 0.0)
        out[k] = {"launches": nf.get(k, 0), "read_bytes": rd, "write_bytes": w.get(k, 0.0),
                  "traffic_bytes": rd + w.get(k, 0.0)}
    # the MLP launches' mean samples: 524,288 when each net's backward is one launch (coarse
    # 262,144 + fine 786,432); bench.py scales the MLP bytes to its own launches by it
    json.dump({"dtype": dtype, "unit": "bytes per launch", "mlp_samples_per_launch": mlp_samples, "kernels": out},
              sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3], *[int(x) for x in sys.argv[4:5]])
