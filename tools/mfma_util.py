"""MFMA utilisation of the MLP kernels from rocprofv3 --pmc CSVs (tools/gpu_pmc_mlp.sh).

    python tools/mfma_util.py <pass-A counter csv> <pass-B counter csv> > profiles/rN/mfma_util.json

Pass A holds SQ_VALU_MFMA_BUSY_CYCLES, pass B GRBM_GUI_ACTIVE and SQ_INSTS_MFMA (each pass is
its own run of tools/mlp_bench.py, so launches are matched by kernel name and order).
Per launch:
- mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8): the share of
  SIMD cycles the matrix cores were busy.  GRBM_GUI_ACTIVE sums the 8 XCDs (MI355X_MICROARCH.md).
  SQ_VALU_MFMA_BUSY_CYCLES counts 32 cycles per 32x32x16 bf16 MFMA, which is the full-rate
  2.5 PFLOP/s issue slot of one SIMD.
- clock_ghz = GRBM_GUI_ACTIVE / 8 / the dispatch's duration (its Start/End timestamps).
- mfma_tflop_issued = SQ_INSTS_MFMA x 32x32x16x2: matrix work issued, including the padding of
  the 63/90-wide PE inputs and the 4-row output heads to 32-row tiles.
"""
import collections
import csv
import json
import sys

SIMDS = 1024
FLOP_PER_MFMA = 32 * 32 * 16 * 2


def per_launch(path):
    d = collections.defaultdict(lambda: collections.defaultdict(dict))
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        if "nerf::mlp::" not in k:
            continue
        k = k.split("(")[0].replace("void ", "").replace("nerf::mlp::", "")
        disp = int(r["Dispatch_Id"])
        e = d[k][disp]
        e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        e["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return {k: [v[i] for i in sorted(v)] for k, v in d.items()}


def main(a_csv, b_csv):
    A, B = per_launch(a_csv), per_launch(b_csv)
    out = {}
    for k in sorted(A):
        if k not in B or "pack" in k:
            continue
        rows = []
        for a, b in zip(A[k], B[k]):
            cyc = b["GRBM_GUI_ACTIVE"] / 8.0
            rows.append({"ms_a": a["ns"] / 1e6, "mfma_busy_frac": a["SQ_VALU_MFMA_BUSY_CYCLES"] / (SIMDS * cyc),
                         "clock_ghz": cyc / b["ns"], "mfma_tflop_issued": b["SQ_INSTS_MFMA"] * FLOP_PER_MFMA / 1e12})
        big = [r for r in rows if r["ms_a"] > 0.3]  # short dispatches read the clock high
        use = big or rows
        out[k] = {"launches": len(rows),
                  **{f: round(sum(r[f] for r in use) / len(use), 4) for f in rows[0]}}
    json.dump({"source": "rocprofv3 --pmc, tools/gpu_pmc_mlp.sh (tools/mlp_bench.py, 786,432 samples)",
               "kernels": out}, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
