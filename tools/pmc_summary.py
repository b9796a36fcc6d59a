"""Summarise rocprofv3 --pmc CSVs per kernel: counters per launch, ratios to SQ_WAVE_CYCLES.
    python tools/pmc_summary.py gpurun_out/pmcA/p_counter_collection.csv [more.csv ...]"""
import collections
import csv
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(float))
launches = collections.defaultdict(set)
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        if "nerf::" not in k:
            continue
        k = k.split("(")[0].replace("void ", "").replace("nerf::mlp::", "")
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        launches[k].add((path, r["Dispatch_Id"]))
for k, v in agg.items():
    wc = v.get("SQ_WAVE_CYCLES", 1.0)
    print(f"{k}  launches={len(launches[k])}")
    for c, x in sorted(v.items()):
        print(f"    {c:28s} {x:16.0f}  /wave_cycles {x / wc:8.3f}")
