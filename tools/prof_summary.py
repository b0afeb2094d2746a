#!/usr/bin/env python3
"""Condense rocprofv3 outputs under gpurun_out/ into the small, committed summaries under profiles/.

usage: tools/prof_summary.py <tag> <out_prefix>
  reads  gpurun_out/prof_<tag>_kt/run_kernel_stats.csv          (--kernel-trace --stats)
         gpurun_out/prof_<tag>_<COUNTER>/run_counter_collection.csv  (one --pmc pass per counter)
  writes profiles/<out_prefix>_kernel_stats.csv  (engine kernels only, names shortened)
         profiles/<out_prefix>_pmc.csv           (per-kernel mean counter values per dispatch)
         profiles/traffic_<kernel>.json          (HBM bytes per launch = (FETCH_SIZE + WRITE_SIZE)·1024)
"""
import collections
import csv
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OURS = re.compile(r"(photometric_block_kernel|geometric_block_kernel|pair_kernel|cr_\w+|assemble\w*|band_\w+|"
                  r"skyline\w*|schur_\w+|linearize\w*|update\w*|reduce\w*|__amd_rocclr_copyBuffer)")


def short(name):
    m = re.search(r"(\w+_kernel|\w+Buffer)(<[^>]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:80]


def main(tag, prefix):
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    ks = os.path.join(ROOT, "gpurun_out", f"prof_{tag}_kt", "run_kernel_stats.csv")
    rows = [r for r in csv.DictReader(open(ks)) if OURS.search(r["Name"])]
    with open(os.path.join(ROOT, "profiles", f"{prefix}_kernel_stats.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "StdDev"])
        for r in rows:
            w.writerow([short(r["Name"]), r["Calls"], r["TotalDurationNs"], r["AverageNs"], r["MinNs"], r["MaxNs"], r["StdDev"]])
    pmc = collections.defaultdict(dict)
    for d in glob.glob(os.path.join(ROOT, "gpurun_out", f"prof_{tag}_*", "run_counter_collection.csv")):
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(d)):
            if OURS.search(r["Kernel_Name"]):
                agg[(short(r["Kernel_Name"]), r["Counter_Name"], r["Grid_Size"])].append(float(r["Counter_Value"]))
        for (k, c, g), v in agg.items():
            pmc[(k, g)][c] = (sum(v) / len(v), len(v))
    with open(os.path.join(ROOT, "profiles", f"{prefix}_pmc.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel", "Grid_Size", "Counter", "MeanPerDispatch", "Dispatches"])
        for (k, g), cs in sorted(pmc.items()):
            for c, (m, n) in sorted(cs.items()):
                w.writerow([k, g, c, m, n])
    for (k, g), cs in pmc.items():
        # the timed bench kernel: MODE 1 (full residual + Jacobian records), not the cost-only MODE 2 launch
        if ("FETCH_SIZE" in cs and "WRITE_SIZE" in cs and "photometric_block_kernel" in k
                and re.search(r"<0, 8, 1(, float)?(, 256)?>$", k)):  # pinhole, 8 lanes, MODE 1, fp32 records
            fetch, write = cs["FETCH_SIZE"][0] * 1024, cs["WRITE_SIZE"][0] * 1024
            out = {"kernel": k, "grid_size": int(g), "fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
                   "hbm_bytes_per_launch": fetch + write, "profile": f"profiles/{prefix}_pmc.csv",
                   "note": "FETCH_SIZE/WRITE_SIZE in KB from separate rocprofv3 --pmc passes of bench.py; reads are "
                           "byte gathers + narrow loads, not wide streams, so the gfx950 2x FETCH correction is not applied"}
            out.update(json.load(open(os.path.join(ROOT, "profiles", "workload.json"))) if os.path.exists(
                os.path.join(ROOT, "profiles", "workload.json")) else {})
            name = re.sub(r"<.*", "", k)
            json.dump(out, open(os.path.join(ROOT, "profiles", f"traffic_{name}.json"), "w"), indent=1)
            print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
