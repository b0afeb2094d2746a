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
                  r"skyline\w*|schur_\w+|linearize\w*|update\w*|reduce\w*|lm_\w+|dist_\w+|intr_\w+|export\w*|import\w*|pyramid\w*|"
                  r"__amd_rocclr_copyBuffer)")


def short(name):
    if name.startswith("_Z"):  # a mangled template instance (rocprofv3 did not demangle it): name<args>
        m = re.search(r"N_\d+([A-Za-z]\w*?_kernel\w*?)I(\w*?)EEv", name)
        if m:
            args = re.findall(r"Li(\d+)E|Lb([01])E|(DF16_)|(?<![A-Za-z])(f)(?=L|E|$)", m.group(2))
            out = []
            for num, b, h, f in args:
                out.append(num if num else ("true" if b == "1" else "false") if b else "_Float16" if h else "float")
            return f"{m.group(1)}<{', '.join(out)}>"
    m = re.search(r"(\w+_kernel|\w+Buffer)(<[^>]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:80]


def main(tag, prefix):
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    # per (kernel, grid size) from the kernel trace: one kernel runs at several sizes in a bench run (the C4 launch,
    # the 1/8 shard, the strong-scaling shard), and rocprofv3's own stats average them together
    kt = os.path.join(ROOT, "gpurun_out", f"prof_{tag}_kt", "run_kernel_trace.csv")
    durs = collections.defaultdict(list)
    for r in csv.DictReader(open(kt)):
        if OURS.search(r["Kernel_Name"]):
            durs[(short(r["Kernel_Name"]), int(r["Grid_Size_X"]))].append(
                int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    with open(os.path.join(ROOT, "profiles", f"{prefix}_kernel_stats.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel", "Grid_Size", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "StdDev"])
        for (k, g), d in sorted(durs.items(), key=lambda kv: -sum(kv[1])):
            m = sum(d) / len(d)
            sd = (sum((x - m) ** 2 for x in d) / len(d)) ** 0.5
            w.writerow([k, g, len(d), sum(d), f"{m:.1f}", min(d), max(d), f"{sd:.1f}"])
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
    # the timed bench kernel: MODE 1 (full residual + Jacobian records; not the cost-only MODE 2 launch) at the full
    # problem's size (the largest grid: the 1/8 shard and strong-scaling legs run the same kernel smaller)
    heads = [(k, g) for (k, g), cs in pmc.items()
             if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs and "photometric_block_kernel" in k
             and re.search(r"<0, 8, 1(, float)?(, 256)?>$", k)]  # pinhole, 8 lanes, MODE 1, fp32 records
    for (k, g) in sorted(heads, key=lambda kg: -int(kg[1]))[:1]:
        cs = pmc[(k, g)]
        if True:
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
