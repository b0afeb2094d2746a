#!/usr/bin/env python3
"""Print a run's bench line summary and the engine kernels' rocprof averages (gpurun_out/, diagnostic)."""
import csv, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1]
d = json.loads(open(os.path.join(ROOT, "gpurun_out", f"bench_{tag}.log")).read().strip().split("\n")[-1])
print(f"{d['value'] / 1e9:.3f} Gblk/s  step {d['ms_per_step'] * 1e3:.1f} us  kernel(ev) {d['roofline']['kernel_avg_us']:.1f} us"
      f"  frac {d['roofline']['frac']:.3f}  GN {d['gn']['ms_per_iteration']:.3f} ms {d['gn']['breakdown_ms_per_iteration']}")
for x in csv.DictReader(open(os.path.join(ROOT, "gpurun_out", f"prof_{tag}_kt", "run_kernel_stats.csv"))):
    if "at::native" not in x["Name"]:
        print(f"  {x['Name'][:72]:72s} {x['Calls']:>4s} {float(x['AverageNs']) / 1e3:8.2f} us")
