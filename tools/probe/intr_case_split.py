#!/usr/bin/env python3
"""Per-case kernel breakdown of tools/probe/intr_probe.py's rocprofv3 kernel trace: the trace is split at every 12th
intr_rows_kernel launch (each case runs 2 + 10 LM iterations) into C3 one camera, C3 two cameras and C4 one camera, and
each kernel's time per LM iteration is printed.

    python3 tools/probe/intr_case_split.py gpurun_out/<dir>/run_kernel_trace.csv
"""
import csv, collections, sys
rows=list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
idx=[i for i,r in enumerate(rows) if 'intr_rows' in r['Kernel_Name']]
bounds=[idx[0], idx[12], idx[24], len(rows)]
names=['C3 1 cam','C3 2 cams','C4 1 cam']
for c in range(3):
    d=collections.defaultdict(list)
    for r in rows[bounds[c]:bounds[c+1]]:
        k=r['Kernel_Name'].replace('void ','').replace('(anonymous namespace)::','').split('(')[0]
        d[k].append((int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3)
    tot=sum(sum(v) for v in d.values())/12
    print(f"{names[c]}: {tot:.1f} us of kernels per iteration")
    for k,v in sorted(d.items(), key=lambda kv:-sum(kv[1])):
        if sum(v)/12 > 3: print(f"   {k[:45]:45s} n {len(v):4d} avg {sum(v)/len(v):7.1f} us  per iter {sum(v)/12:7.1f}")
