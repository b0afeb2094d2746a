#!/usr/bin/env python3
"""Per-iteration kernel timeline of a pba_solve kernel trace (rocprofv3 --kernel-trace: its CSV, or the rocpd
SQLite database rocprofv3 writes by default): the kernels of one LM trial in launch order with their durations and the
idle gaps before them.  Diagnostic.
    python tools/gn_trace.py gpurun_out/<dir>/run_kernel_trace.csv|<name>_results.db [trial]
(trial: the index of the trial's schur_kernel launch in the trace; default the second-to-last trial)"""
import csv
import sys

if sys.argv[1].endswith(".db"):
    import sqlite3
    db = sqlite3.connect(sys.argv[1])
    rows = [{"Kernel_Name": n, "Start_Timestamp": s, "End_Timestamp": e}
            for n, s, e in db.execute("select name, start, end from kernels")]
else:
    rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
first = "schur_gate_kernel" if any("schur_gate_kernel" in r["Kernel_Name"] for r in rows) else "schur_kernel"
idx = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
if len(idx) < 4:
    sys.exit("fewer than 4 trials in the trace")
k = int(sys.argv[2]) if len(sys.argv) > 2 else len(idx) - 3
a, b = idx[k], idx[k + 1]
prev = int(rows[a - 1]["End_Timestamp"])
tot_k = tot_g = 0.0
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap, dur = (s - prev) / 1e3, (e - s) / 1e3
    prev = e
    tot_k += dur
    tot_g += gap
    print(f"{r['Kernel_Name'][:70]:70s} gap {gap:7.2f}  dur {dur:7.2f}")
print(f"kernels {tot_k:.1f} us + gaps {tot_g:.1f} us = {tot_k + tot_g:.1f} us per trial")
