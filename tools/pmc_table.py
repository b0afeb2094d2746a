#!/usr/bin/env python3
"""Per-kernel mean counter values per dispatch from tools/pmc_probe.sh passes (gpurun_out/pmc_<tag>_<i>/), plus
derived per-wave instruction counts and busy fractions.  Diagnostic.
    python tools/pmc_table.py <tag> [<tag> ...]"""
import collections
import csv
import glob
import sys


def load(tag):
    """{kernel name: {counter: mean per dispatch}} over the tag's passes (a pass may cover several kernels)"""
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(f"gpurun_out/pmc_{tag}_*/run_counter_collection.csv")):
        per = collections.defaultdict(float)  # (kernel, dispatch, counter) -> summed over dimensions
        for r in csv.DictReader(open(f)):
            per[(r["Kernel_Name"], r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (k, d, c), v in per.items():
            vals[k][c].append(v)
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in vals.items()}


def show(tag, name, m):
    print(f"== {tag}: {name[:90] if name else '?'}")
    for c in sorted(m):
        print(f"   {c:24s} {m[c]:16.1f}")
    w = m.get("SQ_WAVES", 0)
    if w:
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"):
            if c in m:
                print(f"   {c + ' / wave':24s} {m[c] / w:16.1f}")
    if "GRBM_GUI_ACTIVE" in m and "SQ_BUSY_CYCLES" in m:
        print(f"   GRBM_GUI_ACTIVE us       {m['GRBM_GUI_ACTIVE'] / 2400:16.2f}  (at 2.4 GHz)")
    for c in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_SCA", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
        if c in m and "SQ_WAVE_CYCLES" in m:
            print(f"   {c + ' / wave cyc':30s} {m[c] / m['SQ_WAVE_CYCLES']:10.3f}")
    if "FETCH_SIZE" in m:
        print(f"   FETCH MB {m['FETCH_SIZE'] * 1024 / 1e6:.1f}  WRITE MB {m.get('WRITE_SIZE', 0) * 1024 / 1e6:.1f}")


for tag in sys.argv[1:]:
    for name, m in sorted(load(tag).items()):
        show(tag, name, m)
