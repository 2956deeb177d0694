#!/usr/bin/env python
"""Summarise gpurun_out/pmc/NAME.{sq,tcc,kt} (counters per kernel + times)."""
import collections
import csv
import sys

name = sys.argv[1]
root = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out/pmc"
filt = sys.argv[3] if len(sys.argv) > 3 else "commeff"
agg = collections.OrderedDict()
for part in ("sq", "tcc", "mfma"):
    try:
        rows = csv.DictReader(open(f"{root}/{name}.{part}/run_counter_collection.csv"))
    except FileNotFoundError:
        continue
    for r in rows:
        n = r["Kernel_Name"]
        if filt not in n:
            continue
        n = n.replace("void ", "").replace("commeff::(anonymous namespace)::", "").split("(")[0][:48]
        agg.setdefault((n, r["Grid_Size"]), collections.defaultdict(list))[r["Counter_Name"]].append(
            float(r["Counter_Value"]))
for (n, grid), d in agg.items():
    dd = {c: sum(x) / len(x) for c, x in d.items()}
    wc = dd.get("SQ_WAVE_CYCLES", 1) or 1
    w = dd.get("SQ_WAVES", 1) or 1
    hit, miss = dd.get("TCC_HIT_sum", 0), dd.get("TCC_MISS_sum", 0)
    print(f"{n:48s} grid={grid:>9s} waves={w:7.0f} wait={dd.get('SQ_WAIT_ANY', 0) / wc:.2f} "
          f"waitinst={dd.get('SQ_WAIT_INST_ANY', 0) / wc:.2f} active={dd.get('SQ_ACTIVE_INST_ANY', 0) / wc:.2f} "
          f"valu/wave={dd.get('SQ_INSTS_VALU', 0) / w:.0f} lds/wave={dd.get('SQ_INSTS_LDS', 0) / w:.0f} "
          f"ldsconf={dd.get('SQ_LDS_BANK_CONFLICT', 0):.3g} hit%={100 * hit / max(1, hit + miss):.0f} miss={miss:.3g}"
          + (f" mfma%={100 * dd['SQ_VALU_MFMA_BUSY_CYCLES'] / (dd['GRBM_GUI_ACTIVE'] * 1024):.1f}"
             if dd.get("GRBM_GUI_ACTIVE") else ""))
try:
    for r in csv.DictReader(open(f"{root}/{name}.kt/run_kernel_stats.csv")):
        if filt in r["Name"]:
            print(f"{float(r['AverageNs']) / 1e3:9.1f} us x{r['Calls']:>4s}  {r['Name'][:100]}")
except FileNotFoundError:
    pass
