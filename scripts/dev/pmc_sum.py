"""Per-kernel PMC summary (dispatch-averaged) of rocprofv3 counter CSVs."""
import collections, csv, glob, os, sys

FILT = os.environ.get("PMC_FILTER", "conv")

def load(d):
    f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    dur = collections.defaultdict(float)
    for r in csv.DictReader(open(f[0])):
        k = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").replace("commeff::", "").split("(")[0]
        if FILT not in k:
            continue
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        if r["Dispatch_Id"] not in disp[k]:
            disp[k].add(r["Dispatch_Id"])
            dur[k] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return agg, disp, dur

for i in range(1, len(sys.argv), 2):
    a1, d1, t1 = load(sys.argv[i]); a2, d2, t2 = load(sys.argv[i + 1])
    print("==", sys.argv[i])
    for k in sorted(a1):
        v = dict(a1[k]); v.update(a2.get(k, {}))
        n = len(d1[k]); us = t1[k] / n / 1e3
        wc = max(1.0, v.get("SQ_WAVE_CYCLES", 1))
        busy = v.get("GRBM_GUI_ACTIVE", 0)
        mf = v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0)
        print(f"{k[:58]:58s} n={n:3d} us={us:6.1f} wait={v.get('SQ_WAIT_ANY',0)/wc*100:5.1f}% "
              f"waitinst={v.get('SQ_WAIT_INST_ANY',0)/wc*100:5.1f}% active={v.get('SQ_ACTIVE_INST_ANY',0)/wc*100:5.1f}% "
              f"lds_wait={v.get('SQ_WAIT_INST_LDS',0)/wc*100:5.1f}% "
              f"ldscf={v.get('SQ_LDS_BANK_CONFLICT',0)/max(1,v.get('SQ_LDS_IDX_ACTIVE',1))*100:5.1f}% "
              f"mfma={100*mf/max(1,128*busy):6.1f}% valu/wave={v.get('SQ_INSTS_VALU',0)/max(1,v.get('SQ_WAVES',1)):8.0f} "
              f"salu/wave={v.get('SQ_INSTS_SALU',0)/max(1,v.get('SQ_WAVES',1)):7.0f} lds/wave={v.get('SQ_INSTS_LDS',0)/max(1,v.get('SQ_WAVES',1)):7.0f}")
