"""Effective clock per kernel from a rocprofv3 --pmc GRBM_GUI_ACTIVE run:
GRBM_GUI_ACTIVE (summed over the 8 XCDs) / 8 / dispatch wall time
(MI355X_MICROARCH.md 'DVFS give-back'; reads high on dispatches < ~0.3 ms),
plus MFMA busy share when SQ_VALU_MFMA_BUSY_CYCLES is in the same pass."""
import collections
import csv
import glob
import sys


def main(d, filt=""):
    f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)[0]
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")
        k = k.replace("commeff::", "").split("(")[0]
        if filt not in k:
            continue
        key = (k, r["Dispatch_Id"])
        per[key][r["Counter_Name"]] += float(r["Counter_Value"])
        per[key]["dur_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    agg = collections.defaultdict(list)
    for (k, _), v in per.items():
        agg[k].append(v)
    print(f"{'kernel':60s} {'n':>4s} {'us':>7s} {'GHz':>6s} {'mfma%':>6s}")
    for k, vs in sorted(agg.items(), key=lambda kv: -sum(v["dur_ns"] for v in kv[1])):
        dur = sum(v["dur_ns"] for v in vs)
        grbm = sum(v.get("GRBM_GUI_ACTIVE", 0) for v in vs)
        mf = sum(v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) for v in vs)
        ghz = grbm / 8 / dur if dur else 0
        print(f"{k[:60]:60s} {len(vs):4d} {dur / len(vs) / 1e3:7.1f} {ghz:6.2f} "
              f"{100 * mf / max(1, 128 * grbm):6.1f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
