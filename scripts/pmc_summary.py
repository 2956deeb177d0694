#!/usr/bin/env python
"""Per-kernel hardware-counter summary of rocprofv3 ``--pmc`` passes.

Each pass is one rocprofv3 run (``--pmc <counters> --kernel-trace
--output-format csv``) of the same program; this joins every pass's
``*_counter_collection.csv`` with its ``*_kernel_trace.csv`` (durations, by
Dispatch_Id), averages per dispatch per kernel name, and derives:

  mfma%    SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x kernel cycles); a
           v_mfma_f32_32x32x16_bf16 adds 32 busy cycles, so 100 % = the
           2.5 PFLOP/s dense bf16 peak at the kernel's own clock
  clk GHz  GRBM_GUI_ACTIVE / 8 XCDs / duration (reads high below ~0.3 ms)
  lds-cf%  SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (extra cycles per LDS cycle)
  rd, wr   FETCH_SIZE x 2 (gfx950 tallies a wide coalesced read at half its
           bytes, MI355X_MICROARCH.md) and WRITE_SIZE, in MB per dispatch;
  GB/s     (rd + wr) / duration
  L2 hit%  TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)
  wait%    SQ_WAIT_ANY / SQ_WAVE_CYCLES (waves parked on s_waitcnt/barrier)

    python scripts/pmc_summary.py gpurun_out/pmc/p1 gpurun_out/pmc/p2 ... --top 25

``--marker K --rounds N`` keeps only the dispatches from the N-th last launch
of kernel K on (the timed rounds; plan building and warm-up excluded).
"""
import argparse
import collections
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from round_kernels import short  # noqa: E402

SIMDS = 1024  # 256 CUs x 4


def load_pass(d, marker=None, rounds=0):
    cc = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not cc:
        raise SystemExit(f"{d}: no counter_collection.csv")
    dur = {}
    for fn in kt:
        with open(fn) as f:
            for r in csv.DictReader(f):
                dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    vals = collections.defaultdict(dict)  # dispatch -> counter -> value
    names = {}
    for fn in cc:
        with open(fn) as f:
            for r in csv.DictReader(f):
                did = r["Dispatch_Id"]
                names[did] = short(r["Kernel_Name"])
                c = r["Counter_Name"]
                vals[did][c] = vals[did].get(c, 0.0) + float(r["Counter_Value"])
                if did not in dur and "End_Timestamp" in r and r.get("Start_Timestamp"):
                    dur[did] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    if marker and rounds:
        marks = sorted(int(k) for k, n in names.items() if marker in n)
        if len(marks) >= rounds:
            lo = marks[-rounds]
            vals = {k: v for k, v in vals.items() if int(k) >= lo}
    return names, vals, dur


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("passes", nargs="+")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--marker", default=None)
    ap.add_argument("--rounds", type=int, default=0)
    a = ap.parse_args()
    # kernel -> counter -> [sum, n]; kernel -> [dur sum, n] (per pass: durations
    # of each pass's own dispatches, counters collected there)
    ctr = collections.defaultdict(lambda: collections.defaultdict(lambda: [0.0, 0]))
    durs = collections.defaultdict(lambda: [0.0, 0])
    per_pass_dur = collections.defaultdict(dict)
    for p in a.passes:
        names, vals, dur = load_pass(p, a.marker, a.rounds)
        pd = collections.defaultdict(lambda: [0.0, 0])
        for did, cs in vals.items():
            if did not in names:
                continue
            k = names[did]
            for c, v in cs.items():
                ctr[k][c][0] += v
                ctr[k][c][1] += 1
                if c in ("GRBM_GUI_ACTIVE", "FETCH_SIZE", "WRITE_SIZE"):
                    ctr[k]["_dur_" + c][0] += dur.get(did, 0.0)
                    ctr[k]["_dur_" + c][1] += 1
            if did in dur:
                durs[k][0] += dur[did]
                durs[k][1] += 1
                pd[k][0] += dur[did]
                pd[k][1] += 1
        per_pass_dur[p] = pd

    def m(k, c):
        s, n = ctr[k].get(c, (0.0, 0))
        return s / n if n else None

    order = sorted(durs, key=lambda k: -durs[k][0])
    hdr = (f"{'kernel':60s} {'n':>5s} {'us':>8s} {'mfma%':>6s} {'clkGHz':>6s} {'lds-cf%':>7s} "
           f"{'rdMB':>8s} {'wrMB':>8s} {'GB/s':>7s} {'L2hit%':>6s} {'wait%':>6s}")
    print("# per-dispatch means over every profiled dispatch of the kernel (counters of")
    print("# each pass on that pass's own dispatches); '-' = counter not collected")
    print(hdr)

    def f(x, fmt):
        return format(x, fmt) if x is not None else "-"

    for k in order[:a.top]:
        n = durs[k][1]
        us = durs[k][0] / n * 1e6
        grbm = m(k, "GRBM_GUI_ACTIVE")
        dg = m(k, "_dur_GRBM_GUI_ACTIVE")
        cyc = grbm / 8 if grbm else None
        mf = m(k, "SQ_VALU_MFMA_BUSY_CYCLES")
        mfma = 100 * mf / (SIMDS * cyc) if (mf is not None and cyc) else None
        clk = cyc / dg / 1e9 if (cyc and dg) else None
        bc, la = m(k, "SQ_LDS_BANK_CONFLICT"), m(k, "SQ_LDS_IDX_ACTIVE")
        ldscf = 100 * bc / la if (bc is not None and la) else None
        fs, ws = m(k, "FETCH_SIZE"), m(k, "WRITE_SIZE")
        rd = 2 * fs * 1024 / 1e6 if fs is not None else None
        wr = ws * 1024 / 1e6 if ws is not None else None
        bw = None
        if rd is not None and wr is not None:
            t = (m(k, "_dur_FETCH_SIZE") + m(k, "_dur_WRITE_SIZE")) / 2
            bw = (rd + wr) / 1e3 / t if t else None
        h, mi = m(k, "TCC_HIT_sum"), m(k, "TCC_MISS_sum")
        hit = 100 * h / (h + mi) if (h is not None and mi is not None and h + mi) else None
        wa, wc = m(k, "SQ_WAIT_ANY"), m(k, "SQ_WAVE_CYCLES")
        wait = 100 * wa / wc if (wa is not None and wc) else None
        print(f"{k[:60]:60s} {n:5d} {us:8.1f} {f(mfma, '6.1f'):>6s} {f(clk, '6.2f'):>6s} "
              f"{f(ldscf, '7.1f'):>7s} {f(rd, '8.1f'):>8s} {f(wr, '8.1f'):>8s} {f(bw, '7.0f'):>7s} "
              f"{f(hit, '6.1f'):>6s} {f(wait, '6.1f'):>6s}")


if __name__ == "__main__":
    main()
