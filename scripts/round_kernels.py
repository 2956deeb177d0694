#!/usr/bin/env python
"""Per-round kernel breakdown from a rocprofv3 ``--kernel-trace`` CSV.

Rounds are delimited by a marker kernel that runs once per round (default:
the planned-sketch P1 encode).  Reports, averaged over the last N rounds:
busy time per kernel name, kernel count, and idle gaps on the GPU (time the
queue had nothing to run -- i.e. host-bound stretches).

    python scripts/round_kernels.py gpurun_out/rocprof/bench_kernel_trace.csv --rounds 8
"""
import argparse
import collections
import csv
import re


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\((?!anon).*", "", name)  # drop argument lists
    name = name.replace("commeff::", "")
    name = name.replace("void ", "")
    return name[:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="enc_p1_kernel")
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--tail-ms", type=float, default=0.0,
                    help="no marker: take the kernels of the trace's last TAIL_MS ms "
                         "(e.g. rounds * ms_per_round of the timed steps)")
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    if a.tail_ms > 0:
        t_end = max(r[1] for r in rows)
        sel = [r for r in rows if r[0] >= t_end - a.tail_ms * 1e6]
    else:
        starts = [i for i, r in enumerate(rows) if a.marker in r[2]]
        if len(starts) < a.rounds + 1:
            raise SystemExit(f"only {len(starts)} marker kernels")
        lo, hi = starts[-a.rounds - 1], starts[-1]
        sel = rows[lo:hi]
    n = a.rounds
    wall = (sel[-1][1] - sel[0][0]) / n
    busy = collections.Counter()
    calls = collections.Counter()
    idle = 0
    end = sel[0][0]
    for s, e, k in sel:
        if s > end:
            idle += s - end
        end = max(end, e)
        busy[short(k)] += e - s
        calls[short(k)] += 1
    tot = sum(busy.values())
    print(f"# rounds={n} wall/round={wall / 1e3:.1f}us busy/round={tot / n / 1e3:.1f}us "
          f"idle/round={idle / n / 1e3:.1f}us kernels/round={len(sel) / n:.1f}")
    print("# us/round  calls/round  kernel")
    for k, v in busy.most_common(a.top):
        print(f"{v / n / 1e3:9.1f} {calls[k] / n:6.1f}  {k}")


if __name__ == "__main__":
    main()
