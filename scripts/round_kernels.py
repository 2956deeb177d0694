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
    ap.add_argument("--per-round", type=int, default=0,
                    help="also print every round's wall / busy / idle and the PER_ROUND "
                         "largest kernels' times, from the first marker on")
    ap.add_argument("--gaps", type=int, default=0,
                    help="print the GAPS largest idle gaps per round, by (previous kernel -> "
                         "next kernel), averaged over the selected rounds")
    ap.add_argument("--tail-ms", type=float, default=0.0,
                    help="no marker: take the kernels of the trace's last TAIL_MS ms "
                         "(e.g. rounds * ms_per_round of the timed steps)")
    ap.add_argument("--sequence", action="store_true",
                    help="print the kernels of one round in launch order with their durations "
                         "averaged over the selected rounds (needs a fixed kernel list per round)")
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            grid = r.get("Grid_Size_X") or r.get("Grid_Size") or ""
            wg = r.get("Workgroup_Size_X") or r.get("Workgroup_Size") or ""
            # (the grid in workgroups: rocprofv3 reports work-items)
            nwg = str(int(grid) // max(1, int(wg))) if grid.isdigit() and wg.isdigit() else ""
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], nwg))
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
    if a.per_round and a.tail_ms <= 0:
        per_round(rows, starts, a.per_round)
    if a.sequence and a.tail_ms <= 0:
        sequence(rows, starts[-a.rounds - 1:])
    n = a.rounds
    wall = (sel[-1][1] - sel[0][0]) / n
    busy = collections.Counter()
    calls = collections.Counter()
    idle = 0
    end = sel[0][0]
    for s, e, k, _ in sel:
        if s > end:
            idle += s - end
        end = max(end, e)
        busy[short(k)] += e - s
        calls[short(k)] += 1
    tot = sum(busy.values())
    if a.gaps:
        gap = collections.Counter()
        prev, end = None, sel[0][0]
        for s, e, k, _ in sel:
            if prev is not None and s > end:
                gap[(short(prev)[:40], short(k)[:40])] += s - end
            if e >= end:
                end, prev = e, k
        print(f"# largest idle gaps (us/round): previous kernel -> next kernel")
        for (p0, k0), v in gap.most_common(a.gaps):
            print(f"{v / n / 1e3:9.1f}  {p0} -> {k0}")
    print(f"# rounds={n} wall/round={wall / 1e3:.1f}us busy/round={tot / n / 1e3:.1f}us "
          f"idle/round={idle / n / 1e3:.1f}us kernels/round={len(sel) / n:.1f}")
    print("# us/round  calls/round  kernel")
    for k, v in busy.most_common(a.top):
        print(f"{v / n / 1e3:9.1f} {calls[k] / n:6.1f}  {k}")


def sequence(rows, starts):
    spans = [rows[starts[i]:starts[i + 1]] for i in range(len(starts) - 1)]
    n = min(len(sp) for sp in spans)
    spans = [sp for sp in spans if len(sp) == n]
    print(f"# launch order of one round ({len(spans)} rounds of {n} kernels averaged): "
          "start offset us, duration us, workgroups, kernel")
    for j in range(n):
        d = sum(sp[j][1] - sp[j][0] for sp in spans) / len(spans) / 1e3
        t = sum(sp[j][0] - sp[0][0] for sp in spans) / len(spans) / 1e3
        print(f"{t:9.1f} {d:8.1f} {spans[0][j][3]:>6}  {short(spans[0][j][2])}")


def per_round(rows, starts, top):
    """Round-by-round split: does a round's time change because the GPU waits
    (idle) or because kernels run longer (and which)?"""
    spans = [rows[starts[i]:starts[i + 1]] for i in range(len(starts) - 1)]
    tot = collections.Counter()
    for sp in spans:
        for s, e, k, _ in sp:
            tot[short(k)] += e - s
    names = [k for k, _ in tot.most_common(top)]
    print("# round  wall_us  busy_us  idle_us  " + "  ".join(n[:28] for n in names))
    for i, sp in enumerate(spans):
        wall = sp[-1][1] - sp[0][0]
        busy = collections.Counter()
        idle, end = 0, sp[0][0]
        for s, e, k, _ in sp:
            if s > end:
                idle += s - end
            end = max(end, e)
            busy[short(k)] += e - s
        print(f"{i:7d} {wall / 1e3:8.1f} {sum(busy.values()) / 1e3:8.1f} {idle / 1e3:8.1f}  "
              + "  ".join(f"{busy[n] / 1e3:28.1f}" for n in names))


if __name__ == "__main__":
    main()
