#!/usr/bin/env python
"""Stream timeline of a rocprofv3 kernel trace window: busy time per HIP
stream, the union (GPU busy), and the largest idle gaps with the kernels on
either side -- where a multi-stream round (e.g. GPT-2's side-stream weight
gradients) is waiting.

    python scripts/timeline.py trace.csv --marker enc_p1 --gaps 15   (one round)
    python scripts/timeline.py trace.csv --tail-ms 35
"""
import argparse
import csv
import collections


def _short(name: str) -> str:
    name = name.replace("void ", "").replace("(anonymous namespace)::", "").replace("commeff::", "")
    return name.split("(")[0][:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--tail-ms", type=float, default=0.0, help="window: the trace's last N ms")
    ap.add_argument("--marker", default="", help="window: between the last two starts of this kernel")
    ap.add_argument("--gaps", type=int, default=15)
    ap.add_argument("--min-gap-us", type=float, default=5.0)
    args = ap.parse_args()
    rows = []
    with open(args.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Stream_Id", "0"),
                         _short(r["Kernel_Name"])))
    rows.sort()
    if args.marker:
        marks = [s for s, _, _, n in rows if args.marker in n]
        lo, hi = marks[-2], marks[-1]
        rows = [r for r in rows if lo <= r[0] < hi]
        end = hi
    else:
        end = max(e for _, e, _, _ in rows)
        lo = end - int(args.tail_ms * 1e6)
        rows = [r for r in rows if r[0] >= lo]
    t0 = rows[0][0]
    per = collections.defaultdict(float)
    for s, e, st, _ in rows:
        per[st] += (e - s) / 1e3
    # union of busy intervals
    busy, cur_s, cur_e = 0.0, None, None
    gaps = []
    prev_name = None
    for s, e, st, name in rows:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += (cur_e - cur_s) / 1e3
                gaps.append(((s - cur_e) / 1e3, (cur_e - t0) / 1e3, prev_name, name))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
        prev_name = name if e >= (cur_e or 0) else prev_name
    busy += (cur_e - cur_s) / 1e3
    wall = (end - t0) / 1e3
    print(f"# window {wall:.1f} us  GPU busy (union) {busy:.1f} us  idle {wall - busy:.1f} us  "
          f"kernels {len(rows)}")
    for st, us in sorted(per.items(), key=lambda x: -x[1]):
        print(f"# stream {st}: busy {us:.1f} us")
    print("# largest idle gaps: us, at (us into window), kernel before -> kernel after")
    for g, at, a, b in sorted((g for g in gaps if g[0] >= args.min_gap_us), key=lambda x: -x[0])[:args.gaps]:
        print(f"{g:9.1f} {at:10.1f}  {a}  ->  {b}")


if __name__ == "__main__":
    main()
