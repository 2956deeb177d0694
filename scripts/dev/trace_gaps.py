#!/usr/bin/env python
"""Per-round GPU timeline of a rocprofv3 rocpd database: round boundaries at
each dispatch of a marker kernel (default: the region sketch encode, once per
FetchSGD round); per round the GPU span, busy time, kernel count, and the
idle gap before the round's first kernel (after the previous round's last).
Usage: python scripts/dev/trace_gaps.py RUN_results.db [MARKER_SUBSTRING]"""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else "cs_region_encode"
    c = sqlite3.connect(db)
    ks = c.execute("select start, end, name from kernels order by start").fetchall()
    marks = [i for i, k in enumerate(ks) if marker in k[2]]
    if not marks:
        print("marker not found")
        return
    # a round: from the kernel after the previous marker to this marker (inclusive)
    prev_end_idx = -1
    print(f"{'round':>5} {'gap_before_ms':>13} {'span_ms':>8} {'busy_ms':>8} {'kernels':>7}  largest internal gap (ms, after kernel)")
    for r, mi in enumerate(marks):
        sel = ks[prev_end_idx + 1:mi + 1]
        gap = (sel[0][0] - ks[prev_end_idx][1]) / 1e6 if prev_end_idx >= 0 else 0.0
        span = (sel[-1][1] - sel[0][0]) / 1e6
        busy = sum(k[1] - k[0] for k in sel) / 1e6
        big, after = 0.0, ""
        for a, b in zip(sel, sel[1:]):
            g = (b[0] - a[1]) / 1e6
            if g > big:
                big, after = g, a[2][:60]
        print(f"{r:5d} {gap:13.3f} {span:8.3f} {busy:8.3f} {len(sel):7d}  {big:.3f} after {after}")
        prev_end_idx = mi
    tail = ks[prev_end_idx + 1:]
    if tail:
        print(f"after the last round: {len(tail)} kernels, gap {(tail[0][0] - ks[prev_end_idx][1]) / 1e6:.3f} ms")


if __name__ == "__main__":
    main()
