#!/usr/bin/env python
"""Median duration per (kernel, grid) of a rocprofv3 rocpd database, for kernels
whose name contains PATTERN.  Usage: python scripts/dev/rocpd_grid.py DB PATTERN"""
import collections
import sqlite3
import sys


def main():
    c = sqlite3.connect(sys.argv[1])
    pat = sys.argv[2] if len(sys.argv) > 2 else ""
    rows = c.execute("select name, start, end, grid_x, grid_y, grid_z, workgroup_x from kernels order by start")
    d = collections.defaultdict(list)
    for n, s, e, gx, gy, gz, wx in rows:
        if pat in n:
            d[(n.split("(")[0][-70:], gx // max(1, wx), gy, gz)].append((e - s) / 1e3)
    for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
        v.sort()
        print(f"{len(v):5d} calls  median {v[len(v) // 2]:8.1f} us  grid {k[1]}x{k[2]}x{k[3]}  {k[0]}")


if __name__ == "__main__":
    main()
