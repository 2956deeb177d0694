#!/usr/bin/env python
"""Top kernels of a rocprofv3 rocpd database (``--kernel-trace`` without
``--output-format csv``): per-kernel count and total / per-round time.
Usage: python scripts/dev/rocpd_top.py RUN_results.db [ROUNDS] [N]"""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    rounds = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    c = sqlite3.connect(db)
    tot = c.execute("select sum(end-start)/1e6, count(*) from kernels").fetchone()
    print(f"total {tot[0]:.2f} ms in {tot[1]} dispatches; {tot[0] / rounds:.2f} ms per round ({rounds:g} rounds)")
    print(f"{'ms/round':>9} {'calls/rd':>8} {'us/call':>8}  kernel")
    rows = c.execute("select name, count(*), sum(end-start)/1e6 from kernels group by name "
                     "order by 3 desc limit ?", (top,)).fetchall()
    for name, n, ms in rows:
        print(f"{ms / rounds:9.3f} {n / rounds:8.1f} {ms * 1e3 / n:8.1f}  {name[:120]}")


if __name__ == "__main__":
    main()
