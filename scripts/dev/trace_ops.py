#!/usr/bin/env python
"""Aten ops of a torch.profiler chrome trace whose name matches PATTERN, with
their input shapes / dtypes and the GPU time of the kernels they launched
(per round: divided by ROUNDS).  Usage: trace_ops.py TRACE PATTERN [ROUNDS]"""
import collections
import json
import sys


def main():
    ev = json.load(open(sys.argv[1]))["traceEvents"]
    pat, rounds = sys.argv[2], float(sys.argv[3]) if len(sys.argv) > 3 else 3.0
    ops = [e for e in ev if e.get("ph") == "X" and e.get("cat") == "cpu_op" and pat in e.get("name", "")]
    launches = {e["args"]["correlation"]: e for e in ev if e.get("ph") == "X" and e.get("cat") == "cuda_runtime"
                and "correlation" in e.get("args", {})}
    kern = {e["args"]["correlation"]: e for e in ev if e.get("ph") == "X" and e.get("cat") == "kernel"
            and "correlation" in e.get("args", {})}
    # kernel time of each op: launches inside the op's host interval
    agg = collections.defaultdict(lambda: [0, 0.0])
    for o in ops:
        t0, t1 = o["ts"], o["ts"] + o["dur"]
        g = sum(kern[c]["dur"] for c, l in launches.items() if t0 <= l["ts"] <= t1 and c in kern)
        key = (o["name"], str(o["args"].get("Input Dims")), str(o["args"].get("Input type")))
        agg[key][0] += 1
        agg[key][1] += g
    for (n, d, t), (c, g) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:25]:
        print(f"{c / rounds:5.1f}/round {g / rounds:8.1f} us  {n} {d} {t}")


if __name__ == "__main__":
    main()
