#!/usr/bin/env python
"""Region-sketch codec micro-benchmark (HIP-event medians): encode (with and
without the weight-decay operand), median query, and zeroing at the ResNet-9
and GPT-2 geometries of the FetchSGD configs (5 x 500,000 tables)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from commefficient_amd.ops import CSVec  # noqa: E402


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(n):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    geoms = [("resnet9", 6568640), ("gpt2", 124444417)]
    if len(sys.argv) > 1:
        geoms = [g for g in geoms if g[0] in sys.argv[1:]]
    for name, d in geoms:
        g = torch.randn(d, device="cuda")
        w = torch.randn(d, device="cuda")
        sk = CSVec(d, 500000, 5, device="cuda", kernel="region")
        r = {"geom": name, "d": d, "m": sk.region.m, "nch": sk.region.nch}
        r["encode_w_us"] = timeit(lambda: sk.accumulateVec(g, 0.5, w, 1e-4, overwrite=True))
        r["encode_us"] = timeit(lambda: sk.accumulateVec(g, 0.5, None, 0.0, overwrite=True))
        r["query_us"] = timeit(lambda: sk.query())
        idx, vals = sk.unsketch_sparse(50000)
        r["zero_us"] = timeit(lambda: sk.zero_heavy_hitters(idx, vals))
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
