"""GPT-2-size planned query in coordinate windows: does the r*W vals scratch
written by Q1 stay in the MI355X MALL (256 MB Infinity Cache) for Q2?
Times the full query vs windowed queries (results must be identical)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from commefficient_amd._ext import ops  # noqa: E402
from commefficient_amd.ops import CSVec  # noqa: E402


def timeit(fn, n=10):
    for _ in range(2):
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


d, r, c = 124444417, 5, 500000
g = torch.Generator(device="cuda").manual_seed(0)
v = torch.randn(d, device="cuda", generator=g)
sk = CSVec(d, c, r, device="cuda", numBlocks=20, kernel="planned")
plan = sk._plan()
sk.accumulateVec(v, 1.0, overwrite=True)
geo = [int(x) for x in ops().plan_geometry(d, r, c)]
chunk, nch = geo[2], geo[3]
print("chunk", chunk, "num_chunks", nch, "tiles", geo[1])
full = ops().cs_query_planned(sk.table, d, plan)
print("encode_us", timeit(lambda: sk.accumulateVec(v, 1.0, overwrite=True)))
print("query_full_us", timeit(lambda: ops().cs_query_planned(sk.table, d, plan)))
est = torch.empty(d, device="cuda")
for wcoords in (2 << 20, 4 << 20, 8 << 20, 16 << 20, 32 << 20):
    wch = max(1, wcoords // chunk)

    def windowed():
        for c0 in range(0, nch, wch):
            c1 = min(nch, c0 + wch)
            part = ops().cs_query_planned(sk.table, d, plan, c0, c1)
            lo, hi = c0 * chunk, min(d, c1 * chunk)
            est[lo:hi].copy_(part[lo:hi])
        return est

    out = windowed()
    same = bool(torch.equal(out, full))
    print("window_coords", wcoords, "vals_MB", wcoords * r * 4 >> 20, "query_us",
          timeit(windowed), "equal", same)
