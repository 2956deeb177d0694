#!/usr/bin/env python
"""Micro-benchmark of the native codec kernels at ResNet-9 / GPT-2 sizes
(HIP-event timing, median of N repeats).  Prints one JSON line per op."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from commefficient_amd import ops  # noqa: E402
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
    sizes = [("resnet9", 6568640), ("gpt2", 124444417)]
    if len(sys.argv) > 1:
        sizes = [s for s in sizes if s[0] in sys.argv[1:]]
    for name, d in sizes:
        r, c, k = 5, 500000, 50000
        g = torch.Generator(device="cuda").manual_seed(0)
        v = torch.randn(d, device="cuda", generator=g)
        w = torch.randn(d, device="cuda", generator=g)
        res = {"size": name, "d": d}
        skb = CSVec(d, c, r, device="cuda", numBlocks=20, kernel="binned")
        res["encode_binned_us"] = timeit(lambda: skb.accumulateVec(v, 1.0, w, 1e-3))
        res["query_hash_us"] = timeit(lambda: skb.query())
        from commefficient_amd._ext import ops as _o
        res["query_rows_us"] = timeit(lambda: _o().cs_query_rows(
            skb.table, skb.hashes, skb.blk_off, skb.blk_sign, skb.numBlocks, skb.d))
        torch.testing.assert_close(_o().cs_query_rows(skb.table, skb.hashes, skb.blk_off, skb.blk_sign,
                                                      skb.numBlocks, skb.d), skb.query())
        if d < 2e7:
            res["encode_direct_us"] = timeit(lambda: skb.accumulateVec(v, 1.0, w, 1e-3, dense=False), 5)
        del skb
        torch.cuda.synchronize()
        t0 = torch.cuda.Event(enable_timing=True)
        t1 = torch.cuda.Event(enable_timing=True)
        sk = CSVec(d, c, r, device="cuda", numBlocks=20, kernel="planned")
        t0.record()
        sk._plan()
        t1.record()
        t1.synchronize()
        res["plan_build_ms"] = t0.elapsed_time(t1)
        if sk._plan() is None:  # geometry unsupported by the planned kernels
            sk = CSVec(d, c, r, device="cuda", numBlocks=20, kernel="binned")
        else:
            res["plan_mb"] = sum(t.numel() * t.element_size() for t in sk._plan()) / 2 ** 20
            res["encode_planned_us"] = timeit(lambda: sk.accumulateVec(v, 1.0, w, 1e-3))
        res["query_us"] = timeit(lambda: sk.query())
        est = sk.query()
        res["topk_us"] = timeit(lambda: ops.topk_abs(est, k))
        idx, vals = ops.topk_abs(est, k)
        V = torch.zeros(r, c, device="cuda")
        res["zero_hh_us"] = timeit(lambda: sk.zero_heavy_hitters(idx, vals, V))
        E = torch.zeros(r, c, device="cuda")
        G = torch.randn(r, c, device="cuda")
        res["momentum_ef_rc_us"] = timeit(lambda: ops.momentum_ef(V.view(-1), E.view(-1), G.view(-1), 0.9, 1.0, "virtual"))
        lm = torch.full((d,), -1, dtype=torch.int32, device="cuda")
        res["sparse_apply_us"] = timeit(lambda: ops.sparse_apply(w, idx, vals, 0.0, None, lm, 1))
        thr = torch.arange(0, 100, dtype=torch.int32)
        res["count_ge_100_us"] = timeit(lambda: ops.count_ge(lm, thr))
        res["l2norm_us"] = timeit(lambda: ops.l2norm(v))
        res["topk_dense_d_us"] = timeit(lambda: ops.topk_abs(v, k))
        print(json.dumps({k2: (round(x, 1) if isinstance(x, float) else x) for k2, x in res.items()}),
              flush=True)


if __name__ == "__main__":
    main()
