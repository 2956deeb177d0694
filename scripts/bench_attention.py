#!/usr/bin/env python
"""Fused causal attention (csrc/attention.hip) at the GPT-2 bench shapes:
64 sequences (32 examples x 2 candidates) of SyntheticPersona lengths
(80..190 tokens), 12 heads of 64, attention dropout 0.1 -- forward and
backward µs per call and the achieved TF/s (causal FLOPs, fwd 4·L²·d/2 per
head, bwd 2.5x).  ``--lens`` overrides the length list."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from commefficient_amd._ext import ops  # noqa: E402


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
    ap = argparse.ArgumentParser()
    ap.add_argument("--nseq", type=int, default=64)
    ap.add_argument("--nh", type=int, default=12)
    ap.add_argument("--p", type=float, default=0.1)
    ap.add_argument("--lens", type=str, default="")
    ap.add_argument("--max_len", type=int, default=0, help="0: the longest sequence")
    args = ap.parse_args()
    g = torch.Generator().manual_seed(0)
    if args.lens:
        lens = [int(x) for x in args.lens.split(",")]
    else:
        lens = torch.randint(80, 191, (args.nseq,), generator=g).tolist()
    nh = args.nh
    lens_t = torch.tensor(lens, dtype=torch.int32)
    start = torch.cat([torch.zeros(1, dtype=torch.int32), lens_t.cumsum(0)[:-1].int()])
    M = int(lens_t.sum())
    qkv = (torch.randn(M, 3 * nh * 64, generator=g) * 0.5).to(torch.bfloat16).cuda()
    start, lens_t = start.cuda(), lens_t.cuda()
    L = args.max_len or max(lens)
    o, lse = ops().attn_fwd(qkv, start, lens_t, nh, args.p, 1234, L)
    gout = (torch.randn(o.shape, generator=g) * 0.5).to(torch.bfloat16).cuda()
    fwd = timeit(lambda: ops().attn_fwd(qkv, start, lens_t, nh, args.p, 1234, L))
    bwd = timeit(lambda: ops().attn_bwd(qkv, o, gout, lse, start, lens_t, nh, args.p, 1234, L))
    flops = sum(4 * Ln * Ln * 64 / 2 for Ln in lens) * nh
    print(json.dumps({"nseq": len(lens), "tokens": M, "nh": nh, "p": args.p, "max_len": L,
                      "fwd_us": round(fwd, 1), "bwd_us": round(bwd, 1),
                      "fwd_tflops": round(flops / fwd / 1e6, 1),
                      "bwd_tflops": round(2.5 * flops / bwd / 1e6, 1)}))


if __name__ == "__main__":
    main()
