#!/usr/bin/env python
"""Tied LM head backward variants on the padded logits gradient (rows of
ceil8(V) columns, as the native CE writes it): dh = g W and dW += g^T h,
HIP-event medians per variant (us)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from commefficient_amd import _ext  # noqa: E402
from bench_conv import timeit  # noqa: E402


def main():
    ops = _ext.ops()
    V, H = 50257, 768
    for T in (640, 2048):
        ld = -(-V // 8) * 8
        buf = torch.zeros(T, ld, device="cuda", dtype=torch.bfloat16)
        buf[:, :V] = (torch.randn(T, V, device="cuda") * 1e-3).to(torch.bfloat16)
        gs = buf[:, :V]
        gc = gs.contiguous()
        W = (torch.randn(V, H, device="cuda") * 0.02).to(torch.bfloat16)
        h = torch.randn(T, H, device="cuda").to(torch.bfloat16)
        sink = torch.zeros(V, H, device="cuda")
        dh32 = torch.zeros(T, H, device="cuda")
        res = {"T": T}
        res["dh_mm_strided"] = timeit(lambda: torch.mm(gs, W), n=20)
        res["dh_mm_contig"] = timeit(lambda: torch.mm(gc, W), n=20)
        res["dh_mm_transposed"] = timeit(lambda: torch.mm(W.t(), gs.t()).t(), n=20)

        def tn_dh():
            gt = gs.t().contiguous()
            dh32.zero_()
            ops.gemm_tn_acc(dh32, gt, W)
            return dh32.to(torch.bfloat16)
        res["dh_tn_transpose_copy"] = timeit(tn_dh, n=20)
        res["dW_tn_native"] = timeit(lambda: ops.gemm_tn_acc(sink, gs, h), n=20)
        res["dW_addmm"] = timeit(lambda: torch.addmm(sink, gs.t(), h, out_dtype=torch.float32, out=sink), n=20)
        res["dW_addmm_contig"] = timeit(lambda: torch.addmm(sink, gc.t(), h, out_dtype=torch.float32, out=sink), n=20)
        res["fwd_native_nedge"] = timeit(lambda: ops.mm_nt(h, W, None, buf[:, :V]), n=20)
        res["fwd_mm"] = timeit(lambda: torch.mm(h, W.t()), n=20)
        print(json.dumps({k: (round(v, 1) if isinstance(v, float) else v) for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
