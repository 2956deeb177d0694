#!/usr/bin/env python
"""FedAvg per-client classifier step: fused fa_linear_ce vs the batched GEMM path
(bmm + loss kernel + baddbmm x 2 / 3), isolated, HIP-event medians (us)."""
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
    for G, n, C, F, bias in ((100, 5, 100, 512, True), (100, 5, 10, 512, False)):
        per = C * F + C
        ld = per
        W = torch.randn(G, ld, device="cuda") * 0.05
        dst = W.clone()
        feat = torch.randn(G, n, F, device="cuda").relu()
        y = torch.randint(0, C, (G * n,), device="cuda")
        S = -(-C // 32) if bias else 1
        dfeat = torch.empty((S * G, n, F), device="cuda")
        boff = C * F if bias else -1
        beta, alpha = 0.99, -0.05

        def fused():
            return ops.fa_linear_ce(feat, n * F, F, G, n, W, ld, 0, boff, C, F, 1.0, y, dfeat, n * F, F,
                                    dst, ld, beta, alpha, None, 0, None, 0, G * n * F if S > 1 else 0,
                                    32 if S > 1 else 0)
        ones = torch.ones(G, n, 1, device="cuda")

        def stock():
            Wfc = W[:, :C * F].view(G, C, F)
            logits = torch.bmm(feat, Wfc.transpose(1, 2))
            if bias:
                logits.baddbmm_(ones, W[:, C * F:].view(G, 1, C))
            loss, correct, gl = ops.ce_fwd(logits.view(G * n, C), y)
            gl = gl.view(G, n, C)
            torch.baddbmm(dfeat[:G], gl, Wfc, beta=0.0, alpha=1.0 / n, out=dfeat[:G])
            gW = dst[:, :C * F].view(G, C, F)
            torch.baddbmm(gW, gl.transpose(1, 2), feat, beta=beta, alpha=alpha / n, out=gW)
            if bias:
                gb = dst[:, C * F:].view(G, 1, C)
                torch.baddbmm(gb, ones.transpose(1, 2), gl, beta=beta, alpha=alpha / n, out=gb)
        print(json.dumps({"G": G, "n": n, "C": C, "F": F, "fused_us": round(timeit(fused, n=30), 1),
                          "stock_us": round(timeit(stock, n=30), 1)}), flush=True)


if __name__ == "__main__":
    main()
