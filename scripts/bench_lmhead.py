#!/usr/bin/env python
"""Tied LM head (GPT-2, vocabulary 50,257) forward + backward: native
(ops/transformer.py _LMHead: NT GEMM, split-K TN GEMMs for dh and dW into an
fp32 sink) vs hipBLASLt (nn.Linear), per phase, isolated.

    python scripts/bench_lmhead.py [--tokens 560]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=560)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from commefficient_amd import _ext
    from commefficient_amd.ops import transformer as tx
    _ext.load()
    V, H, T = 50257, 768, a.tokens
    head = torch.nn.Linear(H, V, bias=False).to(torch.bfloat16).cuda()
    m = type("M", (), {})()
    m.lm_head = head
    h = torch.randn(T, H, device="cuda").to(torch.bfloat16).requires_grad_(True)
    gy = torch.randn(T, V, device="cuda").to(torch.bfloat16)
    sink = torch.zeros(V, H, device="cuda")

    def run(native):
        def fwd():
            return tx.lm_head(m, h) if native else head(h)

        def both():
            with tx.grad_sinks({id(head.weight): sink} if native else None):
                y = fwd()
                y.backward(gy)
            tx.join_wgrad_stream()
            h.grad = None
            head.weight.grad = None

        out = {}
        for name, fn in (("fwd", lambda: fwd()), ("fwd_bwd", both)):
            for _ in range(3):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(a.iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            out[name + "_us"] = round(e0.elapsed_time(e1) * 1e3 / a.iters, 1)
        return out

    print(json.dumps({"tokens": T, "native": run(True), "hipblaslt": run(False)}), flush=True)


if __name__ == "__main__":
    main()
