#!/usr/bin/env python
"""Weight-gradient GEMMs of the ResNet-101 ImageNet round (8 clients x 32
images, per-client gradients): the native split-K TN GEMM (csrc/gemm_tn.hip,
ops/nn.py _wgrad_gemm) vs hipBLASLt batched GEMM + split reduction, per
shape.  Prints one JSON line per shape and the round totals weighted by the
layer counts.

    python scripts/bench_wgrad_tn.py [--groups 8 --per 32]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (K = out channels, C = GEMM columns (in channels, or the column-image width),
#  output pixels per image, layers of that shape per round)
SHAPES = [(64, 64, 3136, 1), (64, 256, 3136, 2), (256, 64, 3136, 4), (128, 256, 3136, 1),
          (128, 512, 784, 3), (512, 128, 784, 4), (512, 256, 784, 1), (256, 512, 784, 1),
          (256, 1024, 196, 22), (1024, 256, 196, 23), (1024, 512, 196, 1), (512, 1024, 196, 1),
          (512, 2048, 49, 2), (2048, 512, 49, 3), (2048, 1024, 49, 1),
          # column-image (strided 3x3, 3x3 with 64 channels): C = 9 * in channels
          (64, 576, 3136, 3), (128, 1152, 784, 1), (256, 2304, 196, 1), (512, 4608, 49, 1)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", type=int, default=8)
    ap.add_argument("--per", type=int, default=32)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    from commefficient_amd import _ext
    from commefficient_amd.ops import nn as onn
    _ext.load()
    G = a.groups
    tot = {"native": 0.0, "blas": 0.0}
    for K, C, hw, count in SHAPES:
        P = G * a.per * hw
        g2d = torch.randn(P, K, device="cuda").to(torch.bfloat16)
        x2d = torch.randn(P, C, device="cuda").to(torch.bfloat16)
        into = torch.zeros(G, K, C, device="cuda")
        row = {"K": K, "C": C, "P": P, "layers": count}
        for mode in ("native", "blas"):
            onn._GEMM_NATIVE[0] = mode == "native"
            fn = lambda: onn._wgrad_gemm(g2d, x2d, into, G)  # noqa: E731
            for _ in range(2):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(a.iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / a.iters
            row[mode + "_us"] = round(us, 1)
            row[mode + "_TFs"] = round(2.0 * P * K * C / us / 1e6, 1)
            tot[mode] += count * us
        onn._GEMM_NATIVE[0] = True
        print(json.dumps(row), flush=True)
        del g2d, x2d, into
    print(json.dumps({"round_native_ms": round(tot["native"] / 1e3, 2),
                      "round_blas_ms": round(tot["blas"] / 1e3, 2)}), flush=True)


if __name__ == "__main__":
    main()
