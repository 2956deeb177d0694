#!/usr/bin/env python
"""Ghost batch norm (csrc/bn.hip) micro-benchmark on the ResNet-101 ImageNet
round's BN shapes (8 clients x 32 images, NHWC bf16): forward (+ReLU bits)
and backward (ReLU-gated) op times, effective HBM bandwidth, and the round
total weighted by each shape's layer count.

    python scripts/bench_bn.py [--groups 8 --per 32 --iters 20]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (channels, spatial side, layers of that shape in ResNet-101; residual tails
# = layers that also take the block's addend)
SHAPES = [(64, 112, 1, 0), (64, 56, 6, 0), (256, 56, 4, 3), (128, 56, 1, 0), (128, 28, 7, 0),
          (512, 28, 5, 4), (256, 28, 1, 0), (256, 14, 45, 0), (1024, 14, 24, 23),
          (512, 14, 1, 0), (512, 7, 5, 0), (2048, 7, 4, 3)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", type=int, default=8)
    ap.add_argument("--per", type=int, default=32)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from commefficient_amd import _ext
    _ext.load()
    ops = torch.ops.commeff
    dev = torch.device("cuda")
    G, N = a.groups, a.groups * a.per
    tot_f = tot_b = 0.0
    for C, S, count, tails in SHAPES:
        x = torch.randn(N, C, S, S, device=dev).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        dy = torch.randn_like(x)
        add = torch.randn_like(x)
        w = torch.rand(C, device=dev) + 0.5
        b = torch.randn(C, device=dev)
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        nbt = torch.zeros((), dtype=torch.long, device=dev)
        gw, gb = torch.zeros(C, device=dev), torch.zeros(C, device=dev)

        def fwd(addend=None):
            return ops.ghost_bn_fwd(x, w, b, G, 1e-5, 0.1, rm, rv, True, nbt, addend)

        y, stat, bits = fwd()

        def bwd(dadd=None):
            return ops.ghost_bn_bwd(dy, x, stat, w, G, bits, gw, gb, None, None, dadd)

        dadd = torch.empty_like(x)

        def timed(fn):
            for _ in range(3):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(a.iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) * 1e3 / a.iters

        tf = timed(fwd)
        tb = timed(bwd)
        tfa = timed(lambda: fwd(add)) if tails else tf
        tba = timed(lambda: bwd(dadd)) if tails else tb
        nb = x.numel() * 2
        # fwd: partial reads x, apply reads x + writes y (+ bits); bwd: partial
        # reads x + dy, apply reads x + dy, writes dx (+ bits twice)
        gbf = (3 * nb + x.numel() / 8) / tf / 1e3
        gbb = (5 * nb + x.numel() / 4) / tb / 1e3
        tot_f += (count - tails) * tf + tails * tfa
        tot_b += (count - tails) * tb + tails * tba
        print(json.dumps({"C": C, "S": S, "layers": count, "MB": round(nb / 2**20, 1),
                          "fwd_us": round(tf, 1), "fwd_GBs": round(gbf), "bwd_us": round(tb, 1),
                          "bwd_GBs": round(gbb), "fwd_add_us": round(tfa, 1),
                          "bwd_add_us": round(tba, 1)}), flush=True)
    print(json.dumps({"round_bn_fwd_ms": round(tot_f / 1e3, 2), "round_bn_bwd_ms": round(tot_b / 1e3, 2),
                      "round_bn_ms": round((tot_f + tot_b) / 1e3, 2)}), flush=True)


if __name__ == "__main__":
    main()
