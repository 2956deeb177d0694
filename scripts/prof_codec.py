#!/usr/bin/env python
"""Runs the Count-Sketch encode/query kernels (binned, planned, direct query)
at ResNet-9 size a few times, for rocprofv3 --pmc / --kernel-trace."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from commefficient_amd.ops import CSVec  # noqa: E402


def main():
    d, c, r = 6568640, 500000, 5
    g = torch.Generator(device="cuda").manual_seed(0)
    v = torch.randn(d, device="cuda", generator=g)
    w = torch.randn(d, device="cuda", generator=g)
    for kernel in ("binned", "planned"):
        sk = CSVec(d, c, r, device="cuda", numBlocks=20, kernel=kernel)
        for _ in range(3):
            sk.accumulateVec(v, 1.0, w, 1e-3)
            sk.query()
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
