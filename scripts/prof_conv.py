#!/usr/bin/env python
"""Runs each native conv kernel of the ResNet-9 layers a few times (batch 500)
for rocprofv3 --pmc / --kernel-trace collection."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from commefficient_amd import ops  # noqa: E402

LAYERS = [("layer1", 64, 32, 128), ("res1", 128, 16, 128), ("layer2", 128, 16, 256),
          ("layer3", 256, 8, 512), ("res3", 512, 4, 512)]


def main():
    N = 500
    reps = int(os.environ.get("REPS", "3"))
    only = sys.argv[1:]
    for name, C, H, K in LAYERS:
        if only and name not in only:
            continue
        x = torch.randn(N, C, H, H, device="cuda").to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        dy = torch.randn(N, K, H, H, device="cuda").to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        w = torch.randn(K, C, 3, 3, device="cuda") * 0.05
        wf, wt = ops.conv_weight_prep(w)
        for _ in range(reps):
            ops.conv3x3_fwd(x, wf, True)
            ops.conv3x3_fwd(dy, wt, False)
            ops.conv3x3_wgrad(dy, x)
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
