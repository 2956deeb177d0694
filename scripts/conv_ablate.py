#!/usr/bin/env python
"""Where does the halo conv forward spend its time?  Times the native forward
(and dgrad, the same kernel) per ResNet-9 layer at the bench batch under
COMMEFF_CONV_ABLATE (set by the caller; csrc/kernels.h ConvFwdArgs.ablate):
bit 0 drops the per-K-step weight-tile loads, bit 1 the per-channel-block
window reloads, bit 2 the per-K-step wait + barrier.  Timing only -- the
outputs are wrong under any ablation.  One JSON line per layer."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from commefficient_amd import ops  # noqa: E402
from bench_conv import LAYERS, timeit  # noqa: E402


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 500
    ab = int(os.environ.get("COMMEFF_CONV_ABLATE", "0"))
    for name, C, H, K in LAYERS:
        x = torch.randn(N, C, H, H, device="cuda").to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        dy = torch.randn(N, K, H, H, device="cuda").to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        w = torch.randn(K, C, 3, 3, device="cuda") * 0.05
        wf, wt = ops.conv_weight_prep(w)
        flops = 2.0 * N * H * H * K * C * 9
        f = timeit(lambda: ops.conv3x3_fwd(x, wf, True), n=40)
        d = timeit(lambda: ops.conv3x3_fwd(dy, wt, False), n=40)
        wg = timeit(lambda: ops.conv3x3_wgrad(dy, x), n=40)
        print(json.dumps({"ablate": ab, "layer": name, "fwd_us": round(f, 1),
                          "fwd_tflops": round(flops / f / 1e6, 1),
                          "dgrad_us": round(d, 1), "wgrad_us": round(wg, 1)}), flush=True)


if __name__ == "__main__":
    main()
