#!/usr/bin/env python
"""Per-layer conv3x3 timing at the ResNet-9 bench batch (500 images): native
MFMA kernels (csrc/conv.hip) vs MIOpen (F.conv2d / torch.nn.grad, with
cudnn.benchmark find).  HIP-event medians; one JSON line per layer."""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from commefficient_amd import ops  # noqa: E402

LAYERS = [  # name, C, H(=W), K
    ("layer1", 64, 32, 128), ("res1", 128, 16, 128), ("layer2", 128, 16, 256),
    ("layer3", 256, 8, 512), ("res3", 512, 4, 512),
]


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
    torch.backends.cudnn.benchmark = True
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 500
    tot = {"native": 0.0, "miopen": 0.0}
    for name, C, H, K in LAYERS:
        x = torch.randn(N, C, H, H, device="cuda").to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        dy = torch.randn(N, K, H, H, device="cuda").to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        w = torch.randn(K, C, 3, 3, device="cuda") * 0.05
        wb = w.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        wf, wt = ops.conv_weight_prep(w)
        flops = 2.0 * N * H * H * K * C * 9
        r = {"layer": name, "N": N, "C": C, "HW": H, "K": K}
        r["fwd_native_us"] = timeit(lambda: ops.conv3x3_fwd(x, wf, True))
        r["dgrad_native_us"] = timeit(lambda: ops.conv3x3_fwd(dy, wt, False))
        r["wgrad_native_us"] = timeit(lambda: ops.conv3x3_wgrad(dy, x))
        r["fwd_miopen_us"] = timeit(lambda: F.conv2d(x, wb, padding=1))
        r["dgrad_miopen_us"] = timeit(
            lambda: torch.ops.aten.convolution_backward(dy, x, wb, None, [1, 1], [1, 1], [1, 1],
                                                        False, [0, 0], 1, [True, False, False]))
        r["wgrad_miopen_us"] = timeit(
            lambda: torch.ops.aten.convolution_backward(dy, x, wb, None, [1, 1], [1, 1], [1, 1],
                                                        False, [0, 0], 1, [False, True, False]))
        # calibration: a plain hipBLASLt GEMM of the same M x N x K (no im2col)
        ga = torch.randn(N * H * H, 9 * C, device="cuda").to(torch.bfloat16)
        gb = torch.randn(9 * C, K, device="cuda").to(torch.bfloat16)
        r["gemm_us"] = timeit(lambda: torch.mm(ga, gb))
        r["gemm_tflops"] = round(flops / (r["gemm_us"] * 1e-6) / 1e12, 1)
        gt = torch.randn(K, N * H * H, device="cuda").to(torch.bfloat16)
        r["gemm_wgrad_us"] = timeit(lambda: torch.mm(gt, ga))
        r["gemm_wgrad_tflops"] = round(flops / (r["gemm_wgrad_us"] * 1e-6) / 1e12, 1)
        del ga, gb, gt
        for kind in ("fwd", "dgrad", "wgrad"):
            for be in ("native", "miopen"):
                r[f"{kind}_{be}_tflops"] = round(flops / (r[f"{kind}_{be}_us"] * 1e-6) / 1e12, 1)
        mult = 2 if name.startswith("res") else 1
        for be in ("native", "miopen"):
            tot[be] += mult * sum(r[f"{k}_{be}_us"] for k in ("fwd", "dgrad", "wgrad"))
        print(json.dumps({k: (round(v, 1) if isinstance(v, float) else v) for k, v in r.items()}),
              flush=True)
    print(json.dumps({"total_fwd_bwd_us": {k: round(v, 1) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
