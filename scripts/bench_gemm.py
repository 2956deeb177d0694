#!/usr/bin/env python
"""GEMM micro-benchmark at the GPT-2 and ResNet-101 shapes: the native MFMA
kernels (csrc/gemm.hip) vs hipBLASLt (torch.mm), HIP-event medians, one JSON line per
shape with TF/s and the max relative error against fp32."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from commefficient_amd import _ext  # noqa: E402
from bench_conv import timeit  # noqa: E402

SHAPES = [  # M, N, K, layout
    (9400, 2304, 768, "nn"), (9400, 768, 768, "nn"), (9400, 3072, 768, "nn"), (9400, 768, 3072, "nn"),
    (9400, 768, 2304, "nt"), (9400, 768, 768, "nt"), (9400, 768, 3072, "nt"), (9400, 3072, 768, "nt"),
    (25088, 256, 1024, "nt"), (25088, 1024, 256, "nt"), (6272, 512, 2048, "nt"), (6272, 2048, 512, "nt"),
]


def main():
    ops = _ext.ops()
    for M, N, K, lay in SHAPES:
        a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        if lay == "nn":
            b = (torch.randn(K, N, device="cuda") * K ** -0.5).to(torch.bfloat16)
            nat = lambda: ops.mm_nn(a, b)  # noqa: E731
            lib = lambda: torch.mm(a, b)  # noqa: E731
            ref = a.float() @ b.float()
        else:
            b = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
            nat = lambda: ops.mm_nt(a, b)  # noqa: E731
            lib = lambda: torch.mm(a, b.t())  # noqa: E731
            ref = a.float() @ b.float().t()
        err = ((nat().float() - ref).abs().max() / ref.abs().max()).item()
        tn, tl = timeit(nat, n=30), timeit(lib, n=30)
        fl = 2.0 * M * N * K
        print(json.dumps({"M": M, "N": N, "K": K, "layout": lay, "native_us": round(tn, 1),
                          "native_tflops": round(fl / tn / 1e6, 1), "blas_us": round(tl, 1),
                          "blas_tflops": round(fl / tl / 1e6, 1), "rel_err": round(err, 5)}), flush=True)


if __name__ == "__main__":
    main()
