#!/usr/bin/env python
"""Weight-gradient TN GEMM (csrc/gemm_tn.hip) vs hipBLASLt on the GPT-2
shapes: C[M][N] += A[T][M]^T B[T][N], bf16 in, fp32 accumulate."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from commefficient_amd import _ext  # noqa: E402


def timeit(fn, n=30):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / n


def main():
    ops = _ext.ops()
    T = int(os.environ.get("TN_T", "9400"))
    for M, N in [(768, 2304), (768, 768), (768, 3072), (3072, 768)]:
        a = torch.randn(T, M, device="cuda").bfloat16()
        b = torch.randn(T, N, device="cuda").bfloat16()
        sink = torch.zeros(M, N, device="cuda")
        ref = a.float().t() @ b.float()
        ops.gemm_tn_acc(sink, a, b)
        err = ((sink - ref).norm() / ref.norm()).item()
        tn = timeit(lambda: ops.gemm_tn_acc(sink, a, b))
        tl = timeit(lambda: torch.mm(a.t(), b, out_dtype=torch.float32))
        fl = 2.0 * T * M * N
        print(json.dumps({"T": T, "M": M, "N": N, "native_us": round(tn, 1),
                          "native_tflops": round(fl / tn / 1e6, 1), "blas_us": round(tl, 1),
                          "blas_tflops": round(fl / tl / 1e6, 1), "rel_err": err}), flush=True)


if __name__ == "__main__":
    main()
