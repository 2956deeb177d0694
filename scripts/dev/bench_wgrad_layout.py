"""GPT-2 weight-gradient GEMM layouts: dW[m, n] += o^T @ dp with the operands as
stored (both K-strided, "NT") vs K-contiguous copies (o^T and dp^T made
contiguous first, "TN"); times include the transpose copies."""
import time
import torch

Mr = 5120 + 37
shapes = [(768, 2304), (768, 768), (768, 3072), (3072, 768)]


def bench(fn, it=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / it * 1e6


for m, n in shapes:
    o = torch.randn(Mr, m, device="cuda", dtype=torch.bfloat16)
    dp = torch.randn(Mr, n, device="cuda", dtype=torch.bfloat16)
    sink = torch.zeros(m, n, device="cuda")
    base = bench(lambda: torch.addmm(sink, o.t(), dp, out_dtype=torch.float32, out=sink))
    oT = o.t().contiguous()
    dpT = dp.t().contiguous()
    tn = bench(lambda: torch.addmm(sink, oT, dpT.t(), out_dtype=torch.float32, out=sink))
    tr = bench(lambda: (o.t().contiguous(), dp.t().contiguous()))
    ta = bench(lambda: torch.addmm(sink, oT, dp, out_dtype=torch.float32, out=sink))
    tb = bench(lambda: torch.addmm(sink, o.t(), dpT.t(), out_dtype=torch.float32, out=sink))
    print(f"{m}x{n}: NT {base:.1f} us ({2*m*n*Mr/base/1e6:.0f} TF/s) | TN gemm {tn:.1f} us "
          f"({2*m*n*Mr/tn/1e6:.0f} TF/s) + 2 transposes {tr:.1f} us | A-contig only {ta:.1f} | "
          f"B-contig only {tb:.1f}", flush=True)
