"""GPT-2 weight-gradient GEMM shapes in isolation (T tokens): hipBLASLt
fp32-output accumulate (the current path) vs bf16-output + fp32 add, and
the operand-swapped form."""
import torch


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


for T in (9600,):
    for (m, n) in ((768, 2304), (768, 768), (768, 3072), (3072, 768)):
        x = torch.randn(T, m, device="cuda").to(torch.bfloat16)
        gy = torch.randn(T, n, device="cuda").to(torch.bfloat16)
        sink = torch.zeros(m, n, device="cuda")
        fl = 2.0 * T * m * n
        t0 = timeit(lambda: torch.addmm(sink, x.t(), gy, out_dtype=torch.float32, out=sink))
        t1 = timeit(lambda: sink.add_(torch.mm(x.t(), gy)))
        sinkT = torch.zeros(n, m, device="cuda")
        t2 = timeit(lambda: torch.addmm(sinkT, gy.t(), x, out_dtype=torch.float32, out=sinkT))
        import sys, os
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
        from commefficient_amd._ext import ops
        t3 = timeit(lambda: ops().gemm_tn_acc(sink, x, gy))
        print(f"T={T} {m}x{n}: addmm_fp32 {t0:.1f} us ({fl / t0 / 1e6:.0f} TF/s)  bf16+add {t1:.1f}  "
              f"swapped fp32 {t2:.1f} us  native gemm_tn {t3:.1f} us ({fl / t3 / 1e6:.0f} TF/s)",
              flush=True)
