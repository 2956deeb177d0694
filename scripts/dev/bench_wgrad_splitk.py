"""GPT-2 weight-gradient GEMM shapes (dW[m, n] += o^T[m, Mr] @ dp[Mr, n], bf16 in,
fp32 out): plain fp32-output addmm vs split-K batched GEMM + fixed-order sum."""
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
    res = [f"{m}x{n}: addmm {base:.1f} us ({2 * m * n * Mr / base / 1e6:.0f} TF/s)"]
    for S in (2, 4, 8, 16):
        q = Mr // S

        def split():
            A = o[:S * q].view(S, q, m).transpose(1, 2)
            B = dp[:S * q].view(S, q, n)
            part = torch.bmm(A, B, out_dtype=torch.float32)
            if Mr > S * q:
                torch.addmm(sink, o[S * q:].t(), dp[S * q:], out_dtype=torch.float32, out=sink)
            sink.add_(part.sum(0))
        t = bench(split)
        res.append(f"S={S} {t:.1f} us ({2 * m * n * Mr / t / 1e6:.0f} TF/s)")
    # forward / dgrad shapes for reference
    W = torch.randn(m, n, device="cuda", dtype=torch.bfloat16)
    tf = bench(lambda: torch.mm(o, W))
    res.append(f"fwd mm {tf:.1f} us ({2 * m * n * Mr / tf / 1e6:.0f} TF/s)")
    print("; ".join(res), flush=True)
