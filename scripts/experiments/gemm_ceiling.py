"""hipBLASLt bf16 GEMM throughput on the GEMM shapes of ResNet-9's convs
(batch 500): the library ceiling our implicit-GEMM conv kernels compare to."""
import torch

shapes = {  # name: (M, N, K) for fwd (pixels x out x 9*in) and wgrad (out x 9*in x pixels)
    "layer1 fwd": (512000, 128, 576), "res1 fwd": (128000, 128, 1152),
    "layer2 fwd": (128000, 256, 1152), "layer3 fwd": (32000, 512, 2304),
    "res3 fwd": (8000, 512, 4608),
    "layer1 wgrad": (128, 576, 512000), "res1 wgrad": (128, 1152, 128000),
    "layer2 wgrad": (256, 1152, 128000), "layer3 wgrad": (512, 2304, 32000),
    "res3 wgrad": (512, 4608, 8000),
}
for name, (M, N, K) in shapes.items():
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    if "wgrad" in name:  # both operands K-major along pixels: a^T-like layout
        a = torch.randn(K, M, device="cuda", dtype=torch.bfloat16).t()
        b = torch.randn(K, N, device="cuda", dtype=torch.bfloat16)
    else:
        b = torch.randn(N, K, device="cuda", dtype=torch.bfloat16).t()
    for _ in range(3):
        c = a @ b
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        c = a @ b
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 20 * 1e3
    print(f"{name:14s} M={M:7d} N={N:5d} K={K:7d} {us:8.1f} us {2*M*N*K/us/1e6:7.1f} TF/s", flush=True)
