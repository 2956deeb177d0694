"""Ghost BN forward / backward on ResNet-101 ImageNet shapes (8 clients x 32
images, channels_last bf16) -- run under rocprofv3 --kernel-trace --stats for
the per-kernel split (partial sums / finalize / apply)."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from commefficient_amd import _ext  # noqa: E402

ops = _ext.ops()
G, n = 8, 32
for C, H in ((64, 56), (256, 56), (128, 28), (1024, 14), (512, 7)):
    x = torch.randn(G * n, C, H, H, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    w = torch.rand(C, device="cuda") + 0.5
    b = torch.randn(C, device="cuda")
    rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
    dy = torch.randn_like(x)
    for _ in range(20):
        y, stat, bits = ops.ghost_bn_fwd(x, w, b, G, 1e-5, 0.1, rm, rv, True)
        ops.ghost_bn_bwd(dy, x, stat, w, G, bits)
    torch.cuda.synchronize()
print("done")
