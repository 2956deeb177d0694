"""ImageNet stem max-pool (3x3 / 2, 112x112x64, 256 images) forward + backward."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from commefficient_amd import _ext  # noqa: E402

ops = _ext.ops()
x = torch.randn(256, 64, 112, 112, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
y, codes = ops.maxpool_fwd(x, 3, 2, 1)
gy = torch.randn_like(y)
def t(fn, n=10):
    fn(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / n
print("fwd us", round(t(lambda: ops.maxpool_fwd(x, 3, 2, 1)), 1),
      "bwd us", round(t(lambda: ops.maxpool_bwd(gy, codes, 112, 112, 3, 2, 1)), 1))
