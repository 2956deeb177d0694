"""The ImageNet stem's 7x7 / stride-2 column image (3-channel input, 152
columns) in isolation."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from commefficient_amd import _ext  # noqa: E402

ops = _ext.ops()
x = torch.randn(256, 3, 224, 224, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
for _ in range(3):
    col = ops.im2col(x, 7, 7, 2, 3, 152)
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(10):
    col = ops.im2col(x, 7, 7, 2, 3, 152)
e.record()
torch.cuda.synchronize()
us = s.elapsed_time(e) * 100
print(f"stem im2col {tuple(col.shape)}: {us:.1f} us, {col.numel() * 2 / us / 1e6:.2f} TB/s written")
