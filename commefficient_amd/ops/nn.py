"""Autograd wrappers for fused native NN kernels used by the models.

``relu_maxpool(x, k)`` = ``max_pool2d(relu(x), k)`` (relu and max commute).
On a HIP device with a bf16 channels_last input it runs the fused gfx950
kernels of csrc/pool.hip (one read of the conv output forward, one coalesced
write of the input gradient backward); otherwise it is the plain PyTorch
composition (CPU runs, fp32 runs, odd shapes).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .._ext import ops as _ops


class _ReluMaxPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k):
        y, idx = _ops().relu_maxpool(x, k)
        ctx.save_for_backward(idx)
        ctx.k = k
        return y

    @staticmethod
    def backward(ctx, gy):
        (idx,) = ctx.saved_tensors
        return _ops().relu_maxpool_backward(gy.to(torch.bfloat16), idx, ctx.k), None


def fused_ok(x: torch.Tensor, k: int) -> bool:
    return (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and k in (2, 4)
            and x.shape[1] % 8 == 0 and x.shape[2] % k == 0 and x.shape[3] % k == 0
            and x.is_contiguous(memory_format=torch.channels_last))


def relu_maxpool(x: torch.Tensor, k: int) -> torch.Tensor:
    if fused_ok(x, k):
        return _ReluMaxPool.apply(x, k)
    return F.max_pool2d(F.relu(x), k)
