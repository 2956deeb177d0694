"""Fixup scalar affine maps of the merged-batch (autograd) path.

The Fixup models (models/fixup.py; reference models/fixup_resnet9.py:33-91,
fixup_resnet18.py:24-63 and the external ``fixup.imagenet`` bottleneck used by
fixup_resnet.py:8-10) wrap every convolution in learnable fp32 scalars:
``x + b`` before it, ``relu(conv * s + b (+ residual))`` after it.  As plain
PyTorch ops on bf16 activations each of those is its own pass, an fp32 [1]
parameter promotes the bf16 activation to fp32 (so the next convolution
leaves the native bf16 kernels for an autocast cast + MIOpen), and each
scalar's gradient is a separate fp32 reduction.

``scalar_affine(x, s, b, add, relu)`` is ONE bf16 pass forward
(csrc/fedavg.hip fa_affine_kernel, the FedAvg engine's per-client kernel with
one scalar pair) and ONE pass backward (fa_affine_bwd_kernel: the input
gradient, the residual's gradient and both scalars' sums, then a one-block
fixed-order fold -- deterministic).  CPU tensors, fp32 runs, torch.func
transforms (``stock_ops``) and per-group gradients take the PyTorch
composition.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F

from .._ext import ops as _ops
from . import grouped as _grouped
from . import nn as _nn


_FORK = __import__("os").environ.get("COMMEFF_FX_FORK", "1") == "1"


def _fmt(t: torch.Tensor):
    if t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last) and not t.is_contiguous():
        return torch.channels_last
    return torch.contiguous_format


def _dense(t: torch.Tensor) -> bool:
    return t.is_contiguous() or (t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last))


def _like(t: torch.Tensor, ref: torch.Tensor) -> torch.Tensor:
    """t laid out with ref's strides (autograd may hand back another layout)."""
    if t.stride() == ref.stride() and t.dtype == ref.dtype:
        return t
    return t.to(ref.dtype).contiguous(memory_format=_fmt(ref))


class _FxAffine(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, s, b, add, relu: bool, post):
        y = _ops().fx_affine(x, s, b, add, relu, post)
        ctx.has = (s is not None, b is not None, add is not None, post is not None)
        ctx.relu = relu
        if post is not None:  # relu(x + b) + post: the mask recomputed from x
            ctx.save_for_backward(x, None, s, b)
        else:
            ctx.save_for_backward(x if s is not None else None, y if relu else None, s, None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, s, bm = ctx.saved_tensors
        has_s, has_b, has_add, has_post = ctx.has
        ref = y if y is not None else (x if x is not None else dy)
        dy = _like(dy, ref)
        need_x, need_s, need_b, need_add = ctx.needs_input_grad[:4]
        need_add = need_add and has_add
        # out1 = dpre * s, out2 = dpre (dpre = dy masked by the relu)
        if ctx.relu:
            want1, want2 = (need_x, need_add) if has_s else (need_x or need_add, False)
        else:
            want1, want2 = need_x and has_s, False
        o1, o2, sums = _ops().fx_affine_bwd(dy, s, y, x, want1, want2, bm, has_post, None)
        dx = (o1 if want1 else dy) if need_x else None
        dadd = None
        if need_add:
            dadd = (o2 if has_s else o1) if ctx.relu else dy
        ds = sums[1:2].view_as(s) if (has_s and need_s and not has_post) else None
        db = sums[0:1] if (has_b and need_b) else None
        dpost = sums[1:2] if (has_post and ctx.needs_input_grad[5]) else None
        return dx, ds, db, dadd, None, dpost


class _FxForkBias(torch.autograd.Function):
    """(x + b, x) for a residual block whose input feeds both its first conv
    (through the input bias) and the identity shortcut: the backward takes
    both gradients and writes dx = dxa + didentity with b's gradient sum dxa
    in ONE pass (fa_affine_bwd's add2) -- no separate sum pass and no
    autograd accumulation pass over the block input."""

    @staticmethod
    def forward(ctx, x, b):
        return _ops().fx_affine(x, None, b, None, False, None), x.view_as(x)

    @staticmethod
    def backward(ctx, dxa, did):
        ref = dxa if dxa is not None else did
        if dxa is None:
            return did, torch.zeros(1, device=did.device, dtype=torch.float32) if ctx.needs_input_grad[1] else None
        dxa = _like(dxa, ref)
        add2 = _like(did, dxa) if did is not None else None
        o1, _, sums = _ops().fx_affine_bwd(dxa, None, None, None, add2 is not None, False, None, False, add2)
        dx = o1 if add2 is not None else dxa
        return dx, (sums[0:1] if ctx.needs_input_grad[1] else None)


def fork_bias(x: torch.Tensor, b: torch.Tensor):
    """(x + b, x): a block input's biased copy and its identity shortcut with
    their two gradients summed in the bias's backward pass (native path)."""
    if _FORK and native_ok(x, b) and x.requires_grad:
        return _FxForkBias.apply(x, b.view(1))
    return scalar_affine(x, b=b), x


def native_ok(x: torch.Tensor, *others) -> bool:
    if (_nn.stock_active() or _nn.vmap_native_active() or not x.is_cuda or x.dtype != torch.bfloat16
            or x.numel() % 8 or x.numel() == 0 or not _dense(x)
            or x.data_ptr() % 16):
        return False
    for t in others:
        if t is None:
            continue
        if t.dim() == 1 and t.numel() == 1:  # a scalar parameter
            if t.dtype != torch.float32 or not t.is_cuda:
                return False
            gg = _grouped.active() if t.requires_grad else None
            if gg is not None and gg.view(t) is not None:
                return False  # per-group scalar gradients: the composition
        elif t.shape != x.shape or t.stride() != x.stride() or t.dtype != x.dtype or t.data_ptr() % 16:
            return False
    return True


def scalar_affine(x: torch.Tensor, s: Optional[torch.Tensor] = None, b: Optional[torch.Tensor] = None,
                  add: Optional[torch.Tensor] = None, relu: bool = False,
                  post: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``relu?(x * s + b + add) (+ post)`` with fp32 scalar parameters ``s`` /
    ``b`` / ``post`` (any may be None) and an optional residual ``add`` shaped
    like x.  ``post`` (the next conv's input bias) follows a relu."""
    if post is not None and (s is not None or add is not None or not relu):
        return scalar_affine(scalar_affine(x, s, b, add, relu), b=post)
    if x.is_cuda and x.dtype == torch.bfloat16 and not _dense(x):
        # (e.g. the augmentation kernel's images, channels innermost in a wider pixel)
        cl = x.dim() == 4 and x.stride(1) == 1
        x = x.contiguous(memory_format=torch.channels_last if cl else torch.contiguous_format)
    if add is not None and native_ok(x, s, b) and add.is_cuda and add.shape == x.shape:
        add = _like(add, x)
    if native_ok(x, s, b, add, post):
        if b is not None:
            b = b.view(1)
        if post is not None:
            post = post.view(1)
        return _FxAffine.apply(x, s, b, add, relu, post)
    y = x
    if s is not None:
        y = y * s
    if b is not None:
        y = y + b
    if add is not None:
        y = y + add
    y = F.relu(y) if relu else y
    return y + post if post is not None else y
