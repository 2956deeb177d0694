"""Shared building blocks for the model zoo."""
from __future__ import annotations

import contextlib

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import grouped as _grouped
from ..ops import nn as _nn
from ..ops.nn import (_AffineGrouped, conv1x1_passthrough, conv2d_grouped, conv2d_native,
                      conv2d_native_kind, ghost_batch_norm, ghost_bn_native_ok, linear_grouped,
                      max_pool2d, stock_active)


class Mul(nn.Module):
    """Constant scale (ResNet-9 classifier ×0.125)."""

    def __init__(self, weight: float):
        super().__init__()
        self.weight = weight

    def forward(self, x):
        return x * self.weight


class ScalarScale(nn.Module):
    """Learnable scalar multiplier (Fixup ``scale``)."""

    def __init__(self):
        super().__init__()
        self.scale = nn.Parameter(torch.ones(1))

    def forward(self, x):
        return x * self.scale


class ScalarBias(nn.Module):
    """Learnable scalar bias (Fixup ``bias``)."""

    def __init__(self):
        super().__init__()
        self.bias = nn.Parameter(torch.zeros(1))

    def forward(self, x):
        return x + self.bias


class GhostBatchNorm2d(nn.BatchNorm2d):
    """BatchNorm2d that can normalise G equal-size groups of the batch with
    their own statistics.

    The engine merges the clients of a round into one forward/backward when
    that is exact (parallel/fed_model.py).  With BatchNorm, "exact" means each
    client's examples are normalised with that client's batch statistics, as
    in the reference where every client runs its own forward
    (/root/reference/CommEfficient/fed_worker.py:162-176).  ``ghost_groups``
    is set by the engine for the duration of a merged forward.
    Running statistics are updated once with the group-averaged moments.
    """

    ghost_groups: int = 1

    def __init__(self, num_features, *args, fuse_relu: bool = False, **kw):
        super().__init__(num_features, *args, **kw)
        # relu(bn(x)) in one module (one native kernel each way when merged)
        self.fuse_relu = fuse_relu

    def forward(self, x, addend=None):
        """``addend``: a residual block's tail ``relu(bn(x) + addend)`` (one
        native pass each way; the module's own ``fuse_relu`` is ignored)."""
        if addend is not None:
            y, done = self._bn(x, addend)
            return y if done else F.relu(y + addend)
        y, relu_done = self._bn(x)
        return F.relu(y) if self.fuse_relu and not relu_done else y

    def _bn(self, x, addend=None):
        """(normalised x, whether the fused ReLU (and the addend) was applied)"""
        if stock_active():
            return self._bn_stock(x), False
        G = max(1, self.ghost_groups)
        gg = _grouped.active() if (self.training and self.affine) else None
        if gg is not None and gg.view(self.weight) is None:
            gg = None
        if (self.training and self.momentum is not None and x.shape[0] % G == 0
                and ghost_bn_native_ok(x, self.weight if self.affine else None)):
            # native per-group BN (csrc/bn.hip), also for one group (the
            # per-client path): MIOpen's bf16 NHWC BN took 5 launches + casts
            track = self.track_running_stats and self.running_mean is not None
            fused_add = addend is not None and addend.shape == x.shape and addend.is_cuda
            y = ghost_batch_norm(x, self.weight if self.affine else None,
                                 self.bias if self.affine else None, G, self.eps, self.momentum,
                                 self.running_mean if track else None,
                                 self.running_var if track else None,
                                 relu=fused_add or (self.fuse_relu and addend is None),
                                 num_batches_tracked=self.num_batches_tracked if track else None,
                                 gg=gg, addend=addend if fused_add else None,
                                 tstats=_nn.take_bnstats(x, G))
            return y, (fused_add or self.fuse_relu) if addend is None or fused_add else False
        if gg is None and (not self.training or G <= 1):
            return super().forward(x), False
        N, C = x.shape[0], x.shape[1]
        assert N % G == 0, "ghost batch norm needs equal client batch sizes"
        xf = x.float().reshape(G, N // G, C, -1)
        mean = xf.mean(dim=(1, 3), keepdim=True)
        var = xf.var(dim=(1, 3), keepdim=True, unbiased=False)
        y = (xf - mean) * torch.rsqrt(var + self.eps)
        if self.affine and gg is not None:  # per-group dweight / dbias
            y = _AffineGrouped.apply(y.reshape(N, C, -1), self.weight, self.bias, gg)
        elif self.affine:
            y = y * self.weight.view(1, 1, C, 1) + self.bias.view(1, 1, C, 1)
        if self.track_running_stats and self.running_mean is not None:
            with torch.no_grad():
                n = xf.shape[1] * xf.shape[3]
                self.num_batches_tracked += 1
                m = (self.momentum if self.momentum is not None
                     else 1.0 / float(self.num_batches_tracked.item()))
                self.running_mean.mul_(1 - m).add_(m * mean.mean(dim=0).view(C))
                unb = var.mean(dim=0).view(C) * (n / max(1, n - 1))
                self.running_var.mul_(1 - m).add_(m * unb)
        return y.reshape(x.shape).to(x.dtype).contiguous(memory_format=_fmt(x)), False


    def _bn_stock(self, x):
        """Batch norm as a plain fp32 composition (``ops.nn.stock_ops``: under
        torch.func.vmap each client's statistics and running-statistics
        buffers are its own batched slices; MIOpen's batch norm rejects the
        bf16 weights autocast + vmap hand it)."""
        C = x.shape[1]
        xf = x.float()
        if self.training or not self.track_running_stats or self.running_mean is None:
            mean = xf.mean(dim=(0, 2, 3))
            var = xf.var(dim=(0, 2, 3), unbiased=False)
            if self.training and self.track_running_stats and self.running_mean is not None:
                with torch.no_grad():
                    n = xf.numel() // C
                    self.num_batches_tracked.add_(1)
                    # momentum None: cumulative average (PyTorch's factor 1/num_batches_tracked)
                    m = (self.momentum if self.momentum is not None
                         else 1.0 / self.num_batches_tracked.double())
                    self.running_mean.mul_(1 - m).add_(mean.detach() * m)
                    self.running_var.mul_(1 - m).add_(var.detach() * (m * n / max(1, n - 1)))
        else:
            mean, var = self.running_mean, self.running_var
        y = (xf - mean.view(1, C, 1, 1)) * torch.rsqrt(var.view(1, C, 1, 1) + self.eps)
        if self.affine:
            y = y * self.weight.view(1, C, 1, 1) + self.bias.view(1, C, 1, 1)
        return y.to(x.dtype)


def _fmt(x):
    if x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last):
        return torch.channels_last
    return torch.contiguous_format


@contextlib.contextmanager
def ghost_batchnorm(model: nn.Module, groups: int):
    mods = [m for m in model.modules() if isinstance(m, GhostBatchNorm2d)]
    for m in mods:
        m.ghost_groups = groups
    # the native conv forwards also write their outputs' BN moments for these
    # groups (ops/nn.py _mm_nt_conv)
    prev = _nn._EPI["G"]
    _nn._EPI["G"] = groups if (mods and model.training) else 0
    try:
        yield
    finally:
        _nn._EPI["G"] = prev
        for m in mods:
            m.ghost_groups = 1


def has_batchnorm(model: nn.Module) -> bool:
    return any(isinstance(m, nn.modules.batchnorm._BatchNorm) for m in model.modules())


class NativeConv2d(nn.Conv2d):
    """``nn.Conv2d`` (same parameters / state_dict keys) whose bias-free,
    ungrouped convolutions of bf16 channels-innermost activations run native
    (ops/nn.py ``conv2d_native``): 1x1 as hipBLASLt GEMMs, stride-1 3x3 on the
    MFMA kernels of csrc/conv.hip, anything else (7x7 stems, strided 3x3) as
    column-image GEMMs (csrc/im2col.hip); grouped / dilated convs are the stock
    (MIOpen) convolution."""

    def forward(self, x):
        if (_nn.vmap_native_active() and self.bias is None and self.groups == 1
                and self.in_channels % 64 == 0 and self.out_channels % 64 == 0
                and tuple(self.kernel_size) == (3, 3) and tuple(self.stride) == (1, 1)
                and tuple(self.padding) == (1, 1) and tuple(self.dilation) == (1, 1)
                and self.padding_mode == "zeros"):
            # batched FedAvg under vmap: clients stacked along channels on the
            # grouped native kernels (ops/nn.py vmap_native_convs)
            return _nn.gconv3x3(x, self.weight)
        gg = _grouped.active() if self.weight.requires_grad else None
        if gg is not None and gg.view(self.weight) is None:
            gg = None
        if self.bias is None and self.padding_mode == "zeros":
            kind = conv2d_native_kind(x, self.weight, self.stride, self.padding, self.dilation,
                                      self.groups)
            if kind:
                return conv2d_native(x, self.weight, kind, self.stride[0], gg, self.padding[0])
            if gg is not None:
                return conv2d_grouped(x, self.weight, self.stride, self.padding, self.dilation,
                                      self.groups, gg)
        return super().forward(x)


    def forward_with_identity(self, x):
        """(conv(x), x): a 1x1 stride-1 conv on the native path returns the
        input through the same autograd node, so the residual block's two
        input gradients are summed inside the dgrad GEMM."""
        gg = _grouped.active() if self.weight.requires_grad else None
        if gg is not None and gg.view(self.weight) is None:
            gg = None
        if (self.bias is None and conv2d_native_kind(x, self.weight, self.stride, self.padding,
                                                     self.dilation, self.groups) == "1x1"
                and tuple(self.stride) == (1, 1)):
            return conv1x1_passthrough(x, self.weight, gg)
        return self(x), x


    def forward_pair(self, other: "NativeConv2d", x):
        """(self(x), other(x)) for two 1x1 convs of one input (a downsampling
        bottleneck's conv1 and shortcut conv): on the native path one autograd
        node whose backward sums the two input gradients inside the dgrad GEMM."""
        kinds = [conv2d_native_kind(x, m.weight, m.stride, m.padding, m.dilation, m.groups)
                 if m.bias is None and m.padding_mode == "zeros" else "" for m in (self, other)]
        if kinds == ["1x1", "1x1"] and tuple(self.stride) == (1, 1) and other.stride[0] == other.stride[1]:
            ggs = []
            for m in (self, other):
                gg = _grouped.active() if m.weight.requires_grad else None
                ggs.append(gg if gg is not None and gg.view(m.weight) is not None else None)
            return _nn.conv1x1_pair(x, self.weight, other.weight, other.stride[0], *ggs)
        return self(x), other(x)


class NativeMaxPool2d(nn.MaxPool2d):
    """``nn.MaxPool2d`` whose bf16 channels_last case runs the native
    max-pool (csrc/im2col.hip: window codes + gather backward)."""

    def forward(self, x):
        k, s, p = (self.kernel_size, self.stride, self.padding)
        if (isinstance(k, int) and isinstance(s, int) and isinstance(p, int)
                and self.dilation == 1 and not self.ceil_mode and not self.return_indices):
            return max_pool2d(x, k, s, p)
        return super().forward(x)


class NativeLinear(nn.Linear):
    """``nn.Linear`` that writes per-group weight gradients under
    ``ops.grouped.grouped_grads`` (one batched GEMM over the groups)."""

    def forward(self, x):
        gg = _grouped.active() if self.weight.requires_grad else None
        if gg is not None and gg.view(self.weight) is not None and (
                self.bias is None or gg.view(self.bias) is not None):
            return linear_grouped(x, self.weight, self.bias, gg)
        return super().forward(x)


GROUPED_MODULES = (NativeConv2d, NativeLinear)


def groupable(model: nn.Module) -> bool:
    """Every trainable parameter belongs to a module that can write per-group
    weight gradients (ops/grouped.py): NativeConv2d (no bias), NativeLinear,
    affine GhostBatchNorm2d."""
    for m in model.modules():
        own = [p for p in m.parameters(recurse=False) if p.requires_grad]
        if not own:
            continue
        if isinstance(m, NativeConv2d) and m.bias is None:
            continue
        if isinstance(m, NativeLinear):
            continue
        if isinstance(m, GhostBatchNorm2d) and m.affine:
            continue
        return False
    return True


def conv3x3(c_in, c_out, stride=1):
    return NativeConv2d(c_in, c_out, kernel_size=3, stride=stride, padding=1, bias=False)


def conv1x1(c_in, c_out, stride=1):
    return NativeConv2d(c_in, c_out, kernel_size=1, stride=stride, bias=False)
