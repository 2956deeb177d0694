"""Fixup-initialised residual networks, implemented natively (the reference
imports them from the external, unvendored ``fixup`` package:
/root/reference/CommEfficient/models/fixup_resnet9.py:6,
fixup_resnet.py:4).

* ``FixupResNet9``  -- ResNet-9 topology with Fixup scalar biases/scales
  (reference fixup_resnet9.py:33-91).  Unlike the reference its constructor
  accepts cv_train's model_config kwargs (Appendix C #12) and ``num_classes``.
* ``FixupResNet18`` / ``ResNet18`` -- the reference's CIFAR variants with a
  256-channel last stage and avg||max pooling into Linear(512)
  (fixup_resnet18.py:24-216).
* ``FixupResNet50`` -- ImageNet Fixup bottleneck ResNet-50 (fixup_resnet.py:8-10).

Fixup init (Zhang et al. 2019): the first conv of each residual branch is He
init scaled by L^(-1/(2m-2)) (m = convs per branch), the last conv and the
classifier are zero-initialised.

The scalar biases / scales run as ``ops.fixup.scalar_affine``: one bf16 pass
each way on a GPU (the activations stay bf16, so every conv stays on the
native kernels), the PyTorch composition elsewhere.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.fixup import fork_bias as _fork
from ..ops.fixup import scalar_affine as _sa
from ..ops.nn import relu_maxpool
from .common import (GhostBatchNorm2d, NativeConv2d, NativeLinear, NativeMaxPool2d, ScalarBias,
                     ScalarScale, conv1x1, conv3x3)

__all__ = ["FixupResNet9", "FixupResNet18", "ResNet18", "FixupResNet50"]


def _he_std(conv: nn.Conv2d) -> float:
    return float(np.sqrt(2.0 / (conv.weight.shape[0] * np.prod(conv.weight.shape[2:]))))


class FixupBasicBlock(nn.Module):
    """x -> +b1a -> conv -> +b1b -> relu -> +b2a -> conv -> *s -> +b2b -> (+x) -> relu."""

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.bias1a = nn.Parameter(torch.zeros(1))
        self.conv1 = conv3x3(inplanes, planes, stride)
        self.bias1b = nn.Parameter(torch.zeros(1))
        self.bias2a = nn.Parameter(torch.zeros(1))
        self.conv2 = conv3x3(planes, planes)
        self.scale = nn.Parameter(torch.ones(1))
        self.bias2b = nn.Parameter(torch.zeros(1))
        self.downsample = downsample

    def forward(self, x):
        if self.downsample is None:  # (x + b1a and the identity: one backward pass)
            xa, idt = _fork(x, self.bias1a)
        else:
            xa = _sa(x, b=self.bias1a)
            idt = self.downsample(xa)
        out = _sa(self.conv1(xa), b=self.bias1b, relu=True, post=self.bias2a)
        return _sa(self.conv2(out), s=self.scale, b=self.bias2b, add=idt, relu=True)


class FixupLayer(nn.Module):
    """conv, bias, relu, pool, then num_blocks FixupBasicBlocks."""

    def __init__(self, c_in, c_out, num_blocks, pool):
        super().__init__()
        self.conv = conv3x3(c_in, c_out)
        self.bias1a = nn.Parameter(torch.zeros(1))
        self.bias1b = nn.Parameter(torch.zeros(1))
        self.scale = nn.Parameter(torch.ones(1))
        self.pool = pool
        self.blocks = nn.Sequential(*[FixupBasicBlock(c_out, c_out) for _ in range(num_blocks)])

    def forward(self, x):
        out = self.conv(_sa(x, b=self.bias1a))
        k = _pool2(self.pool)
        if k:  # relu then max-pool, one native pass each way
            out = relu_maxpool(_sa(out, s=self.scale, b=self.bias1b), k)
        else:
            out = _sa(out, s=self.scale, b=self.bias1b, relu=True)
            if self.pool is not None:
                out = self.pool(out)
        return self.blocks(out)


def _pool2(pool) -> int:
    """k of a plain non-overlapping k x k max-pool (else 0)."""
    if type(pool) is not nn.MaxPool2d or pool.padding not in (0, (0, 0)) or pool.dilation not in (1, (1, 1)) \
            or pool.ceil_mode or pool.return_indices:
        return 0
    k, st = pool.kernel_size, pool.stride
    k = k if isinstance(k, int) else (k[0] if k[0] == k[1] else 0)
    st = st if isinstance(st, int) else (st[0] if st[0] == st[1] else -1)
    return k if st == k else 0


class FixupResNet9(nn.Module):
    def __init__(self, channels=None, pool=None, num_classes=10, initial_channels=3, **kw):
        super().__init__()
        self.num_layers = 2
        ch = channels or {"prep": 64, "layer1": 128, "layer2": 256, "layer3": 512}
        self.channels = ch
        pool = pool if pool is not None else nn.MaxPool2d(2)
        self.conv1 = conv3x3(initial_channels, ch["prep"])
        self.bias1a = nn.Parameter(torch.zeros(1))
        self.bias1b = nn.Parameter(torch.zeros(1))
        self.scale = nn.Parameter(torch.ones(1))
        self.layer1 = FixupLayer(ch["prep"], ch["layer1"], 1, pool)
        self.layer2 = FixupLayer(ch["layer1"], ch["layer2"], 0, pool)
        self.layer3 = FixupLayer(ch["layer2"], ch["layer3"], 1, pool)
        self.pool = nn.MaxPool2d(4)
        self.bias2 = nn.Parameter(torch.zeros(1))
        self.linear = nn.Linear(ch["layer3"], num_classes)
        nn.init.normal_(self.conv1.weight, 0, _he_std(self.conv1))
        for m in self.modules():
            if isinstance(m, FixupBasicBlock):
                nn.init.normal_(m.conv1.weight, 0, _he_std(m.conv1) * self.num_layers ** (-0.5))
                nn.init.constant_(m.conv2.weight, 0)
            elif isinstance(m, FixupLayer):
                nn.init.normal_(m.conv.weight, 0, _he_std(m.conv))
            elif isinstance(m, nn.Linear):
                nn.init.constant_(m.weight, 0)
                nn.init.constant_(m.bias, 0)

    def forward(self, x):
        out = _sa(self.conv1(_sa(x, b=self.bias1a)), s=self.scale, b=self.bias1b, relu=True)
        out = self.layer3(self.layer2(self.layer1(out)))
        k = _pool2(self.pool)
        out = (relu_maxpool(out, k) if k else self.pool(out)).flatten(1)  # (out >= 0: relu is exact)
        return self.linear(_sa(out, b=self.bias2))


# ---------------------------------------------------------------- ResNet-18s
class FixupBlock18(nn.Module):
    """Reference fixup_resnet18.py:24-63 (module names add1a/conv1/add1b/add2a/conv2/mul/add2b)."""

    def __init__(self, in_channels, out_channels, stride=1):
        super().__init__()
        self.add1a = ScalarBias()
        self.conv1 = conv3x3(in_channels, out_channels, stride)
        self.add1b = ScalarBias()
        self.add2a = ScalarBias()
        self.conv2 = conv3x3(out_channels, out_channels)
        self.mul = ScalarScale()
        self.add2b = ScalarBias()
        if stride != 1 or in_channels != out_channels:
            self.shortcut = conv1x1(in_channels, out_channels, stride)

    def forward(self, x):
        if hasattr(self, "shortcut"):
            sc, xa = self.shortcut(x), _sa(x, b=self.add1a.bias)
        else:
            xa, sc = _fork(x, self.add1a.bias)
        out = _sa(self.conv1(xa), b=self.add1b.bias, relu=True, post=self.add2a.bias)
        out = self.conv2(out)
        return _sa(out, s=self.mul.scale, b=self.add2b.bias, add=sc, relu=True)


class PreActBlock(nn.Module):
    """Reference fixup_resnet18.py:138-165 (conv-bn-relu x2 + shortcut)."""

    def __init__(self, in_channels, out_channels, stride=1):
        super().__init__()
        # BN + ReLU fused (one native kernel each way in merged rounds)
        self.bn1 = GhostBatchNorm2d(out_channels, fuse_relu=True)
        self.conv1 = conv3x3(in_channels, out_channels, stride)
        self.bn2 = GhostBatchNorm2d(out_channels, fuse_relu=True)
        self.conv2 = conv3x3(out_channels, out_channels)
        if stride != 1 or in_channels != out_channels:
            self.shortcut = nn.Sequential(conv1x1(in_channels, out_channels, stride))

    def forward(self, x):
        out = self.bn1(self.conv1(x))  # relu(bn(.))
        out = self.bn2(self.conv2(out))
        sc = self.shortcut(x) if hasattr(self, "shortcut") else x
        return out + sc


def _avg_max_head(x):
    return torch.cat([F.adaptive_avg_pool2d(x, 1).flatten(1), F.adaptive_max_pool2d(x, 1).flatten(1)], -1)


class _ResNet18Base(nn.Module):
    widths = (64, 128, 256, 256)

    def _make(self, block, num_blocks):
        layers, c_in = [], 64
        for i, (w, n) in enumerate(zip(self.widths, num_blocks)):
            stride = 1 if i == 0 else 2
            blocks = []
            for s in [stride] + [1] * (n - 1):
                blocks.append(block(c_in, w, s))
                c_in = w
            layers.append(nn.Sequential(*blocks))
        return nn.Sequential(*layers)


class FixupResNet18(_ResNet18Base):
    def __init__(self, num_blocks=(2, 2, 2, 2), num_classes=10, initial_channels=3, **kw):
        super().__init__()
        self.num_layers = sum(num_blocks)
        self.prep = conv3x3(initial_channels, 64)
        self.layers = self._make(FixupBlock18, num_blocks)
        self.classifier = NativeLinear(512, num_classes)
        for m in self.modules():
            if isinstance(m, FixupBlock18):
                nn.init.normal_(m.conv1.weight, 0, _he_std(m.conv1) * self.num_layers ** (-0.5))
                nn.init.constant_(m.conv2.weight, 0)
                if hasattr(m, "shortcut"):
                    nn.init.normal_(m.shortcut.weight, 0, _he_std(m.shortcut))
            elif isinstance(m, nn.Linear):
                nn.init.constant_(m.weight, 0)
                nn.init.constant_(m.bias, 0)
        nn.init.normal_(self.prep.weight, 0, _he_std(self.prep))

    def forward(self, x):
        x = self.layers(F.relu(self.prep(x)))
        return self.classifier(_avg_max_head(x))


class ResNet18(_ResNet18Base):
    def __init__(self, num_blocks=(2, 2, 2, 2), num_classes=10, initial_channels=3, **kw):
        super().__init__()
        self.prep = nn.Sequential(conv3x3(initial_channels, 64), nn.ReLU())
        self.layers = self._make(PreActBlock, num_blocks)
        self.classifier = NativeLinear(512, num_classes)

    def forward(self, x):
        return self.classifier(_avg_max_head(self.layers(self.prep(x))))


# ---------------------------------------------------------------- ResNet-50
class FixupBottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.bias1a = nn.Parameter(torch.zeros(1))
        self.conv1 = conv1x1(inplanes, planes)
        self.bias1b = nn.Parameter(torch.zeros(1))
        self.bias2a = nn.Parameter(torch.zeros(1))
        self.conv2 = conv3x3(planes, planes, stride)
        self.bias2b = nn.Parameter(torch.zeros(1))
        self.bias3a = nn.Parameter(torch.zeros(1))
        self.conv3 = conv1x1(planes, planes * self.expansion)
        self.scale = nn.Parameter(torch.ones(1))
        self.bias3b = nn.Parameter(torch.zeros(1))
        self.downsample = downsample

    def forward(self, x):
        if self.downsample is not None:
            # conv1 and the shortcut read xa: one node, input gradients summed in the dgrad GEMM
            xa = _sa(x, b=self.bias1a)
            out, idt = self.conv1.forward_pair(self.downsample, xa)
        else:
            # x + b1a and the identity: their gradients summed in the bias's backward pass
            xa, idt = _fork(x, self.bias1a)
            out = self.conv1(xa)
        out = _sa(out, b=self.bias1b, relu=True, post=self.bias2a)
        out = _sa(self.conv2(out), b=self.bias2b, relu=True, post=self.bias3a)
        return _sa(self.conv3(out), s=self.scale, b=self.bias3b, add=idt, relu=True)


class FixupResNet(nn.Module):
    def __init__(self, block, layers, num_classes=1000, initial_channels=3, **kw):
        super().__init__()
        self.num_layers = sum(layers)
        self.inplanes = 64
        self.conv1 = NativeConv2d(initial_channels, 64, kernel_size=7, stride=2, padding=3, bias=False)
        self.bias1 = nn.Parameter(torch.zeros(1))
        self.maxpool = NativeMaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.bias2 = nn.Parameter(torch.zeros(1))
        self.fc = NativeLinear(512 * block.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, FixupBottleneck):
                f = self.num_layers ** (-0.25)
                nn.init.normal_(m.conv1.weight, 0, _he_std(m.conv1) * f)
                nn.init.normal_(m.conv2.weight, 0, _he_std(m.conv2) * f)
                nn.init.constant_(m.conv3.weight, 0)
                if m.downsample is not None:
                    nn.init.normal_(m.downsample.weight, 0, _he_std(m.downsample))
            elif isinstance(m, nn.Linear):
                nn.init.constant_(m.weight, 0)
                nn.init.constant_(m.bias, 0)

    def _make_layer(self, block, planes, blocks, stride=1):
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = conv1x1(self.inplanes, planes * block.expansion, stride)
        layers = [block(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes * block.expansion
        layers += [block(self.inplanes, planes) for _ in range(1, blocks)]
        return nn.Sequential(*layers)

    def forward(self, x):
        x = self.maxpool(_sa(self.conv1(x), b=self.bias1, relu=True))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.fc(_sa(self.avgpool(x).flatten(1), b=self.bias2))


class FixupResNet50(FixupResNet):
    def __init__(self, num_classes=1000, initial_channels=3, **kw):
        super().__init__(FixupBottleneck, [3, 4, 6, 3], num_classes=num_classes,
                         initial_channels=initial_channels)
