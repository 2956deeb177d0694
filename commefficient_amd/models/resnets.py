"""ResNet family (BasicBlock / Bottleneck) with BatchNorm or LayerNorm.

Equivalent of /root/reference/CommEfficient/models/resnets.py:25-370 (a
torchvision copy modified for LayerNorm with explicit spatial sizes).  Here the
spatial sizes are derived from ``input_hw`` instead of being hard-coded for a
28x28 input, ``in_channels`` is a parameter (the reference hard-codes 1 for
FEMNIST, resnets.py:155), and BasicBlock also supports LayerNorm (the
reference passes ``hw`` into BasicBlock's ``stride`` slot).  With
``in_channels=1, input_hw=28, norm="ln", num_classes=62`` ResNet-101 has the
reference's 43,124,350 parameters; with BatchNorm, 3 channels and 1000 classes
it is the standard 44,549,160-parameter ImageNet ResNet-101.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from .common import (GhostBatchNorm2d, NativeConv2d, NativeLinear, NativeMaxPool2d, conv1x1,
                     conv3x3)

__all__ = ["ResNet", "ResNet101", "resnet18", "resnet34", "resnet50", "resnet101", "resnet152",
           "resnext50_32x4d", "resnext101_32x8d", "wide_resnet50_2", "wide_resnet101_2"]


def _norm(kind: str, c: int, hw: int, relu: bool = False):
    """Normalisation layer; ``relu`` marks a BN followed by ReLU (fused into
    one native kernel each way; LayerNorm keeps the separate ReLU)."""
    if kind == "bn":
        return GhostBatchNorm2d(c, fuse_relu=relu)
    if kind == "ln":
        return nn.LayerNorm((c, hw, hw))
    raise ValueError(kind)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, hw, stride=1, downsample=None, groups=1, base_width=64,
                 dilation=1, norm="bn"):
        super().__init__()
        if groups != 1 or base_width != 64:
            raise ValueError("BasicBlock only supports groups=1 and base_width=64")
        out_hw = math.ceil(hw / stride)
        self.conv1 = conv3x3(inplanes, planes, stride)
        self.bn1 = _norm(norm, planes, out_hw, relu=True)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = conv3x3(planes, planes)
        self.bn2 = _norm(norm, planes, out_hw)
        self.downsample = downsample

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        out = _norm_relu(self.bn1, self.relu, self.conv1(x))
        return _norm_add_relu(self.bn2, self.relu, self.conv2(out), idt)


def _norm_relu(norm: nn.Module, relu: nn.Module, x):
    """relu(norm(x)); a fused GhostBatchNorm2d already applied the ReLU."""
    y = norm(x)
    return y if getattr(norm, "fuse_relu", False) else relu(y)


def _norm_add_relu(norm: nn.Module, relu: nn.Module, x, idt):
    """relu(norm(x) + idt): one native pass each way with GhostBatchNorm2d
    (the residual add and the ReLU in the BN apply kernels)."""
    if isinstance(norm, GhostBatchNorm2d):
        return norm(x, addend=idt)
    return relu(norm(x) + idt)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, hw, stride=1, downsample=None, groups=1, base_width=64,
                 dilation=1, norm="bn"):
        super().__init__()
        width = int(planes * (base_width / 64.0)) * groups
        out_hw = math.ceil(hw / stride)
        self.conv1 = conv1x1(inplanes, width)
        self.bn1 = _norm(norm, width, hw, relu=True)
        self.conv2 = NativeConv2d(width, width, 3, stride=stride, padding=dilation,
                                  groups=groups, bias=False, dilation=dilation)
        self.bn2 = _norm(norm, width, out_hw, relu=True)
        self.conv3 = conv1x1(width, planes * self.expansion)
        self.bn3 = _norm(norm, planes * self.expansion, out_hw)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample

    def forward(self, x):
        if self.downsample is None:
            # conv1 hands x through to the identity branch: its dgrad GEMM
            # adds the identity gradient (no separate accumulation pass)
            h, idt = self.conv1.forward_with_identity(x)
        elif (isinstance(self.downsample, nn.Sequential) and len(self.downsample) == 2
              and isinstance(self.downsample[0], NativeConv2d) and isinstance(self.conv1, NativeConv2d)):
            # conv1 and the shortcut conv read x: one input-gradient pass
            h, d = self.conv1.forward_pair(self.downsample[0], x)
            idt = self.downsample[1](d)
        else:
            h, idt = self.conv1(x), self.downsample(x)
        out = _norm_relu(self.bn1, self.relu, h)
        out = _norm_relu(self.bn2, self.relu, self.conv2(out))
        return _norm_add_relu(self.bn3, self.relu, self.conv3(out), idt)


class ResNet(nn.Module):
    def __init__(self, block=Bottleneck, layers=(3, 4, 23, 3), num_classes=1000,
                 zero_init_residual=False, groups=1, width_per_group=64, norm="bn",
                 in_channels=3, input_hw=224, norm_layer=None, **kw):
        super().__init__()
        if norm_layer is not None:  # reference-style argument
            norm = "ln" if norm_layer is nn.LayerNorm else "bn"
        self.norm = norm
        self.inplanes = 64
        self.groups = groups
        self.base_width = width_per_group
        self.conv1 = NativeConv2d(in_channels, 64, kernel_size=7, stride=2, padding=3, bias=False)
        hw = (input_hw + 2 * 3 - 7) // 2 + 1
        self.bn1 = _norm(norm, 64, hw, relu=True)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = NativeMaxPool2d(kernel_size=3, stride=2, padding=1)
        hw = (hw + 2 - 3) // 2 + 1
        self.layer1, hw = self._make_layer(block, 64, layers[0], hw)
        self.layer2, hw = self._make_layer(block, 128, layers[1], hw, stride=2)
        self.layer3, hw = self._make_layer(block, 256, layers[2], hw, stride=2)
        self.layer4, hw = self._make_layer(block, 512, layers[3], hw, stride=2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = NativeLinear(512 * block.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, (nn.BatchNorm2d, nn.GroupNorm)):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck) and norm == "bn":
                    nn.init.constant_(m.bn3.weight, 0)
                elif isinstance(m, BasicBlock) and norm == "bn":
                    nn.init.constant_(m.bn2.weight, 0)

    def _make_layer(self, block, planes, blocks, hw, stride=1):
        downsample = None
        out_hw = math.ceil(hw / stride)
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = nn.Sequential(conv1x1(self.inplanes, planes * block.expansion, stride),
                                       _norm(self.norm, planes * block.expansion, out_hw))
        layers = [block(self.inplanes, planes, hw, stride, downsample, self.groups,
                        self.base_width, 1, self.norm)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes, out_hw, groups=self.groups,
                                base_width=self.base_width, norm=self.norm))
        return nn.Sequential(*layers), out_hw

    def forward(self, x):
        x = self.maxpool(_norm_relu(self.bn1, self.relu, self.conv1(x)))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.fc(torch.flatten(self.avgpool(x), 1))


def _mk(block, layers, **kw):
    kw.pop("pretrained", None)
    kw.pop("progress", None)
    return ResNet(block, layers, **kw)


def resnet18(**kw): return _mk(BasicBlock, [2, 2, 2, 2], **kw)
def resnet34(**kw): return _mk(BasicBlock, [3, 4, 6, 3], **kw)
def resnet50(**kw): return _mk(Bottleneck, [3, 4, 6, 3], **kw)
def resnet101(**kw): return _mk(Bottleneck, [3, 4, 23, 3], **kw)
def resnet152(**kw): return _mk(Bottleneck, [3, 8, 36, 3], **kw)
def resnext50_32x4d(**kw): return _mk(Bottleneck, [3, 4, 6, 3], groups=32, width_per_group=4, **kw)
def resnext101_32x8d(**kw): return _mk(Bottleneck, [3, 4, 23, 3], groups=32, width_per_group=8, **kw)
def wide_resnet50_2(**kw): return _mk(Bottleneck, [3, 4, 6, 3], width_per_group=128, **kw)
def wide_resnet101_2(**kw): return _mk(Bottleneck, [3, 4, 23, 3], width_per_group=128, **kw)


class ResNet101(ResNet):
    """ImageNet-shaped ResNet-101 (BatchNorm, 3x224x224) -- BASELINE config 3."""

    def __init__(self, num_classes=1000, initial_channels=3, do_batchnorm=True, **kw):
        for k in ("channels", "new_num_classes", "bn_bias_freeze", "bn_weight_freeze"):
            kw.pop(k, None)
        super().__init__(Bottleneck, [3, 4, 23, 3], num_classes=num_classes,
                         in_channels=initial_channels, input_hw=kw.pop("input_hw", 224), norm="bn")
