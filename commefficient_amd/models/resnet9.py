"""ResNet-9 (the cifar10-fast "Page" net) -- the flagship FetchSGD model.

Architecture and parameter names follow /root/reference/CommEfficient/models/
resnet9.py:32-148 so ``state_dict`` keys (``n.prep.conv.weight`` ...) and the
flat parameter order match the reference checkpoint format:
prep(c_in->64) -> layer1(64->128, pool) + res1 -> layer2(128->256, pool) ->
layer3(256->512, pool) + res3 -> maxpool 4 -> linear(512->classes, no bias) -> ×0.125.
BatchNorm is off unless ``do_batchnorm`` (cv_train.py:357).  6,568,640 params
for 10 classes.

MI355X notes: conv+ReLU(+maxpool) units run on the native MFMA implicit-GEMM
kernels of csrc/conv.hip (bf16 channels_last, fused epilogues), the 3-channel
prep conv on csrc/conv_prep.hip; BatchNorm variants use MIOpen.  Fixes reference
quirk Appendix C #12: ``finetune_parameters`` no longer touches an undefined
``self.iid``.
"""
from __future__ import annotations

import itertools

import torch.nn as nn
import torch.nn.functional as F

from ..ops.nn import (conv3x3_input_relu, conv3x3_relu_pool, cross_entropy_correct,
                      fused_head_loss, head_native_ok, input_conv_native_ok,
                      prepared_conv_weights, relu_maxpool, residual_unit)
from .common import GhostBatchNorm2d, Mul

__all__ = ["ResNet9"]


def _k(pool: nn.MaxPool2d) -> int:
    k = pool.kernel_size
    return k if isinstance(k, int) else k[0]


def _square_pool(pool: nn.MaxPool2d) -> bool:
    k, s = pool.kernel_size, pool.stride
    k = k if isinstance(k, int) else (k[0] if k[0] == k[1] else -1)
    s = s if isinstance(s, int) else (s[0] if s[0] == s[1] else -2)
    return k == s and pool.padding in (0, (0, 0)) and pool.dilation in (1, (1, 1))

DEFAULT_CHANNELS = {"prep": 64, "layer1": 128, "layer2": 256, "layer3": 512}


def _bn(c, bn_bias_init=None, bn_bias_freeze=False, bn_weight_init=None, bn_weight_freeze=False):
    m = GhostBatchNorm2d(c)
    if bn_bias_init is not None:
        nn.init.constant_(m.bias, bn_bias_init)
    if bn_weight_init is not None:
        nn.init.constant_(m.weight, bn_weight_init)
    m.bias.requires_grad = not bn_bias_freeze
    m.weight.requires_grad = not bn_weight_freeze
    return m


class ConvBN(nn.Module):
    def __init__(self, do_batchnorm, c_in, c_out, bn_weight_init=1.0, pool=None, **kw):
        super().__init__()
        self.pool = pool
        self.conv = nn.Conv2d(c_in, c_out, kernel_size=3, padding=1, bias=False)
        self.do_batchnorm = do_batchnorm
        if do_batchnorm:
            self.bn = _bn(c_out, bn_weight_init=bn_weight_init, **kw)

    def forward(self, x):
        if not self.do_batchnorm and self.pool is None and input_conv_native_ok(x, self.conv.weight):
            # the 3-channel input conv: native kernel reading the augmentation
            # kernel's padded pixels (csrc/conv_prep.hip)
            return conv3x3_input_relu(x, self.conv.weight)
        if not self.do_batchnorm and (self.pool is None or (
                isinstance(self.pool, nn.MaxPool2d) and _square_pool(self.pool))):
            # conv + relu (+ pool) as one unit: native MFMA conv kernels with
            # fused epilogues when the shapes fit (csrc/conv.hip), else MIOpen
            return conv3x3_relu_pool(x, self.conv.weight,
                                     _k(self.pool) if self.pool is not None else 0)
        x = self.conv(x)
        if self.do_batchnorm:
            x = self.bn(x)
        if isinstance(self.pool, nn.MaxPool2d) and _square_pool(self.pool):
            # fused relu + maxpool (native NHWC bf16 kernels on GPU)
            return relu_maxpool(x, _k(self.pool))
        x = F.relu(x, inplace=True)
        return self.pool(x) if self.pool is not None else x


class Residual(nn.Module):
    def __init__(self, do_batchnorm, c, **kw):
        super().__init__()
        self.res1 = ConvBN(do_batchnorm, c, c, **kw)
        self.res2 = ConvBN(do_batchnorm, c, c, **kw)

    def forward(self, x):
        # reference: x + relu(res2(res1(x))); res2 already ends in a ReLU, so
        # the outer one is the identity and is dropped (saves a fwd+bwd pass
        # over the activation)
        if not self.res1.do_batchnorm:
            # one native unit: skip-add and relu masks fused into conv epilogues
            return residual_unit(x, self.res1.conv.weight, self.res2.conv.weight)
        return x + self.res2(self.res1(x))


class BasicNet(nn.Module):
    def __init__(self, do_batchnorm, channels, weight, pool, num_classes, initial_channels=3,
                 new_num_classes=None, **kw):
        super().__init__()
        self.new_num_classes = new_num_classes
        self.prep = ConvBN(do_batchnorm, initial_channels, channels["prep"], **kw)
        self.layer1 = ConvBN(do_batchnorm, channels["prep"], channels["layer1"], pool=pool, **kw)
        self.res1 = Residual(do_batchnorm, channels["layer1"], **kw)
        self.layer2 = ConvBN(do_batchnorm, channels["layer1"], channels["layer2"], pool=pool, **kw)
        self.layer3 = ConvBN(do_batchnorm, channels["layer2"], channels["layer3"], pool=pool, **kw)
        self.res3 = Residual(do_batchnorm, channels["layer3"], **kw)
        self.pool = nn.MaxPool2d(4)
        self.linear = nn.Linear(channels["layer3"], num_classes, bias=False)
        self.classifier = Mul(weight)

    def conv_weights(self):
        return [m.weight for m in self.modules() if isinstance(m, nn.Conv2d)]

    def features(self, x):
        # every conv weight -> bf16 GEMM images in one launch (native path)
        with prepared_conv_weights(self.conv_weights() if x.is_cuda else []):
            x = self.prep(x)
            x = self.res1(self.layer1(x))
            x = self.layer2(x)
            return self.res3(self.layer3(x))

    def head(self, x):
        # res3's output is >= 0 (relu'd input + relu'd branch), so relu is the
        # identity and the fused kernel computes exactly max_pool2d(x, 4)
        x = relu_maxpool(x, 4).flatten(1)
        return self.classifier(self.linear(x))

    def forward(self, x):
        return self.head(self.features(x))

    def loss(self, x, targets):
        """(per-example CE loss, top-1 correct): with the final pool covering
        the whole 4x4 map, the head + loss run as one native kernel each way
        (csrc/head.hip); otherwise the module head + fused CE."""
        f = self.features(x)
        if (f.shape[2] == 4 and f.shape[3] == 4 and head_native_ok(f, self.linear.weight)
                and self.linear.bias is None and isinstance(self.classifier, Mul)):
            return fused_head_loss(f, self.linear.weight, targets, self.classifier.weight)
        return cross_entropy_correct(self.head(f), targets)


class ResNet9(nn.Module):
    def __init__(self, do_batchnorm=False, channels=None, weight=0.125, pool=None,
                 num_classes=10, new_num_classes=None, initial_channels=3,
                 bn_bias_freeze=False, bn_weight_freeze=False, **kw):
        super().__init__()
        self.channels = dict(channels or DEFAULT_CHANNELS)
        self.weight = weight
        pool = pool if pool is not None else nn.MaxPool2d(2)
        bn_kw = {}
        if do_batchnorm:
            bn_kw = dict(bn_bias_freeze=bn_bias_freeze, bn_weight_freeze=bn_weight_freeze)
        self.n = BasicNet(do_batchnorm, self.channels, weight, pool, num_classes,
                          initial_channels=initial_channels, new_num_classes=new_num_classes,
                          **bn_kw)

    def forward(self, x):
        return self.n(x)

    def loss(self, x, targets):
        return self.n.loss(x, targets)

    def finetune_parameters(self):
        """Replace the head for ``new_num_classes`` and return its params
        (reference resnet9.py:105-113)."""
        n_new = self.n.new_num_classes or self.n.linear.out_features
        self.n.linear = nn.Linear(self.channels["layer3"], n_new, bias=False).to(
            self.n.linear.weight.device)
        self.n.classifier = Mul(self.weight)
        for p in self.n.linear.parameters():
            p.requires_grad = True
        return itertools.chain(self.n.linear.parameters())
