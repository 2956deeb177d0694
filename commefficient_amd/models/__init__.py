"""Model zoo and registry.

CLI choices are the registered names (like the reference's
``dir(models)`` filter, /root/reference/CommEfficient/utils.py:114-118).
``build_model(args, ...)`` reproduces cv_train's model_config construction
(cv_train.py:329-364) including the ``--test`` one-channel network.
"""
from __future__ import annotations

import torch.nn as nn

from .common import GhostBatchNorm2d, ghost_batchnorm, has_batchnorm
from .fixup import FixupResNet9, FixupResNet18, FixupResNet50, ResNet18
from .gpt2 import GPT2DoubleHeads
from .resnet9 import ResNet9
from .resnets import (ResNet, ResNet101, resnet18, resnet34, resnet50, resnet101, resnet152,
                      resnext50_32x4d, resnext101_32x8d, wide_resnet50_2, wide_resnet101_2)


class ResNet101LN(nn.Module):
    """FEMNIST ResNet-101 with LayerNorm (reference models/resnet101ln.py:7-13):
    1 input channel, 28x28, 62 classes -> 43,124,350 params."""

    def __init__(self, *args, num_classes=62, initial_channels=1, input_hw=28, **kwargs):
        super().__init__()
        self.model = resnet101(num_classes=num_classes, norm="ln", in_channels=initial_channels,
                               input_hw=input_hw)

    def forward(self, x):
        return self.model(x)


MODELS = {
    "ResNet9": ResNet9,
    "FixupResNet9": FixupResNet9,
    "FixupResNet18": FixupResNet18,
    "ResNet18": ResNet18,
    "FixupResNet50": FixupResNet50,
    "ResNet101LN": ResNet101LN,
    "ResNet101": ResNet101,
    "ResNet": ResNet,
    "GPT2DoubleHeads": GPT2DoubleHeads,
}


def model_names():
    return sorted(MODELS.keys())


def get_model_class(name: str):
    return MODELS[name]


def cv_model_config(args, num_classes: int, num_new_classes=None):
    """cv_train.py:329-357."""
    if getattr(args, "do_test", False):
        cfg = {"channels": {"prep": 1, "layer1": 1, "layer2": 1, "layer3": 1}}
    else:
        cfg = {"channels": {"prep": 64, "layer1": 128, "layer2": 256, "layer3": 512}}
    cfg.update({"num_classes": num_classes, "new_num_classes": num_new_classes,
                "bn_bias_freeze": args.do_finetune, "bn_weight_freeze": args.do_finetune})
    if args.dataset_name == "EMNIST":
        cfg["initial_channels"] = 1
    cfg["do_batchnorm"] = args.do_batchnorm
    return cfg


def build_model(args, num_classes: int, num_new_classes=None) -> nn.Module:
    cls = MODELS[args.model]
    cfg = cv_model_config(args, num_classes, num_new_classes)
    if cls is ResNet:
        return resnet18(num_classes=num_classes, in_channels=cfg.get("initial_channels", 3))
    return cls(**cfg)


__all__ = ["MODELS", "model_names", "get_model_class", "build_model", "cv_model_config",
           "ResNet9", "FixupResNet9", "FixupResNet18", "ResNet18", "FixupResNet50",
           "ResNet101LN", "ResNet101", "ResNet", "GPT2DoubleHeads", "GhostBatchNorm2d",
           "ghost_batchnorm", "has_batchnorm"]
