"""Per-model training configurations (the reference's models/configs.py:1-37).

``ModelConfig.set_args`` copies a config's attributes onto the global args
namespace.  The reference module is unused and cannot import
(``PiecewiseLinear`` is never imported there); here it is
importable and ``get_config(name)`` returns the config of a model or None.
``FixupResNet50Config`` is the reference's ImageNet step schedule (0.1 divided
by 10 at epochs 30 / 60 / 90).
"""
from __future__ import annotations

from ..utils.schedules import PiecewiseLinear


class ModelConfig:
    def set_args(self, args):
        for name, val in self.__dict__.items():
            setattr(args, name, val)
        return args


class FixupResNet50Config(ModelConfig):
    def __init__(self):
        self.model_config = {}
        self.lr_scale = 0.1
        self.lr_schedule = PiecewiseLinear([0, 30, 30, 60, 60, 90, 90, 100],
                                           [0.1, 0.1, 0.01, 0.01, 0.001, 0.001, 0.0001, 0.0001])


CONFIGS = {"FixupResNet50": FixupResNet50Config}


def get_config(model_name: str):
    cls = CONFIGS.get(model_name)
    return cls() if cls is not None else None
