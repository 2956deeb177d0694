"""LR schedules and epoch arithmetic (/root/reference/CommEfficient/utils.py:26-35,315-321)."""
from __future__ import annotations

import math
from collections import namedtuple

import numpy as np


class PiecewiseLinear(namedtuple("PiecewiseLinear", ("knots", "vals"))):
    def __call__(self, t):
        return float(np.interp([t], self.knots, self.vals)[0])


class Exp(namedtuple("Exp", ("warmup_epochs", "amplitude", "decay_len"))):
    def __call__(self, t):
        if t < self.warmup_epochs:
            return float(np.interp([t], [0, self.warmup_epochs], [0, self.amplitude])[0])
        return self.amplitude * 10 ** (-(t - self.warmup_epochs) / self.decay_len)


def steps_per_epoch(local_batch_size: int, dataset, num_workers: int) -> float:
    if local_batch_size == -1:
        return dataset.num_clients // num_workers
    batch_size = local_batch_size * num_workers
    return math.ceil(len(dataset) / batch_size)


def triangular_lambda(args, spe):
    """cv_train's schedule: 0 -> lr_scale at pivot_epoch -> 0 at num_epochs
    (/root/reference/CommEfficient/cv_train.py:394-404)."""
    sched = PiecewiseLinear([0, args.pivot_epoch, args.num_epochs], [0, args.lr_scale, 0])
    return lambda step: sched(step / spe)


def linear_decay_lambda(args, spe):
    """gpt2_train's schedule: lr_scale linearly to 0 over num_epochs*spe steps
    (/root/reference/CommEfficient/gpt2_train.py:302-307)."""
    sched = PiecewiseLinear([0, args.num_epochs * spe], [args.lr_scale, 0.0])
    return lambda step: sched(step)
