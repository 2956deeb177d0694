"""Logging / timing utilities.

Equivalents of the reference's Logger, TableLogger, TSVLogger, Timer, union
and make_logdir (/root/reference/CommEfficient/utils.py:14-99) with the
``np.float`` bug fixed, plus a TensorBoard-free
scalar writer (tensorboard is not installed in this image; events go to a
JSONL file with the same tag names) and HIP-event phase timers.
"""
from __future__ import annotations

import json
import os
import time
from datetime import datetime
from typing import Dict, Optional

import numpy as np


class Logger:
    def _p(self, msg, args=None):
        print(msg.format(args) if args is not None else msg)

    debug = info = warn = error = critical = _p


class TableLogger:
    def append(self, output: Dict):
        if not hasattr(self, "keys"):
            self.keys = list(output.keys())
            print(*("{:>12s}".format(k) for k in self.keys))
        filtered = [output[k] for k in self.keys]
        print(*("{:12.4f}".format(v) if isinstance(v, (float, np.floating)) else "{:12}".format(v)
                for v in filtered))


class TSVLogger:
    def __init__(self):
        self.log = ["epoch,hours,top1Accuracy"]

    def append(self, output):
        epoch = output["epoch"]
        hours = output["total_time"] / 3600
        acc = output["test_acc"] * 100
        self.log.append("{},{:.8f},{:.2f}".format(epoch, hours, acc))

    def __str__(self):
        return "\n".join(self.log)


def union(*dicts):
    return {k: v for d in dicts for (k, v) in d.items()}


class Timer:
    def __init__(self):
        self.times = [time.time()]
        self.total_time = 0.0

    def __call__(self, include_in_total=True):
        self.times.append(time.time())
        delta_t = self.times[-1] - self.times[-2]
        if include_in_total:
            self.total_time += delta_t
        return delta_t


def make_logdir(args) -> str:
    rows, cols, k, mode = args.num_rows, args.num_cols, args.k, args.mode
    sketch_str = f"{mode}: {rows} x {cols}" if mode == "sketch" else f"{mode}"
    k_str = f"k: {k}" if mode in ["sketch", "true_topk", "local_topk"] else ""
    clients_str = f"{args.num_workers}/{args.num_clients}"
    current_time = datetime.now().strftime("%b%d_%H-%M-%S")
    return os.path.join("runs", current_time + "_" + clients_str + "_" + sketch_str + "_" + k_str)


class ScalarWriter:
    """Minimal SummaryWriter stand-in: ``add_scalar(tag, value, step)`` -> JSONL.

    Uses torch.utils.tensorboard when importable, else writes
    ``<log_dir>/scalars.jsonl``."""

    def __init__(self, log_dir: str):
        self.log_dir = log_dir
        self._tb = None
        try:  # pragma: no cover - tensorboard absent in this image
            from torch.utils.tensorboard import SummaryWriter
            self._tb = SummaryWriter(log_dir=log_dir)
        except Exception:
            os.makedirs(log_dir, exist_ok=True)
            self._f = open(os.path.join(log_dir, "scalars.jsonl"), "a")

    def add_scalar(self, tag, value, step):
        if self._tb is not None:
            self._tb.add_scalar(tag, value, step)
        else:
            self._f.write(json.dumps({"tag": tag, "value": float(value), "step": int(step),
                                      "time": time.time()}) + "\n")
            self._f.flush()

    def close(self):
        if self._tb is not None:
            self._tb.close()
        else:
            self._f.close()


class PhaseTimer:
    """Per-phase device timing with HIP events (fwd/bwd, encode, all-reduce,
    decode, apply...).  Events are recorded on the current stream and only
    resolved at ``summary()`` so timing adds no host syncs to the round."""

    def __init__(self, enabled: bool, device):
        import torch
        self.enabled = enabled and torch.device(device).type == "cuda"
        self.only = None  # optional set of phase names to time (others are free)
        self._pending = []
        self.totals: Dict[str, float] = {}
        self.counts: Dict[str, int] = {}

    def phase(self, name: str):
        return _Phase(self, name)

    def enable_only(self, names) -> None:
        """Time just these phases (e.g. the bench's all-reduce): two event
        records per phase and round, no syncs."""
        import torch
        if torch.cuda.is_available():
            self.enabled = True
            self.only = set(names)

    def discard(self) -> None:
        """Drop the recorded (unresolved) events and the totals, without a sync."""
        self._pending.clear()
        self.totals.clear()
        self.counts.clear()

    def summary(self) -> Dict[str, float]:
        import torch
        if not self.enabled:
            return {}
        torch.cuda.synchronize()
        for name, a, b in self._pending:
            self.totals[name] = self.totals.get(name, 0.0) + a.elapsed_time(b)
            self.counts[name] = self.counts.get(name, 0) + 1
        self._pending.clear()
        return {k: self.totals[k] / self.counts[k] for k in self.totals}


class _Phase:
    def __init__(self, timer: PhaseTimer, name: str):
        self.t, self.name = timer, name

    def __enter__(self):
        self.on = self.t.enabled and (self.t.only is None or self.name in self.t.only)
        if self.on:
            import torch
            self.a = torch.cuda.Event(enable_timing=True)
            self.b = torch.cuda.Event(enable_timing=True)
            self.a.record()
        return self

    def __exit__(self, *exc):
        if self.on:
            self.b.record()
            self.t._pending.append((self.name, self.a, self.b))
        return False
