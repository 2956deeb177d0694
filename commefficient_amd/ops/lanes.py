"""A side lane for work nothing downstream waits for (the convolutions'
weight gradients), overlapping the main chain of the backward.

In ResNet-9's backward each layer runs dgrad (-> the next layer's input
gradient, on the critical path) and wgrad + its split-K reduction (-> the flat
gradient, read only by the encode after the whole backward).  On one stream
they alternate: each kernel's tail of idle CUs and the small reduction
kernels sit on the critical path.  ``fork(*inputs)`` runs the enclosed
launches on a side stream after everything issued so far on the main stream
(the inputs are kept alive until the join), ``join()`` orders the main stream after
the side stream before the gradient is read (parallel/fed_model.py, after
the backward).

Users: the conv / 1x1 / column-image weight gradients of ops/nn.py, the
GPT-2 weight-gradient GEMMs and column sums of ops/transformer.py, and the
native FedAvg engines' fused weight updates (parallel/fedavg_native.py: each
local step joins before its first block reads the updated rows, so the next
step's stem runs beside the lane's last updates).

Eager rounds use PyTorch stream waits; recorded rounds (parallel/tape.py)
also append the fork / join to the launch tape (csrc/tape.cpp), which
replays the lane-1 launches on the side stream between event waits.  The
lane is off (a no-op) on CPU, under ``set_enabled(False)`` (per-parameter
gradient hooks that read gradients during the backward, the
``--wgrad_stream off`` flag) and when ``COMMEFF_CONV_LANE=0``.
"""
from __future__ import annotations

import contextlib
import os

import torch

from .._ext import ops as _ops

_STATE = {"enabled": os.environ.get("COMMEFF_CONV_LANE", "1") != "0", "stream": None, "pending": None,
          "held": []}
_ENV_ON = _STATE["enabled"]


def set_enabled(on: bool) -> None:
    _STATE["enabled"] = bool(on) and _ENV_ON


def enabled() -> bool:
    return _STATE["enabled"]


def side_stream(device) -> "torch.cuda.Stream":
    s = _STATE["stream"]
    if s is None or s.device != torch.device(device):
        s = _STATE["stream"] = torch.cuda.Stream(device=device)
    return s


@contextlib.contextmanager
def fork(*inputs: torch.Tensor):
    """Run the body's launches on the side lane (or inline when it is off)."""
    t0 = inputs[0] if inputs else None
    if not (_STATE["enabled"] and t0 is not None and t0.is_cuda):
        yield
        return
    main = torch.cuda.current_stream(t0.device)
    side = side_stream(t0.device)
    if main == side:  # (nested: already on the lane)
        _STATE["held"].extend(inputs)
        yield
        return
    side.wait_stream(main)
    _ops().tape_fork(side.cuda_stream)
    # inputs allocated on the main stream stay referenced until the join (not
    # record_stream: its deferred frees kept the caching allocator growing --
    # 16 -> 388 device allocations per 6 ImageNet rounds); freed after the
    # main stream's wait on the side lane, any reuse is ordered after it
    _STATE["held"].extend(inputs)
    _STATE["pending"] = main
    with torch.cuda.stream(side):
        yield


def join() -> None:
    """Order the stream that forked after the side lane's work."""
    main = _STATE["pending"]
    if main is None:
        return
    _STATE["pending"] = None
    main.wait_stream(_STATE["stream"])
    _ops().tape_join()
    _STATE["held"].clear()


def pending() -> bool:
    return _STATE["pending"] is not None
