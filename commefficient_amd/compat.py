"""The reference's module-level helper API, for code written against it.

The reference exposes these from ``utils.py`` and ``fed_aggregator.py``
(/root/reference/CommEfficient/utils.py:232-321,
fed_aggregator.py:23-25,464-616); scripts built on the reference call them
directly (e.g. ``get_server_update`` in a custom optimizer loop).  Here they
are thin functions over this package's native ops with the reference's
semantics and return values.  The engine itself does not go through them:
FedModel / ServerState run the same math fused and in place.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Sequence

import numpy as np
import torch

from . import ops
from .ops import CSVec
from .parallel.flat import get_grad_vec, get_param_vec, set_param_vec, trainable_params
from .utils.logging import Logger, TableLogger, Timer, TSVLogger, make_logdir  # noqa: F401
from .utils.schedules import Exp, PiecewiseLinear, steps_per_epoch  # noqa: F401

__all__ = ["_topk", "get_grad", "get_grad_vec", "get_param_vec", "set_param_vec", "zero_grad",
           "clip_grad", "steps_per_epoch", "sm2np", "args2sketch", "get_server_update",
           "split_results", "shms", "PiecewiseLinear", "Exp", "Timer", "TableLogger",
           "TSVLogger", "Logger", "make_logdir"]


def _topk(vec: torch.Tensor, k: int) -> torch.Tensor:
    """Dense vector keeping the k largest-magnitude entries (row-wise for a
    2-D input), utils.py:232-252 -- on the deterministic radix-select kernel
    (ties -> lower index)."""
    return ops.topk_dense(vec, int(k))


def get_grad(model, args) -> torch.Tensor:
    """Flat gradient + (weight_decay / num_workers) * weights, utils.py:254-259."""
    g = get_grad_vec(model)
    if args.weight_decay != 0:
        g.add_(get_param_vec(model), alpha=args.weight_decay / args.num_workers)
    return g.to(args.device)


def zero_grad(model) -> None:
    """utils.py:275-279."""
    for p in model.parameters():
        if p.grad is not None:
            p.grad.detach_()
            p.grad.zero_()


def clip_grad(l2_norm_clip: float, record):
    """L2 clipping of a tensor or (through ``l2estimate``) a CSVec,
    utils.py:305-313."""
    if isinstance(record, CSVec):
        l2 = float(record.l2estimate())
    else:
        l2 = float(torch.linalg.vector_norm(record.float()))
    if l2 < l2_norm_clip:
        return record
    return record / abs(l2 / l2_norm_clip)


def sm2np(sm, shape, dtype=ctypes.c_float) -> np.ndarray:
    """A numpy view of a shared-memory buffer (utils.py:299-303)."""
    arr = np.ndarray(shape, dtype=dtype, buffer=sm)
    assert arr.base is sm
    return arr


def args2sketch(args) -> CSVec:
    """CSVec of the run's geometry (fed_aggregator.py:464-467)."""
    return CSVec(d=args.grad_size, c=args.num_cols, r=args.num_rows, device=args.device,
                 numBlocks=args.num_blocks, seed=getattr(args, "sketch_seed", 42),
                 kernel=getattr(args, "encode", "planned"))


def get_server_update(gradient: torch.Tensor, Vvelocity: torch.Tensor, Verror: torch.Tensor,
                      args, lr, participating: Optional[Sequence[int]] = None,
                      client_velocities: Optional[torch.Tensor] = None):
    """(weight update, Vvelocity, Verror) of one server step
    (fed_aggregator.py:469-613); ``w -= update``.  V / E are updated in
    place.  ``participating`` + ``client_velocities`` ([C, d]) enable the
    true_topk local-velocity masking the reference does through globals
    (fed_aggregator.py:528-533)."""
    mode, rho = args.mode, float(args.virtual_momentum)
    G = gradient
    if mode == "fedavg":
        assert args.error_type == "none" and args.local_momentum == 0 and lr == 1
        ops.momentum_ef(Vvelocity, None, G, rho)
        return Vvelocity, Vvelocity, Verror
    if mode == "uncompressed":
        ops.momentum_ef(Vvelocity, None, G, rho)
        grad = Vvelocity
        if args.do_dp and args.dp_mode == "server":
            grad += torch.normal(0.0, args.noise_multiplier, size=grad.size(), device=grad.device)
        return grad * lr, Vvelocity, Verror
    if mode == "local_topk":
        assert args.error_type in ("local", "none")
        ops.momentum_ef(Vvelocity, None, G, rho)
        return Vvelocity * lr, Vvelocity, Verror
    if mode == "true_topk":
        assert args.error_type == "virtual"
        ops.momentum_ef(Vvelocity, Verror, G, rho, 1.0, "virtual")
        idx, vals = ops.topk_abs(Verror, args.k)
        update = ops.scatter_dense(idx, vals, Verror.numel()).view_as(Verror)
        if args.local_momentum > 0 and participating is not None and client_velocities is not None:
            rows = torch.as_tensor(list(participating), device=client_velocities.device).view(-1, 1)
            client_velocities[rows, idx.to(client_velocities.device).view(1, -1)] = 0
        ops.zero_at(idx, Verror, Vvelocity)
        return update * lr, Vvelocity, Verror
    if mode == "sketch":
        if args.error_type == "local":
            assert args.virtual_momentum == 0
        elif args.error_type == "virtual":
            assert args.local_momentum == 0
        et = args.error_type if args.error_type in ("virtual", "local") else "none"
        ops.momentum_ef(Vvelocity.view(-1), Verror.view(-1) if et != "none" else None,
                        G.reshape(-1), rho, 1.0, et)
        sk = args2sketch(args).like(Verror if et != "none" else Vvelocity)
        idx, vals = sk.unsketch_sparse(args.k)
        update = ops.scatter_dense(idx, vals, args.grad_size)
        # error feedback + momentum-factor masking at the recovered coordinates'
        # buckets (= S(update).nonzero() except exact cancellations)
        if et == "virtual":
            sk.zero_heavy_hitters(idx, vals, Vvelocity)
        else:
            args2sketch(args).like(Vvelocity).zero_heavy_hitters(idx, vals)
        return update * lr, Vvelocity, Verror
    raise ValueError(mode)


def split_results(results, n_results: int):
    """fed_aggregator.py:615-616."""
    return [np.array([r[i] for r in results]) for i in range(n_results)]


def shms():
    """/dev/shm segments of this process (fed_aggregator.py:23-25).  The SPMD
    design shares no host memory between ranks, so this is normally empty."""
    pid = str(os.getpid())
    try:
        return [s for s in os.listdir("/dev/shm") if pid in s]
    except FileNotFoundError:
        return []


def num_trainable(model) -> int:
    return sum(p.numel() for p in trainable_params(model))
