"""SPMD process-group plumbing: one process per GPU, RCCL over xGMI.

Replaces the reference's parameter-server topology (PS on the last GPU,
``torch.distributed.reduce`` to rank 0, weights shipped back through host
shared memory -- /root/reference/CommEfficient/fed_aggregator.py:131-164,455,
fed_worker.py:18-25,41,136-138).  Every rank holds the
replicated weights and server state, executes its slice of the round's
virtual clients, joins ONE all-reduce of the compressed payload, and applies
the identical deterministic server update.

Backend: ``nccl`` (= RCCL on ROCm) for GPU runs, ``gloo`` for CPU runs.
Rendezvous: ``env://`` (torchrun, or our own spawner) on 127.0.0.1.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import numpy as np
import torch
import torch.distributed as dist


@dataclass
class DistCtx:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: str = "none"

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    @property
    def distributed(self) -> bool:
        return self.world_size > 1


_CTX = DistCtx()


def ctx() -> DistCtx:
    return _CTX


# RCCL settings for one MI355X node (8 GPUs, each with 7 point-to-point xGMI
# links to the others).  Set only when the user has not set them:
# * TORCH_NCCL_HIGH_PRIORITY=1 -- RCCL kernels on a high-priority HIP stream, so
#   the bucketed gradient all-reduces issued during the backward
#   (parallel/overlap.py) are not queued behind the compute kernels;
# * TORCH_NCCL_AVOID_RECORD_STREAMS=1 -- no record_stream on the payload, whose
#   buffer is reused round after round (no allocator retention).
# Channel counts and algorithm/protocol choices stay with RCCL's own tuning
# tables for the xGMI mesh: no multi-GPU box was available to measure an
# override against them (round 3 forced NCCL_MIN_NCHANNELS=16 and
# RCCL_MSCCL_ENABLE=1 without a measurement; both were dropped).
# HSA_ENABLE_IPC_MODE_LEGACY=0 (dmabuf IPC) must be in the LAUNCHER's
# environment: the HSA runtime reads it once, before this module runs.
# Override any of them from the environment; COMMEFF_RCCL_DEFAULTS=0 sets none.
RCCL_DEFAULTS = {
    "TORCH_NCCL_HIGH_PRIORITY": "1",
    "TORCH_NCCL_AVOID_RECORD_STREAMS": "1",
}


def apply_rccl_defaults(env=None) -> dict:
    """Fill in ``RCCL_DEFAULTS`` (before ``init_process_group``); returns the
    values that were set."""
    env = os.environ if env is None else env
    if env.get("COMMEFF_RCCL_DEFAULTS", "1") == "0":
        return {}
    out = {}
    for k, v in RCCL_DEFAULTS.items():
        if k not in env:
            env[k] = v
            out[k] = v
    return out


def init(device_type: str = "cuda", port: int = None, timeout_s: int = 1800) -> DistCtx:
    """Initialise from the environment (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_*)."""
    global _CTX
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    if device_type == "cuda":
        n = torch.cuda.device_count()
        if n == 0:
            raise RuntimeError("--device cuda requested but no HIP device is visible")
        torch.cuda.set_device(local % n)
        device = torch.device("cuda", local % n)
        # COMMEFF_DIST_BACKEND=gloo: several ranks sharing one GPU (RCCL refuses
        # duplicate devices) -- rehearses the multi-rank GPU path on a 1-GPU box
        backend = os.environ.get("COMMEFF_DIST_BACKEND", "nccl")
    else:
        device = torch.device("cpu")
        backend = "gloo"
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if port is not None:
            os.environ.setdefault("MASTER_PORT", str(port))
        kw = {}
        if backend == "nccl":
            apply_rccl_defaults()
            kw["device_id"] = device
        dist.init_process_group(backend=backend, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=timeout_s), **kw)
    _CTX = DistCtx(rank, world, local, device, backend if world > 1 else "none")
    return _CTX


# stage through the host-read kernel (csrc/hostcopy.hip), not a hipMemcpyAsync
# blit (GPU idle 56 -> 13 us per round, profiles/r4_experiments.md)
_H2D_KERNEL = True


class _PinnedRing:
    """Persistent pinned staging buffers for small per-round H2D copies.

    ``tensor.pin_memory()`` per call goes through the caching host allocator,
    which falls back to a fresh (device-synchronising) pinned allocation
    whenever its cached blocks still have pending copies -- that kept the
    host in lockstep with the GPU every round.  A ring of fixed slots, each
    guarded by an event recorded after its copy, never allocates: by the time
    a slot comes round again its copy has long completed."""

    def __init__(self, slots: int = 32, slot_bytes: int = 1 << 20):
        self.slots = slots
        self.slot_bytes = slot_bytes
        self.bufs = None
        self.events = None
        self.i = 0

    def copy(self, t: torch.Tensor, device) -> torch.Tensor:
        return self.copy_into(t, torch.empty(t.shape, dtype=t.dtype, device=device))

    def copy_into(self, t: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
        nbytes = t.numel() * t.element_size()
        if nbytes > self.slot_bytes:
            out.copy_(t.pin_memory(), non_blocking=True)
            return out
        if self.bufs is None:
            self.bufs = [torch.empty(self.slot_bytes, dtype=torch.uint8, pin_memory=True)
                         for _ in range(self.slots)]
            self.events = [None] * self.slots
        k = self.i
        self.i = (self.i + 1) % self.slots
        if self.events[k] is not None:
            self.events[k].synchronize()
        stage = self.bufs[k][:nbytes].view(t.dtype).view(t.shape)
        stage.copy_(t)
        from . import tape
        if _H2D_KERNEL and out.is_contiguous() and not tape.recording():
            # a kernel of this stream reads the pinned slot (csrc/hostcopy.hip):
            # no runtime blit with its queue drain and cache maintenance.  (Never
            # inside a recorded round: the replay would re-read this slot.)
            from .._ext import ops as _ops
            _ops().host_read_copy(out, stage)
        else:
            out.copy_(stage, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self.events[k] = ev
        return out


_RING = _PinnedRing()


def h2d(x, device, dtype=None) -> torch.Tensor:
    """Host array / CPU tensor -> ``device`` without a stream sync: a pageable
    ``.to(device)`` waits for every kernel queued before it (the GPU then
    idles while the host enqueues the rest of the round), so stage through
    a persistent pinned ring and copy asynchronously on the current stream."""
    t = x if torch.is_tensor(x) else torch.from_numpy(np.ascontiguousarray(x))
    if dtype is not None and t.dtype != dtype:
        t = t.to(dtype)
    device = torch.device(device)
    if device.type != "cuda":
        return t.to(device)
    return _RING.copy(t.contiguous(), device)


def h2d_into(out: torch.Tensor, x) -> torch.Tensor:
    """Stream-ordered copy of a host array into an existing device tensor
    (e.g. a captured HIP graph's static input) through the pinned ring."""
    t = x if torch.is_tensor(x) else torch.from_numpy(np.ascontiguousarray(x))
    t = t.to(out.dtype).reshape(out.shape).contiguous()
    if out.device.type != "cuda":
        out.copy_(t)
        return out
    return _RING.copy_into(t, out)


def _all_reduce_impl(t: torch.Tensor):
    if t.is_cuda and _CTX.backend == "gloo":
        # gloo reads device memory without ordering against the stream
        torch.cuda.current_stream().synchronize()
    dist.all_reduce(t, op=dist.ReduceOp.SUM)


def all_reduce_(t: torch.Tensor) -> torch.Tensor:
    if _CTX.distributed:
        from . import tape
        # a recorded round (parallel/tape.py) defers the SAME backend-aware
        # call to its replay
        if not tape.eager_step(lambda: _all_reduce_impl(t)):
            _all_reduce_impl(t)
    return t


def _reduce_scatter_impl(out: torch.Tensor, t: torch.Tensor):
    if _CTX.backend == "gloo":
        # gloo has no reduce-scatter: all-reduce + slice (same sums)
        if t.is_cuda:
            torch.cuda.current_stream().synchronize()
        full = t.clone()
        dist.all_reduce(full, op=dist.ReduceOp.SUM)
        n = out.numel()
        out.view(-1).copy_(full.view(-1)[_CTX.rank * n:(_CTX.rank + 1) * n])
        return
    dist.reduce_scatter_tensor(out.view(-1), t.view(-1))


def reduce_scatter_(out: torch.Tensor, t: torch.Tensor) -> torch.Tensor:
    """out (this rank's 1/N of t, summed over ranks) = reduce-scatter of the
    contiguous ``t`` (rank r gets elements [r n, (r+1) n), n = out.numel())."""
    if not _CTX.distributed:
        out.copy_(t.view(out.shape))
        return out
    from . import tape
    if not tape.eager_step(lambda: _reduce_scatter_impl(out, t)):
        _reduce_scatter_impl(out, t)
    return out


def _all_gather_impl(out: torch.Tensor, t: torch.Tensor):
    if t.is_cuda and _CTX.backend == "gloo":
        torch.cuda.current_stream().synchronize()
        dist.all_gather(list(out.chunk(_CTX.world_size)), t.contiguous())
        return
    dist.all_gather_into_tensor(out, t.contiguous())


def all_gather_rows(t: torch.Tensor) -> torch.Tensor:
    """[rows, ...] on every rank -> [world * rows, ...] in rank order (one
    RCCL all-gather; every rank passes the same shape)."""
    if not _CTX.distributed:
        return t
    out = torch.empty((_CTX.world_size * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype,
                      device=t.device)
    from . import tape
    if not tape.eager_step(lambda: _all_gather_impl(out, t)):
        _all_gather_impl(out, t)
    return out


def all_reduce_flag(bad: bool) -> bool:
    """True on every rank when ``bad`` is True on any rank (a collective: a
    decision that changes which collectives follow must be the same on all
    ranks)."""
    if not _CTX.distributed:
        return bool(bad)
    t = torch.tensor([1.0 if bad else 0.0],
                     device=_CTX.device if _CTX.backend == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return bool(t.item() > 0)


def gather_objects(obj):
    """Every rank's ``obj`` (a picklable, e.g. dict of CPU tensors), in rank
    order, on rank 0 (None elsewhere).  A collective: every rank calls it."""
    if not _CTX.distributed:
        return [obj]
    out = [None] * _CTX.world_size if _CTX.rank == 0 else None
    dist.gather_object(obj, out, dst=0)
    return out


def broadcast_(t: torch.Tensor, src: int = 0) -> torch.Tensor:
    if _CTX.distributed:
        dist.broadcast(t, src=src)
    return t


def all_gather_object(obj):
    if not _CTX.distributed:
        return [obj]
    out = [None] * _CTX.world_size
    dist.all_gather_object(out, obj)
    return out


def barrier():
    if _CTX.distributed:
        if _CTX.backend == "nccl":
            dist.barrier(device_ids=[_CTX.device.index])
        else:
            dist.barrier()


def max_over_ranks(x: float) -> float:
    if not _CTX.distributed:
        return x
    t = torch.tensor([x], dtype=torch.float64,
                     device=_CTX.device if _CTX.backend == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def replica_checksum(w: torch.Tensor) -> int:
    """Order-sensitive 64-bit checksum of the BIT pattern of a float tensor
    (one device reduction, one host sync)."""
    x = w.detach().reshape(-1)
    if x.dtype != torch.int32:
        x = x.contiguous().view(torch.int32)
    n = x.numel()
    # position weights keep swapped values from cancelling
    pos = torch.arange(n, device=x.device, dtype=torch.int64).mul_(2654435761).remainder_(
        1 << 31).add_(1)
    return int((x.to(torch.int64) * pos).sum().item())


def check_replicas(w: torch.Tensor, what: str = "weights") -> int:
    """Every rank applies the same deterministic update, so the replicated
    weights must be bitwise identical; a drifted rank (a nondeterministic
    kernel, a missed collective) raises here.  Returns the checksum."""
    c = replica_checksum(w)
    if not _CTX.distributed:
        return c
    allc = all_gather_object(c)
    if len(set(allc)) != 1:
        raise RuntimeError(f"replicated {what} drifted across ranks: checksums {allc}")
    return c


def shutdown():
    if dist.is_initialized():
        dist.destroy_process_group()


def spawn(fn, nprocs: int, args=(), port: int = 29500):
    """Launch ``fn(rank, *args)`` on ``nprocs`` fresh processes with env://
    rendezvous on 127.0.0.1 (used when not started by torchrun).  The parent
    must not have touched the GPU (the children are fresh interpreters)."""
    import torch.multiprocessing as mp
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["WORLD_SIZE"] = str(nprocs)
    mp.spawn(_spawn_entry, args=(fn, nprocs, args), nprocs=nprocs, join=True)


def _spawn_entry(rank, fn, nprocs, args):
    os.environ["RANK"] = str(rank)
    os.environ["LOCAL_RANK"] = str(rank)
    os.environ["WORLD_SIZE"] = str(nprocs)
    fn(rank, *args)
