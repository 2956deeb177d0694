"""Grouped (per-client) weight gradients of ONE merged forward/backward.

The reference computes every client's gradient in its own forward/backward
(/root/reference/CommEfficient/fed_worker.py:60-131, 249-335): for modes whose
client-side processing is nonlinear (local top-k, local momentum / error,
per-client clipping, worker-side DP) the per-client gradients are needed one
by one, so merging clients into one batch is not exact -- unless the backward
produces each client's weight gradient separately.  When every client of the
round computes at the same weights (everything but multi-step FedAvg and top-k
downlink), the forward activations and the input gradients of a concatenated
batch are exactly the per-client ones (per-client BatchNorm statistics via
ghost batch norm); only the weight-gradient reductions must stop at client
boundaries.  With ``grouped_grads(gg)`` active, the native layers
(``NativeConv2d``, ``NativeLinear``, ``GhostBatchNorm2d``) write the weight
gradient of each of the G equal-size example groups into row g of a
client-major ``[G, d]`` fp32 buffer (288 GB of HBM holds it: 8 ResNet-101
clients are 1.4 GB) instead of into the shared flat ``.grad``:

  * 1x1 convolutions / linear layers: one batched GEMM over the G groups
    (bf16 in, fp32 out), split along each group's rows when K x C is small;
  * 3x3 convolutions: the native wgrad kernel on each group's slice,
    accumulating into that group's row;
  * ghost batch norm: the backward finalize kernel writes the per-group
    dweight / dbias it already computes (csrc/bn.hip);
  * other convolutions (7x7 stems, strided 3x3): MIOpen weight gradients of
    each group's slice.

One kernel chain per layer instead of G, and full-batch GEMM shapes instead of
G small ones (parallel/fed_model.py ``_compute_grouped``).
"""
from __future__ import annotations

import contextlib
from typing import Dict, Optional, Tuple

import torch

_ACTIVE = [None]


class GroupedGrads:
    """``buf`` [G, d] fp32 (client-major); ``index`` maps id(param) to its
    (flat offset, shape)."""

    def __init__(self, G: int, buf: torch.Tensor, index: Dict[int, Tuple[int, torch.Size]]):
        assert buf.dim() == 2 and buf.shape[0] == G and buf.dtype == torch.float32
        self.G = G
        self.buf = buf
        self.index = index

    def view(self, p: torch.Tensor) -> Optional[torch.Tensor]:
        """[G, *p.shape] view of the group rows of ``p`` (row stride d)."""
        ent = self.index.get(id(p))
        if ent is None:
            return None
        off, shape = ent
        n = 1
        for s in shape:
            n *= s
        return self.buf[:, off:off + n].view(self.G, *shape) if n else None


def active() -> Optional[GroupedGrads]:
    return _ACTIVE[0]


@contextlib.contextmanager
def grouped_grads(gg: GroupedGrads):
    prev = _ACTIVE[0]
    _ACTIVE[0] = gg
    try:
        yield gg
    finally:
        _ACTIVE[0] = prev


def group_rows(t: torch.Tensor, G: int) -> int:
    n = t.shape[0]
    if n % G:
        raise ValueError(f"grouped gradients need equal groups: batch {n} over {G} groups")
    return n // G
