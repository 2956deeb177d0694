"""Bucketed gradient all-reduce overlapped with the backward pass (dense modes).

In the merged dense modes (uncompressed, true_topk and single-step FedAvg
without per-client state) a rank's upload is its summed gradient plus a weight
decay term, d floats: 26 MB for ResNet-9, 500 MB for GPT-2.  The reference
reduces it to the parameter server after the whole backward
(/root/reference/CommEfficient/fed_worker.py:136-138, fed_aggregator.py:326-332;
SURVEY.md §5.8).  Here the flat gradient is cut into buckets of contiguous
parameters in backward order; as soon as every parameter of a bucket has its
gradient (a post-accumulate-grad hook), the bucket's RCCL all-reduce is issued
asynchronously and runs on the process group's stream while the backward of
the earlier layers continues.  Native backward kernels that accumulate a
weight gradient straight into the flat buffer hand autograd None, so no
AccumulateGrad node (and no hook) runs for that parameter: they announce the
write instead (``ops.nn._grad_written``, called on the stream that wrote it,
which the all-reduce then waits for), and count as ready the same way.  After
the backward any bucket not yet issued is issued, all are waited for, and the
weight decay term -- identical on every rank -- is added once to the reduced
sum (``sum_r (g_r + c_r w) = sum_r g_r + (sum_r c_r) w``).

Every rank must issue the same collectives in the same order: buckets complete
in backward order, which is the same on every rank for the same model and
batch shapes, and the engine only arms the reducer when every rank computes
at least one client.  Bucket size (``--allreduce_bucket_mb``, default 32):
ring all-reduce over xGMI runs near link rate from a few MB, and a bucket
should be small next to one layer group's backward so the last one to
complete is short.
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as tdist


class OverlapReducer:
    def __init__(self, flat, params, bucket_bytes: int, shadow: bool = False):
        """``params``: the parameters whose AccumulateGrad hook fires -- the
        model's (flat.params) or the bf16 replica's (flat.shadow_params); with
        ``shadow`` the hook also moves the replica's bf16 gradient into the
        fp32 flat buffer."""
        self.flat = flat
        self.shadow = shadow
        n = len(flat.params)
        # buckets of consecutive parameters in REVERSE flat order (backward
        # produces the last layers' gradients first)
        self.bucket_of = [0] * n
        self.buckets: List[List[int]] = []
        cur, cur_bytes = [], 0
        for i in reversed(range(n)):
            cur.append(i)
            cur_bytes += flat.numels[i] * 4
            if cur_bytes >= bucket_bytes:
                self.buckets.append(cur)
                cur, cur_bytes = [], 0
        if cur:
            self.buckets.append(cur)
        self.ranges = []
        for b, idxs in enumerate(self.buckets):
            for i in idxs:
                self.bucket_of[i] = b
            lo = min(flat.offsets[i] for i in idxs)
            hi = max(flat.offsets[i] + flat.numels[i] for i in idxs)
            self.ranges.append((lo, hi))
        self.armed = False
        self.pending = [0] * len(self.buckets)
        self.done_param = [False] * n
        self.works: List[Optional[object]] = [None] * len(self.buckets)
        self.issued_early = 0
        self._handles = []
        self._index = {}
        for i, p in enumerate(params):
            self._handles.append(p.register_post_accumulate_grad_hook(self._hook(i)))
            self._index[id(p)] = i
        # native in-place gradient writes (no hook fires for those)
        from ..ops import nn as _nn
        self._nn = _nn
        _nn.add_grad_ready_listener(self._written)

    def _hook(self, i: int):
        def fn(p):
            if not self.armed or self.done_param[i]:
                return
            if self.shadow:
                f = self.flat
                o, n = f.offsets[i], f.numels[i]
                f.g[o:o + n].add_(p.grad.reshape(-1))
                p.grad = None
            self._ready(i)
        return fn

    def _written(self, p):
        i = self._index.get(id(p))
        if i is None or not self.armed or self.done_param[i] or self.shadow:
            return
        self._ready(i)

    def _ready(self, i: int):
        self.done_param[i] = True
        b = self.bucket_of[i]
        self.pending[b] -= 1
        if self.pending[b] == 0:
            self._issue(b)
            self.issued_early += 1

    def _issue(self, b: int):
        lo, hi = self.ranges[b]
        self.works[b] = tdist.all_reduce(self.flat.g[lo:hi], op=tdist.ReduceOp.SUM, async_op=True)

    def arm(self):
        """Before the backward whose gradients complete the round."""
        self.armed = True
        self.pending = [len(ix) for ix in self.buckets]
        self.done_param = [False] * len(self.done_param)
        self.works = [None] * len(self.buckets)
        self.issued_early = 0

    def finish(self):
        """After that backward: move any replica gradients not seen by a hook,
        issue the remaining buckets in index order, wait for all."""
        self.armed = False
        if self.shadow:
            f = self.flat
            for i, p in enumerate(f.shadow_params):
                if not self.done_param[i] and p.grad is not None:
                    o, n = f.offsets[i], f.numels[i]
                    f.g[o:o + n].add_(p.grad.reshape(-1))
                    p.grad = None
        for b in range(len(self.buckets)):
            if self.works[b] is None:
                self._issue(b)
        for w in self.works:
            w.wait()
        return self.issued_early

    def remove(self):
        for h in self._handles:
            h.remove()
        self._handles = []
        self._nn.remove_grad_ready_listener(self._written)
