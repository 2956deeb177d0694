"""HIP-graph execution of the merged-client round.

The reference runs every round op by op from Python in each worker process
(/root/reference/CommEfficient/fed_worker.py:140-335 and the server step
fed_aggregator.py:429-613).  With ~90 kernels per ResNet-9 FetchSGD round the
host needs ~2 ms to enqueue what the GPU executes in ~2.8 ms, so the GPU idles
between launches and any kernel speed-up is capped by Python.  Here a round
of fixed geometry (examples on this rank, clients per round, global batch)
is captured ONCE into two HIP graphs and afterwards replayed:

  compute graph   zero grads -> augment/gather -> bf16 fwd/bwd -> per-client
                  metric sums -> Count-Sketch encode (or dense transmit)
                  -> payload (static buffer)
  [eager]         RCCL all-reduce of the payload; download accounting
  server graph    momentum / error (G / B folded in) -> unsketch (query + top-k) ->
                  heavy-hitter zeroing -> sparse apply + change stamps

Per-round data reaches the graphs through static device buffers filled by
stream-ordered H2D copies from the pinned ring: the round's (row, key)
pairs, per-example client slots and client sizes, and ``step`` = (lr bits,
round index) which the apply kernels read on the device.  The augmentation
seed is folded into the keys (data/device_loader.py ``gather_device``), so
replays are bit-identical to the eager path.

ROCm note: with ROCclr's graph packet capture (AQL packets pre-built at
instantiation, the default in ROCm 7.2) the SECOND launch of the compute
graph at the ResNet-9 bench geometry raises a memory-access fault, although
the first launch is bitwise identical to the eager round
(scripts/dev/graph_cmp.py); with DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 (set by
``commefficient_amd.request_graph_replay()`` when ``--graph`` is requested,
before HIP initialises) every replay is correct.  Graphs are therefore only
used when that variable is 0.

Status of that fault (round 2): not reproduced on purpose -- a faulting
kernel can reset every GPU of a shared host -- so its cause is open.  What is
known: the first replay is bitwise identical to eager (so the captured
arguments and buffers are right at capture time), every replay is correct
with the capture off, and none of this package's kernels uses device-side
assert / printf (no hostcall buffer).  The two packet-capture-specific
candidates are (a) PyTorch kernels compiled with device asserts
(``CUDA_KERNEL_ASSERT`` in its indexing kernels, which the round's gather /
index ops launch) whose hidden hostcall argument is baked into the pre-built
packet, and (b) the >256-byte by-value kernel arguments of the sketch and
conv kernels (``RowHashes`` is 512 bytes) in the pre-built kernarg segment.
Graph replay therefore stays opt-in (``--graph on``), and only then is
DEBUG_CLR_GRAPH_PACKET_CAPTURE set (before HIP initialises).

Measured (1x MI355X, bench.py, 50 rounds): 176.9k img/s replayed vs 176.5k
eager, host enqueue 2.44 vs 2.39 ms/round -- without packet capture the
runtime dispatches each node much like an eager launch, and the GPU (not
the host) bounds this round, so capture is off by default (``--graph on``).

A geometry is first run eagerly (lazy initialisation: sketch plans, kernel
attributes, library handles), captured the second time it is seen, and
replayed from then on.  Capture is skipped for configurations with
host-side per-round state (per-client paths, BatchNorm, DP, multiple LR
groups, the phase timer).
"""
from __future__ import annotations

import os
import warnings
from typing import Dict, Optional, Tuple

import numpy as np
import torch

from .dist import h2d_into


class _capture:
    """Stream capture into ``graph`` on a dedicated side stream.

    Deliberately not ``torch.cuda.graph``: its ``__enter__`` calls
    ``torch.cuda.empty_cache()``, which also drops the BLAS workspaces and
    returns cached blocks to the driver -- memory an already captured graph
    of this round (the compute graph, when the server graph is captured) may
    still address.  Nothing is freed here; allocations during capture go to
    the shared private pool."""

    def __init__(self, graph, pool, stream):
        self.graph, self.pool, self.stream = graph, pool, stream

    def __enter__(self):
        cur = torch.cuda.current_stream()
        cur.synchronize()
        self.stream.wait_stream(cur)
        self._ctx = torch.cuda.stream(self.stream)
        self._ctx.__enter__()
        if self.pool is None:
            self.graph.capture_begin()
        else:
            self.graph.capture_begin(pool=self.pool)
        return self

    def __exit__(self, *exc):
        try:
            self.graph.capture_end()
        finally:
            self._ctx.__exit__(*exc)
            torch.cuda.current_stream().wait_stream(self.stream)
        return False


class _Entry:
    __slots__ = ("count", "idx2", "slots", "n_t", "g_compute", "g_server", "payload_ptr",
                 "n_res", "B")

    def __init__(self):
        self.count = 0
        self.idx2 = self.slots = self.n_t = None
        self.g_compute = None
        self.g_server = None
        self.payload_ptr = None
        self.n_res = None
        self.B = None


class RoundGraphs:
    def __init__(self, fed_model):
        self.fm = fed_model
        a = fed_model.args
        want = str(getattr(a, "graph", "auto")).lower()
        safe = os.environ.get("DEBUG_CLR_GRAPH_PACKET_CAPTURE") == "0"
        if want == "on" and not safe:
            warnings.warn("--graph on ignored: DEBUG_CLR_GRAPH_PACKET_CAPTURE must be 0 before "
                          "HIP initialises (import commefficient_amd first)")
        self.enabled = fed_model.device.type == "cuda" and want in ("on", "auto") and safe
        self.pool = None
        self.entries: Dict[Tuple, _Entry] = {}
        self.step = torch.zeros(2, dtype=torch.int32, device=fed_model.device) \
            if self.enabled else None
        self.pending: Optional[_Entry] = None
        self.replays = 0
        self.stream = torch.cuda.Stream(fed_model.device) if self.enabled else None
        self._hist_ptr = None

    # ---------------------------------------------------------------- policy
    def usable(self, rb, n_local: int) -> bool:
        fm, a = self.fm, self.fm.args
        if not self.enabled or rb.graph_index is None or n_local == 0:
            return False
        if fm.has_bn or fm.timer.enabled:
            return False
        if a.mode not in ("sketch", "uncompressed", "true_topk"):
            return False
        if a.microbatch_size and 0 < a.microbatch_size < n_local:
            return False
        opt = fm.optimizer
        return opt is not None and len(opt.param_groups) == 1

    def key(self, rb, n_local: int, W: int, B: int):
        return (id(getattr(rb.graph_gather, "__self__", rb.graph_gather)), n_local, W, B)

    def seen(self, key) -> bool:
        """Count this geometry; True when it has run eagerly before."""
        e = self.entries.setdefault(key, _Entry())
        e.count += 1
        return e.count >= 2

    def invalidate(self):
        self.entries.clear()
        self.pending = None

    def invalidate_server(self):
        for e in self.entries.values():
            e.g_server = None

    @property
    def hist_ptr(self):
        return self._hist_ptr

    # ------------------------------------------------------------ execution
    def compute(self, key, rb, pos: np.ndarray, slot_per_ex: np.ndarray, counts: np.ndarray,
                W: int, B: int, n_res: int) -> torch.Tensor:
        """Stage this round's inputs and replay (capturing on first use) the
        compute graph.  Returns the payload buffer (transmit + metric sums)."""
        fm = self.fm
        e = self.entries[key]
        n_local = len(pos)
        payload = fm._payload_buf(n_res * W)
        if e.payload_ptr is not None and e.payload_ptr != payload.data_ptr():
            e.g_compute = e.g_server = None  # payload moved: recapture
        if e.idx2 is None:
            dev = fm.device
            e.idx2 = torch.empty(2, n_local, dtype=torch.int64, device=dev)
            e.slots = torch.empty(n_local, dtype=torch.int64, device=dev)
            e.n_t = torch.empty(W, dtype=torch.float32, device=dev)
        h2d_into(e.idx2, rb.graph_index(pos))
        h2d_into(e.slots, slot_per_ex)
        h2d_into(e.n_t, counts.astype(np.float32))
        if e.g_compute is None:
            gather = rb.graph_gather
            g = torch.cuda.CUDAGraph()
            with _capture(g, self.pool, self.stream):
                fm._merged_body(lambda: gather(e.idx2), e.slots, e.n_t, n_local, W, payload,
                                capture=True)
            self.pool = g.pool()
            e.g_compute = g
            e.payload_ptr = payload.data_ptr()
            e.n_res = n_res
            e.B = B
        e.g_compute.replay()
        self.replays += 1
        self.pending = e
        return payload

    def server(self, G: torch.Tensor, lr: float, round_idx: int):
        """Server update of the pending graph round (G unscaled)."""
        fm = self.fm
        e = self.pending
        self.pending = None
        lr_bits = np.array([lr], dtype=np.float32).view(np.int32)[0]
        h2d_into(self.step, np.array([lr_bits, round_idx], dtype=np.int32))
        if e.g_server is None:
            inv_b = 1.0 / e.B
            g = torch.cuda.CUDAGraph()
            with _capture(g, self.pool, self.stream):
                # 1/B folded into the momentum kernel exactly as in the eager
                # step (a separate G *= 1/B rounds differently and can flip a
                # top-k near-tie between the two paths)
                fm.server.update(G, 0.0, fm.w, fm.accountant.last_mod, 0, None, None,
                                 step=self.step, hist=fm.accountant.hist, gscale=inv_b)
            self._hist_ptr = fm.accountant.hist.data_ptr()
            self.pool = g.pool()
            e.g_server = g
        e.g_server.replay()
