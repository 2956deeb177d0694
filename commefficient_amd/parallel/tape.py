"""Launch tapes: a federated round replayed from C++ (csrc/launch.h, tape.cpp).

The reference enqueues every round op by op from Python in each worker and
in the parameter server (/root/reference/CommEfficient/fed_worker.py:26-138,
fed_aggregator.py:429-613).  Here, too, the eager round is Python driving
~45 native kernels through autograd, the torch dispatcher and the engine's
bookkeeping: ~1.0-1.4 ms of host time per ResNet-9 round against ~1.65 ms of
GPU time.  That is too close: after every host sync (the bench's timed
region starts with one) the GPU waits for the host for the first ~15 rounds
until the enqueue lead has built up again (``bench.py --round-times``: 1.83 ->
1.64 ms over rounds 2..15).

A round of fixed geometry is therefore recorded ONCE and replayed:

* recording runs the round's Python body under a PyTorch graph capture (so
  nothing executes and every intermediate tensor comes from a private memory
  pool that stays reserved: the recorded device addresses remain valid) while
  ``COMMEFF_LAUNCH`` appends each native kernel launch -- kernel, grid, block,
  LDS bytes and a by-value copy of its arguments -- to a C++ launch tape;
* collectives (``dist.all_reduce_`` / ``dist.all_gather_rows``) split the
  recording into segments: tape, collective, tape, ...; a replay re-issues
  the tapes from C++ and runs the collectives eagerly on the same buffers;
* completeness check: the captured HIP graph must hold exactly as many
  kernel + memset nodes as the tapes and nothing else, in a single chain of
  dependencies -- a launch that bypassed the tape (a PyTorch kernel, a copy)
  or work forked onto a second stream (a replay issues no cross-stream
  waits) makes the geometry fall back to the eager path for good (with a
  one-line warning naming the counts) -- except the side lane's recorded
  forks / joins (ops/lanes.py), which the tape replays with event waits.

The HIP graph itself is never launched (ROCm 7.2's graph packet capture
faulted on the second replay of this round in round 1 and was throughput-
neutral without it); it only provides the capture semantics and the memory
pool.  Per-round scalars (learning rate, round index) reach the recorded
kernels through a device ``step`` buffer; per-round inputs through static
device buffers filled by stream-ordered H2D copies before each replay.
"""
from __future__ import annotations

import gc
import warnings
from typing import Callable, List, Optional

import torch

from .._ext import ops as _ops
from ..ops import lanes as _lanes

_REC: Optional["_Recording"] = None


class _Recording:
    def __init__(self):
        self.segments: List = []  # ("tape", id) | ("call", fn)
        _ops().tape_begin()

    def cut(self, fn: Callable[[], None]):
        """End the current tape, add an eager step (a collective), open the next tape."""
        _lanes.join()  # (a tape's side-lane work ends inside it)
        self.segments.append(("tape", _ops().tape_end()))
        self.segments.append(("call", fn))
        _ops().tape_begin()

    def close(self):
        _lanes.join()
        self.segments.append(("tape", _ops().tape_end()))


def recording() -> bool:
    return _REC is not None


def eager_step(fn: Callable[[], None]) -> bool:
    """Called by the collective wrappers (parallel/dist.py): while a round is
    recorded, ``fn`` becomes an eager step of the replay (and is not run now:
    nothing executes under capture).  Returns True when it was deferred."""
    if _REC is None:
        return False
    _REC.cut(fn)
    return True


class Replay:
    """One recorded part of a round: its segments, the capture that owns
    the memory pool, and the result its Python body returned."""

    def __init__(self, segments, graph, result):
        self.segments = segments
        self.graph = graph
        self.result = result
        self.valid = True
        self.side = 0  # the side lane's stream handle (tapes with forks)

    def run(self, call_ctx=None):
        for kind, x in self.segments:
            if kind == "tape":
                _ops().tape_replay(x, self.side)
            elif call_ctx is not None:
                with call_ctx():
                    x()
            else:
                x()

    def free(self):
        for kind, x in self.segments:
            if kind == "tape":
                _ops().tape_free(x)
        self.segments = []
        self.graph = None
        self.valid = False


class RoundTapes:
    """Recorder / replayer of one engine's rounds (parallel/fed_model.py)."""

    def __init__(self, device):
        self.device = torch.device(device)
        self.stream = torch.cuda.Stream(self.device)
        self.pool = None
        self.failed = set()
        self.replays = 0
        self.last_counts = None
        self._live: List[Replay] = []
        # context around the eager steps (collectives) of a replay, e.g. a phase timer
        self.call_ctx = None

    def record(self, key, body: Callable[[], object]) -> Optional[Replay]:
        """Record ``body`` (nothing executes).  None when the tape would be
        incomplete (the geometry ``key`` then stays eager)."""
        global _REC
        if key in self.failed:
            return None
        self._live = [r for r in self._live if r.valid]
        if not self._live:
            # every graph of the shared pool was freed: PyTorch released the
            # pool with the last one, so the next capture starts a new pool
            self.pool = None
        cur = torch.cuda.current_stream(self.device)
        cur.synchronize()
        self.stream.wait_stream(cur)
        try:
            g = torch.cuda.CUDAGraph(keep_graph=True)
        except TypeError:  # older torch: no keep_graph
            g = torch.cuda.CUDAGraph()
        rec = None
        result = None
        # no garbage collection inside the capture: a collected object whose
        # finaliser calls the runtime (an unreachable engine's graphs, events
        # or side-stream tensor frees) aborts a capturing process -- so the
        # collector is held off until the capture ends (a full gc.collect()
        # first, as torch.cuda.graph does, cost 30-80 ms of GPU idle in the
        # recording rounds with torch's heap and gains nothing once the
        # collector cannot run inside the capture)
        gc_was = gc.isenabled()
        gc.disable()
        try:
            with torch.cuda.stream(self.stream):
                if self.pool is None:
                    g.capture_begin()
                else:
                    g.capture_begin(pool=self.pool)
                try:
                    rec = _REC = _Recording()
                    result = body()
                finally:
                    _REC = None
                    if rec is not None:
                        rec.close()
                    g.capture_end()
        finally:
            if gc_was:
                gc.enable()
        cur.wait_stream(self.stream)
        self.pool = g.pool()
        counts = [int(c) for c in _ops().graph_node_counts(g.raw_cuda_graph())]
        self.last_counts = counts
        n_tape = sum(int(_ops().tape_size(x)) for kind, x in rec.segments if kind == "tape")
        rep = Replay(rec.segments, g, result)
        self._live.append(rep)
        forks = sum(int(_ops().tape_forks(x)) for kind, x in rec.segments if kind == "tape")
        if forks:
            # replayed as recorded: lane-1 launches on the side lane's stream,
            # between event waits at the recorded forks / joins
            rep.side = _lanes.side_stream(self.device).cuda_stream
        chain = forks > 0 or len(counts) < 7 or (counts[4] <= 1 and counts[5] <= 1 and counts[6] <= 1)
        if counts[1] or counts[3] or counts[0] + counts[2] != n_tape or not chain:
            warnings.warn(f"launch tape for {key!r} incomplete (graph nodes: {counts[0]} kernels, "
                          f"{counts[1]} copies, {counts[2]} memsets, {counts[3]} other; tape: "
                          f"{n_tape} launches; roots / max deps / max dependents: "
                          f"{counts[4:7]}): this round "
                          f"geometry stays eager")
            rep.free()
            self.failed.add(key)
            return None
        return rep

    def replay(self, rep: Replay):
        rep.run(self.call_ctx)
        self.replays += 1
