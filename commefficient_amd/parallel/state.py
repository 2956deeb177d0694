"""Per-client state (local momentum, local error, stale downlink weights) and
upload/download byte accounting.

Reference: client state lives in host shared memory as ``[C, d]`` arrays
(/root/reference/CommEfficient/fed_aggregator.py:105-129) and, on GPU runs,
worker updates are made on ``.to(device)`` *copies* and lost
(fed_worker.py:169-174).  Here rows are written
back, live in HBM when they fit (288 GB per MI355X) and are allocated lazily
on first participation on the rank that owns the client.  Ownership is
balanced per round (``assign``): every client has a home rank (initially
``client % world``); when a round's clients would load the ranks unevenly,
the surplus clients of the fuller ranks move to the emptier ones -- clients
without state first -- and the moved clients' rows travel with them (one
batched point-to-point exchange), so per-rank work differs by at most one
client, as with the reference's even chunking (fed_aggregator.py:230-237).

Byte accounting reproduces fed_aggregator.py:170-299 exactly in both of the
reference's regimes with one mechanism: a per-coordinate ``last_mod`` round
index (written by the apply kernels) and a per-client ``last_seen`` round;
a participating client downloads ``4 * #{i : last_mod[i] >= last_seen[c]}``
bytes, read off a change histogram the apply kernels maintain (no host
history deque; the reference's 10/participation truncation disappears).  Upload is ``4 * {d | k | r*c}`` per participating client
(fed_aggregator.py:291-298).  The true on-wire RCCL volume is reported too.
"""
from __future__ import annotations

from typing import Dict, Iterable, Optional

import numpy as np
import torch

from .. import ops
from .dist import h2d


class ClientStateStore:
    KINDS = ("velocity", "error", "weights")

    def __init__(self, args, d: int, num_clients: int, device, rank: int, world: int,
                 init_weights: Optional[torch.Tensor] = None):
        self.args = args
        self.d = d
        self.num_clients = num_clients
        self.rank, self.world = rank, world
        self.kinds = []
        if args.local_momentum > 0 and args.mode != "sketch":
            self.kinds.append("velocity")
        if args.error_type == "local":
            self.kinds.append("error")
        if args.do_topk_down:
            self.kinds.append("weights")
        want = getattr(args, "client_state_device", "auto")
        per_rank_bytes = len(self.kinds) * d * 4 * (num_clients // max(1, world) + 1)
        if want == "auto":
            want = "gpu"
            if torch.device(device).type == "cuda":
                free, _ = torch.cuda.mem_get_info(torch.device(device))
                if per_rank_bytes > 0.6 * free:
                    want = "cpu"
        self.store_device = torch.device(device) if want == "gpu" else torch.device("cpu")
        self.compute_device = torch.device(device)
        self.rows: Dict[str, Dict[int, torch.Tensor]] = {k: {} for k in self.kinds}
        self.init_weights = init_weights.detach().clone().to(self.store_device) \
            if (init_weights is not None and "weights" in self.kinds) else None
        # host-tier rows: the round's next clients are copied ahead on a side
        # stream (``begin_round``), so a client's H2D copy overlaps the previous
        # clients' compute instead of sitting in front of its own
        self.prefetch_depth = int(getattr(args, "client_prefetch", 4))
        self._order: list = []
        self._next = 0
        self._staged: Dict[tuple, tuple] = {}
        self._copy_stream = None
        # replicated on every rank (identical updates): home rank of every client
        # that was ever assigned, and the clients that hold rows
        self.home: Dict[int, int] = {}
        self.seen: set = set()
        self.migrated = 0  # rows moved between ranks so far (diagnostics)

    @property
    def host_tier(self) -> bool:
        return self.store_device.type == "cpu" and self.compute_device.type == "cuda"

    def begin_round(self, clients: Iterable[int]):
        """The order in which this rank will ``get`` the round's clients:
        starts the first ``prefetch_depth`` host -> device copies."""
        self._staged.clear()
        self._order = [int(c) for c in clients]
        self._next = 0
        if self.host_tier and self.prefetch_depth > 0:
            self._advance()

    def _advance(self):
        if self._copy_stream is None:
            self._copy_stream = torch.cuda.Stream(self.compute_device)
        cur = torch.cuda.current_stream(self.compute_device)
        while self._next < len(self._order) and \
                len({c for (_, c) in self._staged}) < self.prefetch_depth:
            c = self._order[self._next]
            self._next += 1
            for kind in self.kinds:
                row = self.rows[kind].get(c)
                if row is None:
                    continue  # first participation: created on the device side by get()
                # (the row's previous write-back, on the compute stream, lands first)
                self._copy_stream.wait_stream(cur)
                with torch.cuda.stream(self._copy_stream):
                    # allocated on the copy stream: a staged copy dropped before
                    # get() (begin_round's clear) returns its block to THIS
                    # stream's pool, ordered behind the copy still writing it
                    dev = torch.empty(self.d, device=self.compute_device)
                    dev.copy_(row, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self._copy_stream)
                self._staged[(kind, c)] = (dev, ev)

    @property
    def active(self) -> bool:
        return bool(self.kinds)

    def owner(self, client: int) -> int:
        c = int(client)
        return self.home.get(c, c % self.world)

    def assign(self, clients) -> np.ndarray:
        """This rank's share of the round's ``clients`` (sorted unique,
        identical on every rank).  Per-rank counts differ by at most one.  A
        collective when rows have to move: every rank calls it once per round."""
        clients = np.asarray(clients, dtype=np.int64)
        N, R = self.world, self.rank
        if N == 1:
            self.seen.update(int(c) for c in clients)
            return clients
        W = len(clients)
        target = [(r + 1) * W // N - r * W // N for r in range(N)]  # = the stateless split
        by_rank = [[] for _ in range(N)]
        for c in clients:
            by_rank[self.owner(c)].append(int(c))
        surplus = []
        for r in range(N):
            extra = len(by_rank[r]) - target[r]
            if extra > 0:
                # release clients without state first (nothing to move), then the
                # highest ids; deterministic on every rank
                cand = sorted(by_rank[r], key=lambda c: (c in self.seen, -c))
                out = cand[:extra]
                by_rank[r] = [c for c in by_rank[r] if c not in set(out)]
                surplus += [(c, r) for c in out]
        moves = []  # (client, src, dst) of clients that hold rows
        si = 0
        for r in range(N):
            while len(by_rank[r]) < target[r]:
                c, src = surplus[si]
                si += 1
                by_rank[r].append(c)
                self.home[c] = r
                if c in self.seen:
                    moves.append((c, src, r))
        for r in range(N):
            for c in by_rank[r]:
                self.home.setdefault(c, r)
        if moves:
            self._migrate(moves)
        self.seen.update(int(c) for c in clients)
        return np.array(sorted(by_rank[R]), dtype=np.int64)

    def _migrate(self, moves):
        """Send the rows of the moved clients from their old to their new home
        (one batched isend / irecv exchange; RCCL needs device buffers)."""
        import torch.distributed as tdist
        from . import dist as _dist
        ctx = _dist.ctx()
        dev = self.compute_device if ctx.backend == "nccl" else torch.device("cpu")
        if self.host_tier:
            # a host-tier row's last write-back (``put``) is a non_blocking D2H copy on
            # the compute stream; over gloo ``row.to(cpu)`` is the pinned row itself, so
            # the send could ship it before that copy lands
            torch.cuda.current_stream(self.compute_device).synchronize()
        p2p, recv = [], []
        for (c, src, dst) in moves:
            for kind in self.kinds:
                if self.rank == src:
                    row = self.rows[kind].pop(c, None)
                    if row is None:  # (seen but never materialised: zeros)
                        row = self.init_weights if kind == "weights" else torch.zeros(self.d)
                    buf = row.to(dev)
                    p2p.append(tdist.P2POp(tdist.isend, buf.contiguous(), dst))
                elif self.rank == dst:
                    buf = torch.empty(self.d, device=dev)
                    p2p.append(tdist.P2POp(tdist.irecv, buf, src))
                    recv.append((kind, c, buf))
        self.migrated += len(moves)
        if not p2p:
            return
        for req in tdist.batch_isend_irecv(p2p):
            req.wait()
        for kind, c, buf in recv:
            pin = self.store_device.type == "cpu" and self.compute_device.type == "cuda"
            row = torch.empty(self.d, device=self.store_device, pin_memory=pin)
            row.copy_(buf)
            self.rows[kind][c] = row

    def get(self, kind: str, client: int) -> Optional[torch.Tensor]:
        """Device tensor for the row (created on first use).  For CPU-resident
        storage the returned tensor is a device copy; call ``put`` after
        mutating it."""
        if kind not in self.kinds:
            return None
        rows = self.rows[kind]
        c = int(client)
        if c not in rows:
            if kind == "weights":
                rows[c] = self.init_weights.clone()
            else:
                rows[c] = torch.zeros(self.d, device=self.store_device,
                                      pin_memory=self.store_device.type == "cpu" and
                                      self.compute_device.type == "cuda")
        t = rows[c]
        if t.device != self.compute_device:
            hit = self._staged.pop((kind, c), None)
            if hit is not None:
                dev, ev = hit
                torch.cuda.current_stream(self.compute_device).wait_event(ev)
                # the compute stream uses a copy-stream block from here on
                dev.record_stream(torch.cuda.current_stream(self.compute_device))
                if self.host_tier:
                    self._advance()
                return dev
            out = t.to(self.compute_device, non_blocking=True)
            if self.host_tier and self._order:
                self._advance()
            return out
        return t

    def put(self, kind: str, client: int, value: torch.Tensor):
        if kind not in self.kinds:
            return
        row = self.rows[kind][int(client)]
        if row.data_ptr() != value.data_ptr():
            row.copy_(value, non_blocking=True)

    def zero_velocity_at(self, clients: Iterable[int], idx: torch.Tensor):
        """true_topk momentum masking of the participating clients' local
        velocities (fed_aggregator.py:528-533)."""
        if "velocity" not in self.kinds:
            return
        for c in clients:
            c = int(c)
            if self.owner(c) != self.rank or c not in self.rows["velocity"]:
                continue
            row = self.rows["velocity"][c]
            if row.device == idx.device:
                ops.zero_at(idx, row)
            else:
                row[idx.to(row.device)] = 0

    def state_dict(self):
        """Every rank's rows (a collective on > 1 rank: the rows live on their
        owners; rank 0 receives the union, the other ranks None)."""
        from . import dist as _dist
        own = {k: {c: t.cpu() for c, t in v.items()} for k, v in self.rows.items()}
        if self.world == 1:
            return own
        parts = _dist.gather_objects(own)
        if parts is None:
            return None
        out = {k: {} for k in self.rows}
        for p in parts:
            for k, v in p.items():
                out.setdefault(k, {}).update(v)
        return out

    def load_state_dict(self, sd):
        """Keep the rows this rank owns (home ``client % world`` after a resume:
        any world size can resume any checkpoint)."""
        self.home = {}
        self.seen = set()
        for k, v in sd.items():
            if k in self.rows:
                self.seen.update(int(c) for c in v)
                self.rows[k] = {int(c): t.to(self.store_device) for c, t in v.items()
                                if self.owner(int(c)) == self.rank}


class ByteAccountant:
    """Upload / download byte accounting (fed_aggregator.py:170-299).

    Download: every apply kernel stamps ``last_mod[i] = round`` where a weight
    changes and moves the coordinate between the bins of a change histogram
    ``hist[r + 1] = #{i : last_mod[i] == r}`` (bin 0: never changed).  A
    client that last synchronised at round s downloads
    ``4 * #{i : last_mod[i] >= s}`` = 4 * (sum of bins >= s + 1), so a round's
    accounting is one tiny kernel over the bins (``account_hist``) instead of
    a pass over all d stamps."""

    HIST_CAP = 1 << 16  # rounds before the histogram grows

    def __init__(self, args, d: int, num_clients: int, device, world: int, payload_numel: int):
        self.args = args
        self.d = d
        self.num_clients = num_clients
        self.device = device
        self.world = world
        self.last_mod = torch.full((d,), -1, dtype=torch.int32, device=device)
        self.hist = torch.zeros(self.HIST_CAP, dtype=torch.int32, device=device)
        self.hist[0] = d
        self.last_seen = np.zeros(num_clients, dtype=np.int64)
        mode = args.mode
        self.upload_per_client = 4 * {"uncompressed": d, "true_topk": d, "local_topk": args.k,
                                      "sketch": args.num_rows * args.num_cols, "fedavg": d}[mode]
        self.payload_numel = payload_numel
        # on-device running totals (no host sync per round)
        self.client_download = torch.zeros(num_clients, dtype=torch.float64, device=device)
        self.client_upload = torch.zeros(num_clients, dtype=torch.float64, device=device)

    def hist_for(self, round_idx: int) -> torch.Tensor:
        """The change histogram, grown (doubling) so that round ``round_idx``
        has a bin."""
        if round_idx + 2 > self.hist.numel():
            cap = self.hist.numel()
            while round_idx + 2 > cap:
                cap *= 2
            h = torch.zeros(cap, dtype=torch.int32, device=self.device)
            h[:self.hist.numel()].copy_(self.hist)
            self.hist = h
        return self.hist

    def wire_bytes_per_rank(self, payload_numel: int) -> float:
        """Bytes each rank sends in a ring all-reduce of the payload."""
        n = self.world
        return 0.0 if n == 1 else 2.0 * (n - 1) / n * payload_numel * 4

    def round_meta(self, clients: np.ndarray) -> np.ndarray:
        """Host int64 [last_seen (W) | clients (W)] for ``round``."""
        return np.concatenate([self.last_seen[clients], clients]).astype(np.int64)

    def round(self, clients: np.ndarray, round_idx: int, meta: Optional[torch.Tensor] = None):
        """Account one round for the participating ``clients`` (unique, sorted).
        Must be called before the round's server update (clients download the
        pre-update weights).  ``meta``: ``round_meta(clients)`` already on the
        device.  Returns (download bytes [W] device f64, upload bytes float)."""
        W = len(clients)
        if meta is None:
            meta = h2d(self.round_meta(clients), self.device)
        # bins above the current round are empty: scan only [0, round + 1]
        nb = min(self.hist.numel(), round_idx + 2)
        dl = ops.account_hist(self.hist[:nb], meta, W, self.client_download, self.client_upload,
                              float(self.upload_per_client))
        self.last_seen[clients] = round_idx
        return dl, float(self.upload_per_client) * W

    def state_dict(self):
        return {"last_mod": self.last_mod.cpu(), "last_seen": torch.from_numpy(self.last_seen),
                "client_download": self.client_download.cpu(),
                "client_upload": self.client_upload.cpu()}

    def load_state_dict(self, sd):
        self.last_mod.copy_(sd["last_mod"])
        self.last_seen = sd["last_seen"].numpy().astype(np.int64)
        if "client_download" in sd:
            self.client_download.copy_(sd["client_download"])
            self.client_upload.copy_(sd["client_upload"])
        top = int(self.last_mod.max().item()) if self.d else -1
        cap = self.HIST_CAP
        while top + 2 > cap:
            cap *= 2
        counts = torch.bincount((self.last_mod.long() + 1), minlength=cap)
        self.hist = counts.to(torch.int32).to(self.device)
