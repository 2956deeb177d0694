"""Region Count-Sketch hash family (``--encode region``, the default).

The coordinates are cut into chunks of ``m = 64`` consecutive coordinates and
each table row into regions of ``m`` buckets, ``g = 32`` regions per group
(``G = c // (g*m)`` groups; the few leftover buckets of a row are unused).
Chunks are dealt to the groups (random balanced order).  Inside its group a
chunk sits in a batch of ``W = 32`` chunks, and in row ``j`` the batch's chunks
take ``W`` distinct regions of the group (a random injection per (row,
batch)).  Coordinate ``o`` of chunk ``q`` goes in row ``j`` to bucket
``region_j(q)*m + (P_j(o) + shift_j(q)) mod m`` with sign
``S_j(o) * sigma_j(q)``, where ``P_j`` is a random permutation of ``[m]`` and
``shift_j``, ``sigma_j`` are random per (row, chunk).

Collisions.  Chunk-mates never collide (a bijection inside the chunk).  Two
coordinates of one group collide in row ``j`` with probability ``~G/c``,
independently across rows; of different groups never: ``~1/c`` per row, like
uniform hashing, every bucket receiving one coordinate from each chunk of its
region.  Because the region a chunk takes is drawn independently per row, a
"hot" chunk (part of a layer with large gradients) meets a different random
``1/g`` of its group in every row and the median filters it
(tests/test_sketch_region.py checks this against the csvec layout).  (A
first version shared one region assignment across all rows so that the
encode would read each chunk once: then a hot chunk pollutes the same
region-mates in every row, and ResNet-9 training stalled -- bench loss after
250 rounds 0.9994 vs 0.0005, profiles/r3_experiments.md.)  The reference's
CSVec also reuses one hash per block with a per-block offset and sign
(numBlocks, /root/reference/CommEfficient/fed_aggregator.py:464-467 builds it).

Why this family on MI355X: a group's ``r x g`` regions (40 KB) fit in LDS, so
the encode is one block per group reading each of its chunks once (one
wavefront per chunk; the batch structure makes a batch's updates
conflict-free, so no atomics) and the query one block per group staging its
regions once and gathering for all its chunks (csrc/sketch_region.hip): no
plan arrays, no ``r*d`` intermediate.  The parameters (a 4-byte word per
(row, chunk), the permutations, the grouped chunk list) are built once from
the seed with numpy, identical on every rank.

The CPU implementation below (dense bucket / sign arrays, ``index_add_``,
``torch.median`` = lower median) defines the same family for CPU runs and is
the reference the GPU kernels are tested against.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from .._ext import ops


def region_geometry(c: int, r: int, m: int = 64, g: int = 32, W: int = 32):
    """(m, g, G, W): chunk / region size m (<= 64: one wavefront per chunk),
    g regions per group (r*g*m floats fit in LDS), G = c // (g*m) groups, W
    chunks per batch (<= g; 16 wavefronts per block, two chunks per wavefront
    at W = 32: one barrier per two chunks)."""
    m = max(1, min(int(m), int(c)))
    g = max(1, min(int(g), int(c) // m, (160 * 1024) // (4 * m * max(1, int(r)))))
    W = max(1, min(int(W), g))
    if 16 < W < 32:
        W = 16
    return m, g, int(c) // (g * m), W


class RegionHash:
    """Parameters of one (d, c, r, seed) region sketch.

    Host arrays (numpy): ``P`` [r, m] permutation, ``S`` [r, m] sign bit,
    ``group`` [nch], ``region`` [r, nch] (global region index), ``shift``
    [r, nch], ``sigma`` [r, nch] sign bit, ``lists`` / ``goffs`` the chunks
    group by group in batch order.  Device tensors (``tensors(device)``):
    perm / cinfo (by chunk) / cinfo_l (in list order) / lists / goffs as the
    kernels read them (csrc/kernels.h)."""

    def __init__(self, d: int, c: int, r: int, seed: int = 42, **geom):
        self.d, self.c, self.r = int(d), int(c), int(r)
        self.m, self.g, self.G, self.W = region_geometry(self.c, self.r, **geom)
        m_, g_, G, W, r_ = self.m, self.g, self.G, self.W, self.r
        self.R = G * g_
        nch = self.nch = -(-self.d // m_)
        rng = np.random.default_rng([int(seed), 0x5E611, self.d, self.c, self.r])
        self.P = np.stack([rng.permutation(m_) for _ in range(r_)]).astype(np.int64)
        self.S = rng.integers(0, 2, size=(r_, m_), dtype=np.int64)
        order = rng.permutation(nch)
        group = np.empty(nch, dtype=np.int64)
        within = np.empty(nch, dtype=np.int64)
        group[order] = np.arange(nch) % G      # dealt evenly
        within[order] = np.arange(nch) // G    # position inside the group's list
        self.group = group
        self.lists = np.concatenate([order[x::G] for x in range(G)]).astype(np.int32)
        self.goffs = np.concatenate([[0], np.cumsum([len(order[x::G]) for x in range(G)])]).astype(np.int32)
        batch, slot = within // W, within % W
        nbatch = int(batch.max()) + 1
        region = np.empty((r_, nch), dtype=np.int64)
        for j in range(r_):
            # per (group, batch): the batch's W chunks take W distinct regions
            inj = np.argsort(rng.random((G, nbatch, g_)), axis=-1)[..., :W]
            region[j] = group * g_ + inj[group, batch, slot]
        self.region = region
        self.shift = rng.integers(0, m_, size=(r_, nch), dtype=np.int64)
        self.sigma = rng.integers(0, 2, size=(r_, nch), dtype=np.int64)
        self._dev = {}
        self._cpu = None

    # ---------------------------------------------------------------- device
    def tensors(self, device) -> dict:
        device = torch.device(device)
        key = str(device)
        if key not in self._dev:
            perm = (self.P | (self.S << 31)).astype(np.uint32).view(np.int32)
            cinfo = (self.region | (self.shift << 24) | (self.sigma << 31)).astype(np.uint32).view(np.int32)
            t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)  # noqa: E731
            self._dev[key] = {"perm": t(perm), "cinfo": t(cinfo), "lists": t(self.lists),
                              "goffs": t(self.goffs),
                              # list order, rows innermost: the encode / query stream it
                              "cinfo_l": t(cinfo[:, self.lists].T)}
        return self._dev[key]

    def chunk_bounds(self, world: int) -> list:
        """Shard boundaries at chunk granularity: shard q = chunks
        [nch*q//world, nch*(q+1)//world)."""
        return [self.nch * q // world for q in range(world + 1)]

    # ------------------------------------------------------------------- CPU
    def dense(self):
        """(bucket [r, d] int64, sign [r, d] f32) of every coordinate."""
        if self._cpu is None:
            i = np.arange(self.d, dtype=np.int64)
            q, o = i // self.m, i % self.m
            b = self.region[:, q] * self.m + (self.P[:, o] + self.shift[:, q]) % self.m
            s = 1.0 - 2.0 * (self.S[:, o] ^ self.sigma[:, q]).astype(np.float32)
            self._cpu = (torch.from_numpy(b), torch.from_numpy(s))
        return self._cpu

    def buckets_of(self, idx: torch.Tensor) -> torch.Tensor:
        """[r, k] buckets of coordinates ``idx`` (host computation)."""
        i = idx.detach().cpu().numpy().astype(np.int64)
        q, o = i // self.m, i % self.m
        b = self.region[:, q] * self.m + (self.P[:, o] + self.shift[:, q]) % self.m
        return torch.from_numpy(b)


def encode(h: RegionHash, table: torch.Tensor, vec: torch.Tensor, scale: float = 1.0,
           wvec: Optional[torch.Tensor] = None, wscale: float = 0.0, overwrite: bool = False,
           zero_vec: bool = False) -> bool:
    """table (+)= S(scale*vec + wscale*wvec).  ``zero_vec``: also clear vec
    (the GPU encode reads every element once and stores a zero behind it --
    no separate fill kernel for the next accumulation); returns whether it did."""
    v = vec.reshape(-1)
    if table.is_cuda:
        t = h.tensors(table.device)
        zero_vec = bool(zero_vec) and v.data_ptr() == vec.data_ptr() and v.is_contiguous()
        ops().cs_region_encode(table, v, float(scale), wvec.reshape(-1) if wvec is not None else None,
                               float(wscale), h.m, h.g, h.W, t["perm"], t["cinfo_l"], t["lists"],
                               t["goffs"], bool(overwrite), zero_vec)
        return zero_vec
    x = v.float() * scale
    if wvec is not None and wscale != 0.0:
        x = x + wscale * wvec.reshape(-1).float()
    b, s = h.dense()
    if overwrite:
        table.zero_()
    tv = table.view(h.r, h.c)
    for j in range(h.r):
        tv[j].index_add_(0, b[j], s[j] * x)
    return False


def query(h: RegionHash, table: torch.Tensor, q0: int = 0, q1: int = -1) -> torch.Tensor:
    """Lower median over rows of the signed cells of every coordinate (only
    chunks [q0, q1) when given, the rest left unset on the GPU)."""
    if table.is_cuda:
        t = h.tensors(table.device)
        return ops().cs_region_query(table, h.d, h.m, h.g, h.W, t["perm"], t["cinfo_l"], t["lists"],
                                     t["goffs"], int(q0), int(q1))
    b, s = h.dense()
    tv = table.view(h.r, h.c)
    vals = torch.stack([s[j] * tv[j][b[j]] for j in range(h.r)])
    return vals.median(dim=0).values


MOM_MODE = {"virtual": 1, "none": 2}


def _topk_ws(h: RegionHash, device, q0: int, q1: int) -> Optional[torch.Tensor]:
    """The candidate-list top-k workspace of this hash and chunk range, kept
    across calls (zeroed once; the kernels leave it zeroed): no memset per
    call.  None when the op sizes its own."""
    cache = h.__dict__.setdefault("_topk_ws", {})
    key = (str(device), int(q0), int(q1))
    ws = cache.get(key)
    if ws is None:
        nb = int(ops().cs_region_topk_ws_bytes(h.d, h.m, int(q0), int(q1)))
        ws = cache[key] = torch.zeros(nb, dtype=torch.uint8, device=device) if nb > 0 else False
    return ws if ws is not False else None


def topk(h: RegionHash, table: torch.Tensor, k: int, hint: Optional[torch.Tensor] = None,
         q0: int = 0, q1: int = -1, mom=None):
    """(idx, vals): the k largest-magnitude median estimates of the
    coordinates of chunks [q0, q1) (idx relative to q0*m, ascending; ties ->
    lower index).  GPU: one fused launch sequence -- the query also builds the
    selection's first histogram (csrc/topk.hip, no extra pass over est).
    ``mom = (V, G, rho, gscale, error_type)``: first the server momentum of
    ops.momentum_ef on the table (error_type "virtual": table is E, V = rho V +
    gscale G, E += V; "none": table is V = rho V + gscale G), on the GPU
    inside the query's staging of the table (every region, whatever the range)."""
    q1 = h.nch if q1 < 0 else q1
    lo, hi = q0 * h.m, min(h.d, q1 * h.m)
    if table.is_cuda and 1 <= k < hi - lo:
        t = h.tensors(table.device)
        mv = mg = None
        rho = gs = 0.0
        mode = 0
        if mom is not None:
            V, G, rho, gs, et = mom
            mode = MOM_MODE[et]
            mv, mg = (V.view(table.shape) if mode == 1 else None), G.view(table.shape)
        return ops().cs_region_topk(table, h.d, h.m, h.g, h.W, t["perm"], t["cinfo_l"], t["lists"],
                                    t["goffs"], int(k), hint, int(q0), int(q1), mv, mg, float(rho),
                                    float(gs), mode, _topk_ws(h, table.device, q0, q1))
    if mom is not None:
        from . import momentum_ef
        V, G, rho, gs, et = mom
        momentum_ef(V.view(-1), table.view(-1) if et == "virtual" else None, G.view(-1), rho, gs, et)
    est = query(h, table, q0, q1)
    return ops().topk_abs(est[lo:hi].contiguous(), int(k), hint)


def zero_buckets(h: RegionHash, t1: torch.Tensor, t2: Optional[torch.Tensor], idx: torch.Tensor,
                 vals: Optional[torch.Tensor]):
    """Zero cells (j, bucket_j(i)) of t1 (and t2) of the coordinates in idx
    with nonzero vals (all of idx when vals is None)."""
    if t1.is_cuda:
        t = h.tensors(t1.device)
        ops().cs_region_zero(t1, t2, idx.contiguous(), vals.contiguous() if vals is not None else None,
                             h.d, h.m, h.g, t["perm"], t["cinfo"])
        return
    sel = idx if vals is None else idx[vals != 0]
    if sel.numel() == 0:
        return
    b = h.buckets_of(sel)
    for t in (t1, t2):
        if t is None:
            continue
        tv = t.view(h.r, h.c)
        for j in range(h.r):
            tv[j, b[j]] = 0.0


def collision_rate(h: RegionHash, pairs: int = 200000, seed: int = 0) -> float:
    """Empirical per-row collision probability of random coordinate pairs
    (for tests: ~1/c like uniform hashing)."""
    b, _ = h.dense()
    g = np.random.default_rng(seed)
    a = torch.from_numpy(g.integers(0, h.d, pairs))
    c = torch.from_numpy(g.integers(0, h.d, pairs))
    keep = a != c
    return float((b[:, a[keep]] == b[:, c[keep]]).float().mean())


__all__ = ["RegionHash", "region_geometry", "encode", "query", "topk", "zero_buckets", "collision_rate"]
