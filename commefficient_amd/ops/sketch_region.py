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

    # ---------------------------------------------------- table layouts
    # A table is row-major [r, c] (every group) or group-major [Gs, r, g*m]
    # holding groups [g0, g0 + Gs) -- the sharded server's per-rank state and
    # its padded payload (csrc/kernels.h RegionLayout).
    def shard_groups(self, world: int) -> int:
        """Groups per rank of the sharded server (the payload pads G to
        world * this)."""
        return -(-self.G // int(world))

    def cells(self, table: torch.Tensor, g0: int = 0):
        """(cell [r, d] int64 flat index into ``table``, valid [d] bool: the
        coordinate's group lies in the table) for the table's layout."""
        key = (tuple(table.shape), int(g0))
        cache = self.__dict__.setdefault("_cells", {})
        if key not in cache:
            b, _ = self.dense()
            gm = self.g * self.m
            grp = b // gm
            if table.dim() == 3:
                Gs = table.shape[0]
                cell = (grp - g0) * (self.r * gm) + torch.arange(self.r).view(-1, 1) * gm + (b - grp * gm)
                valid = (grp[0] >= g0) & (grp[0] < g0 + Gs)  # (a chunk's group is the same in every row)
            else:
                cell = torch.arange(self.r).view(-1, 1) * self.c + b
                valid = torch.ones(self.d, dtype=torch.bool)
            cache[key] = (torch.where(valid.view(1, -1), cell, torch.zeros_like(cell)), valid)
        return cache[key]

    def shard_ok(self, world: int, k: int) -> bool:
        """Every rank's groups hold more than k coordinates (the sharded
        server's per-rank top-k needs k < shard size)."""
        Gp = self.shard_groups(world)
        for r in range(world):
            mine = int(np.sum((self.group >= r * Gp) & (self.group < (r + 1) * Gp)))
            if mine * self.m - (self.nch * self.m - self.d) <= k:
                return False
        return True

    def shard_maps(self, g0: int, g1: int, device):
        """(cpos [nch] int32: compact position of every chunk of groups
        [g0, g1), -1 elsewhere; cmap [nsh] int32: the shard's chunks ascending;
        ncoord: its coordinates) -- the sharded query writes the shard's
        estimates compactly, in ascending coordinate order."""
        key = (int(g0), int(g1), str(torch.device(device)))
        cache = self.__dict__.setdefault("_shard_maps", {})
        if key not in cache:
            mine = np.nonzero((self.group >= g0) & (self.group < g1))[0]
            cpos = np.full(self.nch, -1, dtype=np.int32)
            cpos[mine] = np.arange(len(mine), dtype=np.int32)
            ncoord = len(mine) * self.m
            if len(mine) and mine[-1] == self.nch - 1:  # the last chunk may be partial
                ncoord -= self.nch * self.m - self.d
            t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)  # noqa: E731
            cache[key] = (t(cpos), t(mine.astype(np.int32)), int(ncoord))
        return cache[key]

    def group_major(self, rm: torch.Tensor, world: int) -> torch.Tensor:
        """Row-major [r, c] -> the padded group-major [world * Gp, r, g*m]."""
        gm, Gp = self.g * self.m, self.shard_groups(world)
        out = torch.zeros(world * Gp, self.r, gm, dtype=rm.dtype, device=rm.device)
        out[:self.G] = rm.view(self.r, self.c)[:, :self.G * gm].reshape(self.r, self.G, gm).permute(1, 0, 2)
        return out

    def row_major(self, gmj: torch.Tensor, g0: int = 0) -> torch.Tensor:
        """Group-major groups [g0, g0 + Gs) -> row-major [r, c] (zeros elsewhere)."""
        gm = self.g * self.m
        out = torch.zeros(self.r, self.c, dtype=gmj.dtype, device=gmj.device)
        n = max(0, min(gmj.shape[0], self.G - g0))
        out[:, g0 * gm:(g0 + n) * gm] = gmj[:n].permute(1, 0, 2).reshape(self.r, n * gm)
        return out

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
    _, s = h.dense()
    cell, valid = h.cells(table)
    assert bool(valid.all()), "region encode: the table must hold every group"
    if overwrite:
        table.zero_()
    tf = table.view(-1)
    for j in range(h.r):
        tf.index_add_(0, cell[j], s[j] * x)
    return False


def query(h: RegionHash, table: torch.Tensor, q0: int = 0, q1: int = -1, g0: int = 0) -> torch.Tensor:
    """Lower median over rows of the signed cells of every coordinate (only
    chunks [q0, q1) -- and, for a group-major shard, the coordinates of its
    groups -- when given; the rest left unset on the GPU, 0 on the CPU)."""
    if table.is_cuda:
        t = h.tensors(table.device)
        return ops().cs_region_query(table, h.d, h.m, h.g, h.W, t["perm"], t["cinfo_l"], t["lists"],
                                     t["goffs"], int(q0), int(q1), int(g0))
    _, s = h.dense()
    cell, valid = h.cells(table, g0)
    tf = table.reshape(-1)
    vals = torch.stack([s[j] * tf[cell[j]] for j in range(h.r)])
    return torch.where(valid, vals.median(dim=0).values, torch.zeros((), dtype=vals.dtype))


MOM_MODE = {"virtual": 1, "none": 2}


def _topk_ws(h: RegionHash, device, q0: int, q1: int, tag=None) -> Optional[torch.Tensor]:
    """The candidate-list top-k workspace of this hash and chunk range, kept
    across calls (zeroed once; the kernels leave it zeroed): no memset per
    call.  None when the op sizes its own."""
    q1 = h.nch if q1 < 0 else q1
    cache = h.__dict__.setdefault("_topk_ws", {})
    key = (str(device), int(q0), int(q1), tag)
    ws = cache.get(key)
    if ws is None:
        nb = int(ops().cs_region_topk_ws_bytes(h.d, h.m, int(q0), int(q1)))
        ws = cache[key] = torch.zeros(nb, dtype=torch.uint8, device=device) if nb > 0 else False
    return ws if ws is not False else None


def topk(h: RegionHash, table: torch.Tensor, k: int, hint: Optional[torch.Tensor] = None,
         q0: int = 0, q1: int = -1, mom=None, g0: int = 0):
    """(idx, vals): the k largest-magnitude median estimates of the
    coordinates of chunks [q0, q1) (idx relative to q0*m, ascending; ties ->
    lower index).  GPU: one fused launch sequence -- the query also builds the
    selection's first histogram (csrc/topk.hip, no extra pass over est).
    ``mom = (V, G, rho, gscale, error_type)``: first the server momentum of
    ops.momentum_ef on the table (error_type "virtual": table is E, V = rho V +
    gscale G, E += V; "none": table is V = rho V + gscale G), on the GPU
    inside the query's staging of the table (every region, whatever the range).
    A group-major shard (table [Gs, r, g*m] of groups [g0, g0 + Gs)): only
    its groups' coordinates are candidates; idx are global and ascending."""
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
        if table.dim() == 3:  # a group-major shard: compact estimates, global idx
            cpos, cmap, ncoord = h.shard_maps(g0, g0 + table.shape[0], table.device)
            li, lv = ops().cs_region_topk(table, h.d, h.m, h.g, h.W, t["perm"], t["cinfo_l"], t["lists"],
                                          t["goffs"], int(k), hint, 0, -1, mv, mg, float(rho), float(gs),
                                          mode, _topk_ws(h, table.device, 0, -1, ("shard", g0)), int(g0),
                                          cpos, ncoord)
            return li, lv, cmap
        return ops().cs_region_topk(table, h.d, h.m, h.g, h.W, t["perm"], t["cinfo_l"], t["lists"],
                                    t["goffs"], int(k), hint, int(q0), int(q1), mv, mg, float(rho),
                                    float(gs), mode, _topk_ws(h, table.device, q0, q1))
    if mom is not None:
        from . import momentum_ef
        V, G, rho, gs, et = mom
        momentum_ef(V.view(-1), table.view(-1) if et == "virtual" else None, G.view(-1), rho, gs, et)
    est = query(h, table, q0, q1, g0)
    if table.dim() == 3:  # candidates: the shard's coordinates only (ascending), global idx
        _, valid = h.cells(table, g0)
        cand = torch.nonzero(valid).view(-1)
        p, v = ops().topk_abs(est[cand].contiguous(), int(k), hint)
        return cand[p], v, None
    return ops().topk_abs(est[lo:hi].contiguous(), int(k), hint)


def zero_buckets(h: RegionHash, t1: torch.Tensor, t2: Optional[torch.Tensor], idx: torch.Tensor,
                 vals: Optional[torch.Tensor], g0: int = 0):
    """Zero cells (j, bucket_j(i)) of t1 (and t2) of the coordinates in idx
    with nonzero vals (all of idx when vals is None) -- for a group-major
    shard only those of its groups."""
    if t1.is_cuda:
        t = h.tensors(t1.device)
        ops().cs_region_zero(t1, t2, idx.contiguous(), vals.contiguous() if vals is not None else None,
                             h.d, h.m, h.g, t["perm"], t["cinfo"], int(g0))
        return
    sel = idx if vals is None else idx[vals != 0]
    cell, valid = h.cells(t1, g0)
    sel = sel[valid[sel]]
    if sel.numel() == 0:
        return
    for t in (t1, t2):
        if t is None:
            continue
        tf = t.view(-1)
        for j in range(h.r):
            tf[cell[j][sel]] = 0.0


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
