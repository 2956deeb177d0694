"""Region-permutation Count-Sketch hash family (``--encode region``, default).

The coordinates are cut into chunks of ``m`` consecutive coordinates and each
table row into ``R = c // m`` regions of ``m`` buckets.  In row ``j`` chunk
``q`` is dealt to region ``rho_j(q)`` (a random order, dealt evenly) and its
coordinate ``o`` goes to bucket ``rho_j(q)*m + (P_j(o) + shift_j(q)) mod m``
with sign ``S_j(o) * sigma_j(q)``, where ``P_j`` is a random permutation of
``[m]``.  Chunk-mates never collide (a bijection inside the chunk); two
coordinates of different chunks collide with probability ``1/(R*m) ~= 1/c`` per
row, independently across rows -- the pairwise property the Count-Sketch
unbiasedness and variance bounds use (csvec's own ``numBlocks`` layout also
reuses one hash per block with a per-block offset and sign:
/root/reference/CommEfficient/fed_aggregator.py:464-467 builds it).

Why this family on MI355X: the encode becomes "add each chunk into its region"
(region-sized LDS accumulators, no atomics, no plan arrays, no r*d
intermediate) and the median query "stage the chunk's r regions in LDS and
gather" (csrc/sketch_region.hip).  The parameters are a few hundred KB built
once from the seed with numpy, identical on every rank.

The CPU implementation below (dense bucket / sign arrays, ``index_add_``,
``torch.median`` = lower median) defines the same family for CPU runs and
serves as the reference the GPU kernels are tested against.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from .._ext import ops


def region_size(c: int, r: int, target: int = 2048) -> int:
    """Chunk / region size m for a c-column, r-row table: about ``target``
    (one 8 KB LDS copy per wave in the encode), r regions in LDS for the query
    (r*m*4 <= 160 KB), and c // m regions (at most R - 1 buckets unused)."""
    target = max(1, min(int(target), (160 * 1024) // (4 * max(1, r))))
    if c <= target:
        return int(c)
    R = -(-c // target)
    return int(c // R)


class RegionHash:
    """Parameters of one (d, c, r, seed) region sketch.

    Host arrays (numpy): ``P`` [r, m] permutation, ``S`` [r, m] sign bit,
    ``region`` [r, nch], ``shift`` [r, nch], ``sigma`` [r, nch] sign bit.
    Device tensors (``tensors(device)``): perm / cinfo / lists / offs as the
    kernels read them (csrc/kernels.h)."""

    def __init__(self, d: int, c: int, r: int, seed: int = 42, m: Optional[int] = None):
        self.d, self.c, self.r = int(d), int(c), int(r)
        self.m = int(m) if m else region_size(self.c, self.r)
        assert 1 <= self.m <= self.c
        self.R = self.c // self.m
        self.nch = -(-self.d // self.m)
        rng = np.random.default_rng([int(seed), 0x5E610, self.d, self.c, self.r])
        r_, m_, nch, R = self.r, self.m, self.nch, self.R
        self.P = np.stack([rng.permutation(m_) for _ in range(r_)]).astype(np.int64)
        self.S = rng.integers(0, 2, size=(r_, m_), dtype=np.int64)
        region = np.empty((r_, nch), dtype=np.int64)
        for j in range(r_):
            order = rng.permutation(nch)
            region[j, order] = np.arange(nch) % R  # dealt evenly
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
            r_, m_, nch, R = self.r, self.m, self.nch, self.R
            perm = (self.P | (self.S << 31)).astype(np.uint32).view(np.int32)
            cinfo = np.empty((r_, nch, 2), dtype=np.uint32)
            cinfo[..., 0] = (self.region * m_).astype(np.uint32)
            cinfo[..., 1] = (self.shift | (self.sigma << 31)).astype(np.uint32)
            lists = np.empty((r_, nch), dtype=np.int32)
            offs = np.empty((r_, R + 1), dtype=np.int32)
            for j in range(r_):
                order = np.lexsort((np.arange(nch), self.region[j]))  # by region, then chunk
                lists[j] = order
                offs[j] = np.searchsorted(self.region[j][order], np.arange(R + 1))
            t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)  # noqa: E731
            self._dev[key] = {"perm": t(perm), "cinfo": t(cinfo.view(np.int32)),
                              "lists": t(lists), "offs": t(offs)}
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
           wvec: Optional[torch.Tensor] = None, wscale: float = 0.0, overwrite: bool = False):
    """table (+)= S(scale*vec + wscale*wvec)."""
    v = vec.reshape(-1)
    if table.is_cuda:
        t = h.tensors(table.device)
        ops().cs_region_encode(table, v, float(scale), wvec.reshape(-1) if wvec is not None else None,
                               float(wscale), h.m, t["perm"], t["cinfo"], t["lists"], t["offs"],
                               bool(overwrite))
        return
    x = v.float() * scale
    if wvec is not None and wscale != 0.0:
        x = x + wscale * wvec.reshape(-1).float()
    b, s = h.dense()
    if overwrite:
        table.zero_()
    tv = table.view(h.r, h.c)
    for j in range(h.r):
        tv[j].index_add_(0, b[j], s[j] * x)


def query(h: RegionHash, table: torch.Tensor, q0: int = 0, q1: int = -1) -> torch.Tensor:
    """Lower median over rows of the signed cells of every coordinate (only
    chunks [q0, q1) when given, the rest left unset on the GPU)."""
    if table.is_cuda:
        t = h.tensors(table.device)
        return ops().cs_region_query(table, h.d, h.m, t["perm"], t["cinfo"], int(q0), int(q1))
    b, s = h.dense()
    tv = table.view(h.r, h.c)
    vals = torch.stack([s[j] * tv[j][b[j]] for j in range(h.r)])
    return vals.median(dim=0).values


def zero_buckets(h: RegionHash, t1: torch.Tensor, t2: Optional[torch.Tensor], idx: torch.Tensor,
                 vals: Optional[torch.Tensor]):
    """Zero cells (j, bucket_j(i)) of t1 (and t2) of the coordinates in idx
    with nonzero vals (all of idx when vals is None)."""
    if t1.is_cuda:
        t = h.tensors(t1.device)
        ops().cs_region_zero(t1, t2, idx.contiguous(), vals.contiguous() if vals is not None else None,
                             h.d, h.m, t["perm"], t["cinfo"])
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


__all__ = ["RegionHash", "region_size", "encode", "query", "zero_buckets", "collision_rate"]
