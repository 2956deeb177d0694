"""Count Sketch backed by the native ``commeff`` ops.

API-compatible with the ``csvec.CSVec`` object the reference uses
(SURVEY.md §2.4 X1): ``CSVec(d, c, r, device, numBlocks)``, ``accumulateVec``,
``accumulateTable``, ``unSketch(k)``, ``zero()``, ``l2estimate()``, ``.table``
and ``/``.  Call sites in the reference:
/root/reference/CommEfficient/fed_worker.py:313-320,
/root/reference/CommEfficient/fed_aggregator.py:464-467,584-595,
/root/reference/CommEfficient/utils.py:305-313.

Differences by design (MI355X-first):
* hashes are recomputed inside the kernels from 4 coefficients per row
  (``hashes`` is a tiny CPU int64 tensor), so no r x d index tables exist --
  except for the default GPU "planned" kernels, which trade a one-time
  permutation plan (ops/sketch_plan.py, ~0.4 GB at ResNet-9 size) for
  atomic-free, bitwise-deterministic encode and query;
* ``unSketch`` returns the dense vector like CSVec, while ``unsketch_sparse``
  returns the ``(idx, vals)`` pair straight from the deterministic radix
  select, which is what the server step uses;
* ``zero_heavy_hitters`` zeroes the r cells of each recovered coordinate
  directly instead of re-sketching the update and taking ``nonzero()``
  (identical except when two heavy hitters cancel exactly in a bucket).
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np
import torch

from .._ext import ops

def make_hashes(r: int, c: int, num_blocks: int = 1, seed: int = 42):
    """Deterministic hash coefficients (identical on every rank for one seed).

    Per row: multiply-add-shift parameters (a, b) for the bucket and (a2, b2)
    for the sign, as u64 bit patterns in an int64 tensor (a, a2 odd); see
    csrc/sketch_hash.h.  Returns ``(hashes[r,4] int64 cpu, blk_off[r,nb] int32
    cpu, blk_sign[r,nb] f32 cpu)``.
    """
    rng = np.random.RandomState(seed)
    u = rng.randint(0, 2 ** 32, size=(r, 4, 2), dtype=np.uint64)
    words = (u[..., 0] << np.uint64(32)) | u[..., 1]
    words[:, 0] |= np.uint64(1)
    words[:, 2] |= np.uint64(1)
    hashes = torch.from_numpy(words.view(np.int64).copy())
    nb = max(1, int(num_blocks))
    blk_off = torch.from_numpy(rng.randint(0, c, size=(r, nb)).astype(np.int32))
    blk_sign = torch.from_numpy(
        (rng.randint(0, 2, size=(r, nb)) * 2 - 1).astype(np.float32))
    return hashes, blk_off, blk_sign



def _rg():
    from . import sketch_region
    return sketch_region


def _topk_hint(tag, device):
    from . import topk_hint
    return topk_hint(tag, device)

class CSVec:
    """Count Sketch of a d-dimensional vector into an r x c fp32 table."""

    def __init__(self, d: int, c: int, r: int, device="cpu", numBlocks: int = 1,
                 seed: int = 42, table: Optional[torch.Tensor] = None,
                 _hashes=None, _scratch=None, kernel: str = "planned"):
        self.d = int(d)
        self.c = int(c)
        self.r = int(r)
        self.device = torch.device(device)
        self.numBlocks = max(1, int(numBlocks))
        self.seed = seed
        # GPU encode/query kernels: "planned" (precomputed permutation, atomic
        # free, deterministic), "binned" (LDS atomics) or "direct" (global
        # atomics / random gathers) on the multiply-shift family below, or
        # "region": the region-permutation family of ops/sketch_region.py
        # (its own hashes; CPU and GPU)
        self.kernel = kernel
        if _hashes is None:
            h, bo, bs = make_hashes(self.r, self.c, self.numBlocks, seed)
            bo = bo.to(self.device)
            bs = bs.to(self.device)
            _hashes = (h, bo, bs)
        self.hashes, self.blk_off, self.blk_sign = _hashes
        fresh = table is None
        if fresh:
            table = torch.zeros(self.r, self.c, device=self.device, dtype=torch.float32)
        self.table = table
        # GPU encode/query plans, built once per geometry (the hash -> tile
        # mapping is data-independent) and shared by every sketch derived
        # with like()
        self._scratch = _scratch if _scratch is not None else {}
        self.region = None
        if kernel == "region":
            if "region" not in self._scratch:
                from .sketch_region import RegionHash
                self._scratch["region"] = RegionHash(self.d, self.c, self.r, seed)
            self.region = self._scratch["region"]
            if fresh and self._scratch.get("layout_world", 1) > 1:
                self.table = self.new_table()

    # -- construction helpers -------------------------------------------------
    def like(self, table: Optional[torch.Tensor] = None) -> "CSVec":
        """A sketch with the same hashes (cheap: shares the coefficient tensors
        and the kernel plans)."""
        return CSVec(self.d, self.c, self.r, self.device, self.numBlocks, self.seed,
                     table=table, _hashes=(self.hashes, self.blk_off, self.blk_sign),
                     _scratch=self._scratch, kernel=self.kernel)

    def _binned_layout(self):
        """[counts, base, seg, entries] for the binned GPU encode."""
        if self.device.type != "cuda" or self.r * self.c > 2048 * 8192:
            return []  # direct encode (binned run tables must fit in LDS)
        if "binned" not in self._scratch:
            counts, base, seg = ops().cs_layout(self.hashes, self.blk_off, self.blk_sign,
                                                self.numBlocks, self.d, self.c, self.blk_off)
            nbytes = ops().binned_scratch_bytes(self.d, self.r, self.c, self.numBlocks)
            entries = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
            self._scratch["binned"] = [counts, base, seg, entries]
        return self._scratch["binned"]

    def _plan(self):
        if "planned" not in self._scratch:
            from .sketch_plan import build_plan
            self._scratch["planned"] = build_plan(self.hashes, self.blk_off, self.blk_sign,
                                                  self.numBlocks, self.d, self.r, self.c,
                                                  self.device)
        return self._scratch["planned"]

    def _use_plan(self) -> bool:
        # the plan is None when the geometry does not fit the planned kernels
        # (csrc/sketch_planned.hip); the binned kernels are used then
        return self.device.type == "cuda" and self.kernel == "planned" and self._plan() is not None

    # -- CSVec API --------------------------------------------------------------
    def zero(self):
        self.table.zero_()

    def accumulateVec(self, vec: torch.Tensor, scale: float = 1.0,
                      wvec: Optional[torch.Tensor] = None, wscale: float = 0.0,
                      dense: bool = True, overwrite: bool = False, zero_vec: bool = False) -> bool:
        """table += S(scale*vec + wscale*wvec) (``overwrite``: table = S(...),
        no separate zeroing pass on the planned path).  ``dense=False`` uses
        the direct-atomic kernel (best for sparse vectors).  ``zero_vec``: the
        region GPU encode may clear vec behind its reads; returns True if it
        did (the caller then skips its own zeroing of vec)."""
        assert vec.numel() == self.d, (vec.numel(), self.d)
        if self.region is not None:
            return _rg().encode(self.region, self.table, vec, scale, wvec, wscale, overwrite, zero_vec)
        if dense and self._use_plan():
            ops().cs_encode_planned(self.table, vec.reshape(-1), float(scale), wvec,
                                    float(wscale), self.c, self._plan(), bool(overwrite))
            return False
        if overwrite:
            self.table.zero_()
        layout = self._binned_layout() if (dense and self.kernel != "direct") else []
        ops().cs_encode(self.table, vec.reshape(-1), self.hashes, self.blk_off, self.blk_sign,
                        self.numBlocks, float(scale), wvec, float(wscale), layout)
        return False

    def accumulateTable(self, table: torch.Tensor):
        self.table.add_(table.view(self.r, self.c))

    def query(self) -> torch.Tensor:
        """Median-of-rows estimate of every coordinate (dense, length d)."""
        if self.region is not None:
            return _rg().query(self.region, self.table)
        if self._use_plan():
            return ops().cs_query_planned(self.table, self.d, self._plan())
        if self.device.type == "cuda" and self.kernel != "direct":
            # no plan (e.g. GPT-2's 249 entries per bucket): one gather pass per
            # table row (an L2-resident 2 MB row) + a median pass; 2x the
            # hash-on-the-fly query at GPT-2 size (scripts/bench_codec.py)
            return ops().cs_query_rows(self.table, self.hashes, self.blk_off, self.blk_sign,
                                       self.numBlocks, self.d)
        return ops().cs_query(self.table, self.hashes, self.blk_off, self.blk_sign,
                              self.numBlocks, self.d)

    def unsketch_sparse(self, k: int, mom=None) -> Tuple[torch.Tensor, torch.Tensor]:
        """``mom = (V, G, rho, gscale, error_type)``: apply the server momentum
        to the table first (ops.momentum_ef; fused into the query on the GPU
        region path)."""
        if self.region is not None:
            return _rg().topk(self.region, self.table, int(k),
                              _topk_hint(("unsketch", self.d, int(k)), self.table.device), mom=mom)
        self._momentum(mom)
        est = self.query()
        return ops().topk_abs(est, int(k), _topk_hint(("unsketch", self.d, int(k)), est.device))

    def shard_bounds(self, world: int) -> Optional[list]:
        """Coordinate shard boundaries [b_0 = 0, ..., b_world = d] at plan-chunk
        granularity (shard q = chunks [nch*q//world, nch*(q+1)//world)), or
        None when the query is not planned (no chunk structure)."""
        if self.region is not None:
            m = self.region.m
            return [min(self.d, q * m) for q in self.region.chunk_bounds(world)]
        if not self._use_plan():
            return None
        geom = ops().plan_geometry(self.d, self.r, self.c)
        chunk, nch = int(geom[2]), int(geom[3])
        return [min(self.d, (nch * q // world) * chunk) for q in range(world + 1)]

    def _momentum(self, mom):
        if mom is not None:
            from . import momentum_ef
            V, G, rho, gs, et = mom
            momentum_ef(V.view(-1), self.table.view(-1) if et == "virtual" else None, G.view(-1), rho,
                        gs, et)

    def unsketch_sparse_sharded(self, k: int, rank: int, world: int, all_gather_rows, mom=None):
        """``unsketch_sparse`` with the median query and the top-k split over
        ``world`` ranks: rank r estimates only its coordinate shard, selects
        the shard's k largest |estimates| (ties -> lower index), the k-lists
        are all-gathered (one collective of 2k int64 per rank) and every rank
        selects the k best of the N*k candidates.  The candidates are in
        ascending coordinate order (shards ascend with the rank, each list is
        sorted), so "lower position" is "lower index" and the result is
        bitwise the unsharded one: every member of the global top-k is in its
        shard's top-k.  Falls back to the unsharded path when a shard holds
        fewer than k coordinates or the query is not planned."""
        k = int(k)
        b = self.shard_bounds(world) if world > 1 else None
        if b is None or min(b[q + 1] - b[q] for q in range(world)) < k:
            return self.unsketch_sparse(k, mom=mom)
        pack = self.unsketch_shard(k, rank, world, b, mom=mom)
        return self.merge_shards(all_gather_rows(pack.view(1, 2 * k)), world, k)

    def unsketch_shard(self, k: int, rank: int, world: int, bounds=None, mom=None) -> torch.Tensor:
        """This rank's candidates: [2, k] int64 = (global indices, fp32 bits of
        the estimates) of its shard's top-k."""
        b = bounds if bounds is not None else self.shard_bounds(world)
        lo, hi = b[rank], b[rank + 1]
        hint = _topk_hint(("unsketch_shard", self.d, k, rank, world), self.table.device)
        if self.region is not None:
            qb = self.region.chunk_bounds(world)
            li, lv = _rg().topk(self.region, self.table, k, hint, qb[rank], qb[rank + 1], mom=mom)
        else:
            self._momentum(mom)
            nch = int(ops().plan_geometry(self.d, self.r, self.c)[3])
            est = ops().cs_query_planned(self.table, self.d, self._plan(), nch * rank // world,
                                         nch * (rank + 1) // world)
            li, lv = ops().topk_abs(est[lo:hi], k, hint)
        pack = torch.empty(2, k, dtype=torch.int64, device=self.device)
        pack[0] = li + lo
        pack[1] = lv.view(torch.int32)
        return pack

    @staticmethod
    def merge_shards(allp: torch.Tensor, world: int, k: int):
        """(idx, vals) of the k best of every rank's candidates (rank order)."""
        allp = allp.view(world, 2, k)
        idx_all = allp[:, 0].reshape(-1)
        val_all = allp[:, 1].to(torch.int32).view(torch.float32).reshape(-1)
        pos, vals = ops().topk_abs(val_all, k)
        return idx_all.index_select(0, pos), vals

    def unSketch(self, k: int) -> torch.Tensor:
        idx, vals = self.unsketch_sparse(k)
        return ops().scatter_dense(idx, vals, self.d)

    def zero_heavy_hitters(self, idx: torch.Tensor, vals: Optional[torch.Tensor],
                           other: Optional[torch.Tensor] = None):
        """Zero cells (j, h_j(i)) of this table (and ``other``) for recovered
        coordinates i with nonzero value -- the reference's
        ``nz = S(delta).nonzero(); table[nz] = 0``."""
        if self.region is not None:
            _rg().zero_buckets(self.region, self.table, other, idx, vals)
            return
        ops().cs_zero_buckets(self.table, other, idx, vals, self.hashes, self.blk_off,
                              self.blk_sign, self.numBlocks, self.d)

    def zero_heavy_hitters_apply(self, idx: torch.Tensor, vals: torch.Tensor, other: Optional[torch.Tensor],
                                 w: torch.Tensor, lr: float, lr_vec, last_mod, round_idx: int, hist,
                                 step: Optional[torch.Tensor] = None, g0: int = 0) -> bool:
        """zero_heavy_hitters + ops.sparse_apply(w, idx, vals, ...) in one GPU
        kernel (region family; ``g0``: a group-major shard's first group).
        Returns False (nothing done) where the fused kernel does not apply;
        the caller then runs the two steps."""
        if self.region is None or not self.table.is_cuda or w.numel() != self.d or self.r > 8:
            return False
        t = self.region.tensors(self.table.device)
        ops().cs_region_zero_apply(self.table, other, idx.contiguous(), vals.contiguous(), self.d,
                                   self.region.m, self.region.g, t["perm"], t["cinfo"], w, float(lr),
                                   lr_vec, last_mod, int(round_idx), hist, step, int(g0))
        return True

    # -- group-major tables (sharded server, parallel/server.py) -------------
    def layout_world(self) -> int:
        return getattr(self, "_layout_world", 1)

    def set_group_layout(self, world: int):
        """Tables of this sketch (and of ``like``/``new_table``) become the
        padded group-major [world * Gp, r, g*m] of the region family, so a
        reduce-scatter hands every rank a contiguous slice of whole groups."""
        assert self.region is not None, "group layout: region family only"
        self._layout_world = int(world)
        self._scratch["layout_world"] = int(world)
        self.table = self.new_table()

    def table_shape(self):
        w = self._scratch.get("layout_world", 1)
        if self.region is None or w <= 1:
            return (self.r, self.c)
        h = self.region
        return (w * h.shard_groups(w), self.r, h.g * h.m)

    def table_numel(self) -> int:
        n = 1
        for x in self.table_shape():
            n *= x
        return n

    def new_table(self) -> torch.Tensor:
        return torch.zeros(self.table_shape(), device=self.device, dtype=torch.float32)

    def table_view(self, flat: torch.Tensor) -> torch.Tensor:
        return flat.view(self.table_shape())

    def l2estimate(self) -> torch.Tensor:
        if self.table.dim() == 3:  # group-major: row sums over the groups
            rs = self.table.double().square().sum(dim=(0, 2))
            return rs.median().sqrt().float()
        return ops().cs_l2estimate(self.table)

    def __truediv__(self, other):
        return self.like(self.table / float(other))

    def __iadd__(self, other):
        if isinstance(other, CSVec):
            self.table += other.table
        else:
            self.table += other
        return self
