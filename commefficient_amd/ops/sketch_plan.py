"""One-time plan of the atomic-free ("planned") Count-Sketch encode / query
(kernels: csrc/sketch_planned.hip).

The hashes are data-independent, so the r*d (coordinate, row) entries are laid
out once, tile-major: T-bucket table tiles (T = 512..4096, chosen so that a
tile's whole segment of entries fits in LDS), then coordinate chunks, then
(i, j) order.  Returned tensors (all on ``device``):

  src_info[i*r+j]  int16  slot of entry (i, j) in its chunk's LDS stage
  ent_info[e]      int16  in-tile bucket | sign << 15, entry (segment) order
  perm[cm]         int16  at an entry's chunk-major position (encode P1's output
                          layout): its segment-local bucket-order index | sign << 15
  csr              int32  [num_tiles*T + 1] bucket starts in perm
  base             int32  [num_chunks, num_tiles] global start of each run
  off              int32  [num_chunks, num_tiles + 1] in-chunk run starts
  seg              int32  [num_tiles + 1] tile segment starts
  vals             f32    [d*r] scratch shared by encode and query

Built with device sorts (one-time O(rd log rd)): ~0.35 GB for ResNet-9.
Dense geometries (GPT-2: ~249 entries per bucket, a tile's segment does not
fit in LDS) get the dense plan: 8192-bucket tiles, encode P2 accumulating
in LDS in 64-bit fixed point (integer atomics: fast and order independent),
slot 2 (``perm``) holding each entry's in-tile bucket | sign at its
chunk-major position, and slot 10 the fixed-point scratch; the query kernels
are the same.  ``build_plan``
returns None only when d*r >= 2^31.
"""
from __future__ import annotations

from typing import List, Optional

import torch

from .._ext import ops

SEG_CAP = 32767
# entries per bucket the dense plan's 64-bit fixed-point encode has headroom for
# (2^(62 - 46), csrc/sketch_planned.hip kFxBits)
FX_BUCKET_CAP = 1 << 16


def _to_i16(x: torch.Tensor) -> torch.Tensor:
    """u16 bit pattern (0..65535 in an int32/64 tensor) -> int16 tensor."""
    x = x.to(torch.int32)
    return torch.where(x >= 32768, x - 65536, x).to(torch.int16)


def _excl_cumsum(x: torch.Tensor, dim: int = -1) -> torch.Tensor:
    return torch.cumsum(x, dim) - x


@torch.no_grad()
def build_plan(hashes, blk_off, blk_sign, num_blocks: int, d: int, r: int, c: int,
               device) -> Optional[List[torch.Tensor]]:
    geo = [int(v) for v in ops().plan_geometry(d, r, c)]
    if not geo:
        return None
    tile, num_tiles, chunk, num_chunks, dense, p2_splits = geo
    n = d * r
    i64 = torch.int64
    hs = ops().cs_hash_all(hashes, blk_off, blk_sign, num_blocks, d, c, blk_off)  # [d, r]
    neg = (hs < 0).view(-1)
    gb = ((hs & 0x7FFFFFFF).to(i64) + torch.arange(r, device=device, dtype=i64).view(1, r) * c)
    gb = gb.view(-1)
    del hs
    tile_id = gb // tile
    chunk_id = (torch.arange(d, device=device, dtype=i64) // chunk).repeat_interleave(r)
    key = tile_id * num_chunks + chunk_id
    # global (segment) order: by (tile, chunk), stable in (i, j) order
    sorted_key, order = torch.sort(key, stable=True)
    global_pos = torch.empty_like(order)
    global_pos[order] = torch.arange(n, device=device, dtype=order.dtype)
    counts_tc = torch.bincount(key, minlength=num_tiles * num_chunks).view(num_tiles, num_chunks)
    del key
    seg_len = counts_tc.sum(1)
    if not dense and int(seg_len.max()) > SEG_CAP:
        return None
    base_tc = _excl_cumsum(counts_tc.reshape(-1)).view(num_tiles, num_chunks)
    base = base_tc.t().contiguous()                                  # [chunk, tile]
    counts_ct = counts_tc.t().contiguous()
    off = torch.zeros(num_chunks, num_tiles + 1, dtype=i64, device=device)
    off[:, 1:] = torch.cumsum(counts_ct, 1)                          # in-chunk run starts
    local = off[chunk_id, tile_id] + (global_pos - base[chunk_id, tile_id])
    del chunk_id
    src_info = _to_i16(local)
    del local
    seg = torch.zeros(num_tiles + 1, dtype=i64, device=device)
    seg[1:] = torch.cumsum(seg_len, 0)
    sign_bit = neg.to(i64) << 15
    lb = gb & (tile - 1)
    ent_info = torch.empty(n, dtype=torch.int16, device=device)
    ent_info[global_pos] = _to_i16(lb | sign_bit)
    del tile_id, global_pos
    if dense and int(torch.bincount(gb, minlength=r * c).max()) > FX_BUCKET_CAP:
        return None  # the fixed-point encode's headroom (never at hashed loads)
    if dense:
        # encode P2 accumulates with LDS atomics: slot 2 holds each entry's
        # in-tile bucket | sign at its CHUNK-MAJOR position (P1's output
        # layout); no bucket-order permutation
        cm = (torch.arange(d, device=device, dtype=i64) // chunk).repeat_interleave(r) \
            * (chunk * r) + src_info.to(i64).bitwise_and(0xFFFF)
        cm_info = torch.empty(n, dtype=torch.int16, device=device)
        cm_info[cm] = _to_i16(lb | sign_bit)
        del cm, lb, sign_bit, order, sorted_key
        csr = torch.zeros(num_tiles * tile + 1, dtype=i64, device=device)
        perm = cm_info
    else:
        del lb
        perm, csr = _bucket_order(gb, order, sorted_key, num_chunks, seg, src_info, chunk, d, r,
                                  n, sign_bit, tile, num_tiles, device)
    del gb
    vals = torch.empty(n, dtype=torch.float32, device=device)
    # encode P2 gathers tile t's run of every chunk from the chunk-major P1
    # output: tile-major run metadata (start in chunk-major vals, start in
    # the segment)
    p2_src = (torch.arange(num_chunks, device=device, dtype=i64).view(1, -1) * (chunk * r)
              + off[:, :num_tiles].t())
    p2_pos = torch.zeros(num_tiles, num_chunks + 1, dtype=i64, device=device)
    p2_pos[:, 1:] = torch.cumsum(counts_tc, 1)
    i32 = torch.int32
    plan = [src_info, ent_info, perm, csr.to(i32), base.to(i32), off.to(i32), seg.to(i32), vals,
            p2_src.to(i32).contiguous(), p2_pos.to(i32)]
    if dense:
        # fixed-point encode P2 scratch: int64 split partials [p2_splits,
        # num_tiles*tile], then (as floats) max|v| per chunk and overall
        plan.append(torch.empty(p2_splits * num_tiles * tile + (num_chunks + 2) // 2 + 1,
                                dtype=torch.int64, device=device))
    return plan


def _bucket_order(gb, order, sorted_key, num_chunks, seg, src_info, chunk, d, r, n, sign_bit,
                  tile, num_tiles, device):
    """(perm, csr) of the exact plan: each entry's segment-local bucket-order
    index | sign at its chunk-major position, and the bucket starts."""
    i64 = torch.int64
    # bucket order: entries (in segment order) stably sorted by global bucket;
    # encode P2 scatters each entry straight to its bucket-order slot, so the
    # plan stores, at the entry's CHUNK-MAJOR position (P1's output layout),
    # its segment-local bucket-order index | sign << 15
    gb_pos = gb[order]
    _, perm_pos = torch.sort(gb_pos, stable=True)           # bucket order -> segment pos
    bo_of_pos = torch.empty_like(perm_pos)
    bo_of_pos[perm_pos] = torch.arange(n, device=device, dtype=perm_pos.dtype)
    tile_of_pos = sorted_key // num_chunks
    bo_local = bo_of_pos - seg[tile_of_pos]                 # per segment position
    del gb_pos, perm_pos, bo_of_pos, tile_of_pos
    # entry e = i*r+j: segment position global_pos_e, chunk-major position
    # chunk(i)*chunk*r + slot_e
    cm = (torch.arange(d, device=device, dtype=i64) // chunk).repeat_interleave(r) * (chunk * r) \
        + src_info.to(i64).bitwise_and(0xFFFF)
    gpos_e = torch.empty_like(order)
    gpos_e[order] = torch.arange(n, device=device, dtype=order.dtype)
    perm = torch.empty(n, dtype=torch.int16, device=device)
    perm[cm] = _to_i16(bo_local[gpos_e] | sign_bit)
    del cm, gpos_e, bo_local
    csr = torch.zeros(num_tiles * tile + 1, dtype=i64, device=device)
    csr[1:] = torch.cumsum(torch.bincount(gb, minlength=num_tiles * tile), 0)
    return perm, csr
