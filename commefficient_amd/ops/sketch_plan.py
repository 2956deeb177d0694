"""One-time plan of the atomic-free ("planned") Count-Sketch encode / query.

The hashes are data-independent, so the r*d (coordinate, row) entries can be
laid out once, tile-major (8192-bucket table tile, then coordinate chunk, then
(i, j) order), with everything the kernels of csrc/sketch_planned.hip need:

  src_info[i*r+j]  int16  in-chunk LDS staging slot | sign << 15
  ent_info[e]      int16  bucket inside the tile    | sign << 15  (entry order)
  perm[x]          int32  entry indices sorted by (tile, bucket)
  csr              int32  [num_tiles*8192 + 1] bucket boundaries into perm
  base, off        int32  [num_chunks, num_tiles] run starts (global / in-chunk)
  seg              int32  [num_tiles + 1] tile segment starts
  vals             f32    [d*r] scratch shared by encode and query

Built with two stable device sorts (torch), so it costs one-time O(rd log rd)
work; ~0.4 GB of plan for ResNet-9, ~7 GB for GPT-2 (288 GB HBM per MI355X).
"""
from __future__ import annotations

from typing import List

import torch

from .._ext import ops


def _to_i16(x: torch.Tensor) -> torch.Tensor:
    """u16 bit pattern (0..65535 in an int32/64 tensor) -> int16 tensor."""
    x = x.to(torch.int32)
    return torch.where(x >= 32768, x - 65536, x).to(torch.int16)


@torch.no_grad()
def build_plan(hashes, blk_off, blk_sign, num_blocks: int, d: int, r: int, c: int,
               device) -> List[torch.Tensor]:
    tile, num_tiles, chunk, num_chunks = [int(v) for v in ops().binned_plan(d, r, c)]
    n = d * r
    if n >= 2 ** 31:
        raise ValueError("planned sketch supports d*r < 2^31 entries")
    hs = ops().cs_hash_all(hashes, blk_off, blk_sign, num_blocks, d, c, blk_off)  # [d, r]
    neg = (hs < 0).view(-1)
    bucket = (hs & 0x7FFFFFFF).to(torch.int64)
    del hs
    gb = bucket + torch.arange(r, device=device, dtype=torch.int64).view(1, r) * c
    del bucket
    tile_id = (gb >> 13).view(-1)
    lb = (gb & (tile - 1)).view(-1)
    del gb
    chunk_id = (torch.arange(d, device=device, dtype=torch.int64) // chunk).repeat_interleave(r)
    key = tile_id * num_chunks + chunk_id
    # entries sorted by (tile, chunk), stable in (i, j) order
    sorted_key, order = torch.sort(key, stable=True)
    global_pos = torch.empty_like(order)
    global_pos[order] = torch.arange(n, device=device, dtype=order.dtype)
    counts_flat = torch.bincount(key, minlength=num_tiles * num_chunks)  # [tile, chunk] flat
    del key
    base_flat = torch.cumsum(counts_flat, 0) - counts_flat
    counts_ct = counts_flat.view(num_tiles, num_chunks).t().contiguous()      # [chunk, tile]
    base = base_flat.view(num_tiles, num_chunks).t().contiguous()             # [chunk, tile]
    off = torch.cumsum(counts_ct, 1) - counts_ct                              # in-chunk
    local = off[chunk_id, tile_id] + (global_pos - base[chunk_id, tile_id])
    del chunk_id
    sign_bit = neg.to(torch.int64) << 15
    src_info = _to_i16(local | sign_bit)
    del local
    ent_info = torch.empty(n, dtype=torch.int16, device=device)
    ent_info[global_pos] = _to_i16(lb | sign_bit)
    del global_pos, sign_bit
    ent_tile = sorted_key // num_chunks
    ent_lb = lb[order]
    del sorted_key, order, lb, tile_id
    key2 = ent_tile * tile + ent_lb
    del ent_tile, ent_lb
    _, perm = torch.sort(key2, stable=True)
    csr = torch.cat([torch.zeros(1, dtype=torch.int64, device=device),
                     torch.cumsum(torch.bincount(key2, minlength=num_tiles * tile), 0)])
    del key2
    seg = torch.cat([torch.zeros(1, dtype=torch.int64, device=device),
                     torch.cumsum(counts_flat.view(num_tiles, num_chunks).sum(1), 0)])
    vals = torch.empty(n, dtype=torch.float32, device=device)
    return [src_info.contiguous(), ent_info, perm.to(torch.int32), csr.to(torch.int32),
            base.to(torch.int32), off.to(torch.int32).contiguous(), seg.to(torch.int32), vals]
