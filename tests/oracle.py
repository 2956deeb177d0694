"""Pure-PyTorch fp32/fp64 reference implementations used ONLY as test oracles.

They restate the math of the reference's codecs (CSVec semantics, SURVEY.md
§2.4 X1; ``_topk`` /root/reference/CommEfficient/utils.py:232-252; server
helpers fed_aggregator.py:483-613) with plain torch ops, with our hash family
(sketch_hash.h) so tables can be compared cell by cell.
"""
from __future__ import annotations

import torch

P = (1 << 31) - 1


def hash_coords(hashes, blk_off, blk_sign, d, c, num_blocks):
    """buckets[r,d] int64, signs[r,d] f32 for every coordinate (numpy u64 math,
    the multiply-add-shift family of csrc/sketch_hash.h)."""
    import numpy as np
    r = hashes.shape[0]
    i = np.arange(d, dtype=np.uint64)
    nb = max(1, num_blocks)
    if nb > 1:
        bs = np.uint64((d + nb - 1) // nb)
        blk = (i // bs).astype(np.int64)
        t = i - blk.astype(np.uint64) * bs
    else:
        blk = np.zeros(d, np.int64)
        t = i
    # murmur3 finaliser on u32 (sketch_hash.h mix32)
    x = t.astype(np.uint32)
    with np.errstate(over="ignore"):
        x ^= x >> np.uint32(16)
        x *= np.uint32(0x85ebca6b)
        x ^= x >> np.uint32(13)
        x *= np.uint32(0xc2b2ae35)
        x ^= x >> np.uint32(16)
    t = x.astype(np.uint64)
    H = hashes.numpy().view(np.uint64)
    buckets = torch.empty(r, d, dtype=torch.int64)
    signs = torch.empty(r, d, dtype=torch.float32)
    with np.errstate(over="ignore"):
        for j in range(r):
            a, b, a2, b2 = H[j, 0] | np.uint64(1), H[j, 1], H[j, 2] | np.uint64(1), H[j, 3]
            x = a * t + b
            bk = ((x >> np.uint64(32)) * np.uint64(c)) >> np.uint64(32)
            y = a2 * t + b2
            sg = np.where((y >> np.uint64(63)) == 1, -1.0, 1.0).astype(np.float32)
            bk = bk.astype(np.int64)
            if nb > 1:
                bk = (bk + blk_off[j].numpy().astype(np.int64)[blk]) % c
                sg = sg * blk_sign[j].numpy()[blk]
            buckets[j] = torch.from_numpy(bk)
            signs[j] = torch.from_numpy(sg)
    return buckets, signs


class OracleSketch:
    def __init__(self, hashes, blk_off, blk_sign, d, c, r, num_blocks):
        self.d, self.c, self.r = d, c, r
        self.buckets, self.signs = hash_coords(hashes, blk_off, blk_sign, d, c, num_blocks)
        self.table = torch.zeros(r, c, dtype=torch.float64)

    def accumulate_vec(self, vec):
        vec = vec.to(torch.float64).cpu()
        for j in range(self.r):
            self.table[j].index_add_(0, self.buckets[j], self.signs[j].double() * vec)

    def query(self):
        vals = torch.stack([self.signs[j].double() * self.table[j][self.buckets[j]]
                            for j in range(self.r)])
        # torch.median returns the lower median, like CSVec
        return vals.median(dim=0).values

    def l2estimate(self):
        return (self.table ** 2).sum(dim=1).median().sqrt()


def topk_oracle(x, k):
    """k largest |x| with ties broken by lower index; ascending index output."""
    x = x.cpu()
    key = x.view(torch.int32) & 0x7fffffff
    n = x.numel()
    k = min(k, n)
    order = sorted(range(n), key=lambda i: (-int(key[i]), i))[:k]
    idx = torch.tensor(sorted(order), dtype=torch.int64)
    return idx, x[idx]
