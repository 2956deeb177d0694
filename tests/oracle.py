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
    """buckets[r,d] int64, signs[r,d] f32 for every coordinate (int64 math)."""
    r = hashes.shape[0]
    i = torch.arange(d, dtype=torch.int64)
    nb = max(1, num_blocks)
    if nb > 1:
        bs = (d + nb - 1) // nb
        blk = i // bs
        t = i - blk * bs
    else:
        t = i
    buckets = torch.empty(r, d, dtype=torch.int64)
    signs = torch.empty(r, d, dtype=torch.float32)
    for j in range(r):
        a, b, c0, c1, c2, c3 = [int(v) for v in hashes[j]]
        x = ((a * t + b) % P) % c
        s = (c3 * t + c2) % P
        s = (s * t + c1) % P
        s = (s * t + c0) % P
        sg = 1.0 - 2.0 * (s & 1).to(torch.float32)
        if nb > 1:
            x = (x + blk_off[j].to(torch.int64)[blk]) % c
            sg = sg * blk_sign[j].to(torch.float32)[blk]
        buckets[j] = x
        signs[j] = sg
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
