// Count-Sketch hash family shared by the HIP kernels (device) and the CPU
// kernels (host).  One definition so that a table built on the GPU and one
// built on the CPU with the same seed are identical up to fp32 summation order.
//
// Semantics follow the CSVec used by the reference (SURVEY.md §2.4 X1;
// call sites /root/reference/CommEfficient/fed_worker.py:313-320 and
// fed_aggregator.py:464-467,584-595): each row j has a bucket hash
// h_j: [d] -> [c] and a sign hash s_j: [d] -> {-1,+1}; with numBlocks > 1
// coordinate i = blk * blockSize + t reuses the hashes of t with a per-(row,
// block) bucket offset and sign flip.
//
// Family (MI355X-first choice): Dietzfelbinger multiply-add-shift on 64-bit
// words -- strongly 2-universal for the top 32 bits of (a*t + b) mod 2^64 --
// mapped to [0, c) with a multiply-high ("fastrange"), and the sign is the top
// bit of an independent (a', b') pair.  Pairwise independence of buckets and
// signs is what the Count Sketch unbiasedness/variance bounds use.  Cost: ~10
// VALU ops per (coordinate, row) instead of ~100 for polynomials mod a
// Mersenne prime (the first version of this file; measured 3x slower encode
// and query on MI355X, profiles/r1_v1_bench_kernel_stats.txt).  Nothing is
// materialised: no r x d index tables, so a 124M-coordinate GPT-2 gradient
// needs no extra memory.
#pragma once
#include <cstdint>

#if defined(__HIPCC__)
#define CE_HD __host__ __device__ __forceinline__
#else
#define CE_HD inline
#endif

namespace commeff {

// per-row parameter layout in the int64 `hashes` tensor [r, kHashParams]
// (bit patterns of u64): bucket (a, b), sign (a2, b2); a and a2 are odd.
constexpr int kHashParams = 4;

CE_HD uint64_t mul64hi(uint64_t a, uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __umul64hi(a, b);
#else
  return static_cast<uint64_t>((static_cast<unsigned __int128>(a) * b) >> 64);
#endif
}

// Reciprocal for x / d with x, d < 2^32, d >= 1 (Lemire): no hardware integer
// divide on CDNA, a u32 `/` is ~40 VALU ops, this is ~4.
struct FastDivU32 {
  uint64_t M;
  uint32_t d;
};
inline FastDivU32 make_fastdiv(uint32_t d) {
  FastDivU32 f;
  f.d = d;
  f.M = d <= 1 ? 0 : (~0ull) / d + 1;
  return f;
}
CE_HD uint32_t fdiv(uint32_t x, const FastDivU32& f) {
  return f.d <= 1 ? x : static_cast<uint32_t>(mul64hi(f.M, x));
}

struct RowHash {
  uint64_t a, b, a2, b2;
};

constexpr int kMaxRows = 16;

struct RowHashes {
  RowHash row[kMaxRows];
};

// Geometry shared by every kernel that hashes coordinates.
struct SketchGeom {
  uint32_t d;          // vector length
  uint32_t r;          // rows
  uint32_t c;          // columns (buckets per row)
  uint32_t num_blocks; // CSVec numBlocks
  FastDivU32 div_bs;   // block size = ceil(d / num_blocks)
};

inline SketchGeom make_geom(uint32_t d, uint32_t r, uint32_t c, uint32_t nb) {
  SketchGeom g;
  g.d = d;
  g.r = r;
  g.c = c;
  g.num_blocks = nb < 1 ? 1 : nb;
  uint32_t bs = (d + g.num_blocks - 1) / g.num_blocks;
  if (bs == 0) bs = 1;
  g.div_bs = make_fastdiv(bs);
  return g;
}

// Bijective 32-bit mixer (murmur3 finaliser: xor-shifts and odd multiplies
// are invertible).  Applied to the in-block coordinate before the universal
// hash: injectivity keeps the family pairwise independent, and it breaks the
// arithmetic progression that multiply-shift maps consecutive keys onto --
// consecutive lanes then hit pseudo-random table cells (no HBM-channel or LDS
// bank camping).  Computed once per coordinate, shared by all rows.
CE_HD uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x85ebca6bu;
  x ^= x >> 13;
  x *= 0xc2b2ae35u;
  x ^= x >> 16;
  return x;
}

// block index / mixed in-block key (shared by all rows of one coordinate)
CE_HD void split_block(uint32_t i, const SketchGeom& g, uint32_t* blk, uint32_t* t) {
  uint32_t tt = i;
  *blk = 0;
  if (g.num_blocks > 1) {
    *blk = fdiv(i, g.div_bs);
    tt = i - *blk * g.div_bs.d;
  }
  *t = mix32(tt);
}

// hash of the in-block coordinate t for one row (+ block offset / sign)
CE_HD void hash_t(const RowHash& h, uint32_t t, uint32_t blk, const SketchGeom& g,
                  const int32_t* blk_off, const float* blk_sign, uint32_t* bucket,
                  float* sign) {
  const uint64_t x = h.a * t + h.b;  // mod 2^64
  uint32_t bk = static_cast<uint32_t>(((x >> 32) * static_cast<uint64_t>(g.c)) >> 32);
  const uint64_t y = h.a2 * t + h.b2;
  float sg = (y >> 63) ? -1.f : 1.f;
  if (g.num_blocks > 1) {
    bk += static_cast<uint32_t>(blk_off[blk]);  // blk_off in [0, c)
    if (bk >= g.c) bk -= g.c;
    sg *= blk_sign[blk];
  }
  *bucket = bk;
  *sign = sg;
}

// Full hash of coordinate i for one row.
CE_HD void hash_coord(const RowHash& h, uint32_t i, const SketchGeom& g,
                      const int32_t* blk_off, const float* blk_sign, uint32_t* bucket,
                      float* sign) {
  uint32_t blk, t;
  split_block(i, g, &blk, &t);
  hash_t(h, t, blk, g, blk_off, blk_sign, bucket, sign);
}

}  // namespace commeff
