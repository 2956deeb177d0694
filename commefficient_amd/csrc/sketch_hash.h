// Count-Sketch hash family shared by the HIP kernels (device) and the CPU
// kernels (host).  One definition so that a table built on the GPU and one
// built on the CPU with the same seed are identical up to fp32 summation order.
//
// Semantics follow the CSVec used by the reference (SURVEY.md §2.4 X1;
// call sites /root/reference/CommEfficient/fed_worker.py:313-320 and
// fed_aggregator.py:464-467,584-595):
//   * bucket hash: 2-wise independent  ((a*t + b) mod P) mod c
//   * sign hash:   4-wise independent  ((c3 t^3 + c2 t^2 + c1 t + c0) mod P) & 1
//   * P = 2^31 - 1 (Mersenne), so every product of two residues fits a u64.
//   * numBlocks > 1: coordinate i = blk * blockSize + t reuses the hashes of t
//     with a per-(row, block) bucket offset and sign flip.
// Unlike CSVec nothing is materialised: hashes are recomputed on the fly, so
// a GPT-2 sized vector (124M coords) needs no r x d index tables.
//
// Integer division/modulo by the runtime constants c and blockSize uses
// Lemire's 64-bit multiply-high reciprocal (no hardware integer divide on
// CDNA: a u32 `%` is ~40 VALU ops, this is ~6).
#pragma once
#include <cstdint>

#if defined(__HIPCC__)
#define CE_HD __host__ __device__ __forceinline__
#else
#define CE_HD inline
#endif

namespace commeff {

constexpr uint64_t kMersenneP = (1ull << 31) - 1;
// per-row parameter layout in the int64 `hashes` tensor [r, kHashParams]
constexpr int kHashParams = 6;  // a, b, c0, c1, c2, c3

CE_HD uint64_t mul64hi(uint64_t a, uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __umul64hi(a, b);
#else
  return static_cast<uint64_t>((static_cast<unsigned __int128>(a) * b) >> 64);
#endif
}

// Reciprocal for x / d and x % d with x, d < 2^32, d >= 1.
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
CE_HD uint32_t fmod(uint32_t x, const FastDivU32& f) {
  return f.d <= 1 ? 0u : static_cast<uint32_t>(mul64hi(f.M * x, f.d));
}

CE_HD uint64_t mod_p(uint64_t x) {
  // x < 2^62  ->  result in [0, P)
  x = (x & kMersenneP) + (x >> 31);
  x = (x & kMersenneP) + (x >> 31);
  return x >= kMersenneP ? x - kMersenneP : x;
}

struct RowHash {
  uint32_t a, b, c0, c1, c2, c3;
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
  FastDivU32 div_c;
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
  g.div_c = make_fastdiv(c);
  g.div_bs = make_fastdiv(bs);
  return g;
}

// Full hash of coordinate i for one row.
//   blk_off / blk_sign: per-row arrays of length num_blocks (unused if 1 block)
CE_HD void hash_coord(const RowHash& h, uint32_t i, const SketchGeom& g,
                      const int32_t* blk_off, const float* blk_sign,
                      uint32_t* bucket, float* sign) {
  uint32_t blk = 0, t = i;
  if (g.num_blocks > 1) {
    blk = fdiv(i, g.div_bs);
    t = i - blk * g.div_bs.d;
  }
  // bucket: ((a t + b) mod P) mod c
  uint32_t x = static_cast<uint32_t>(mod_p(static_cast<uint64_t>(h.a) * t + h.b));
  uint32_t bk = fmod(x, g.div_c);
  // sign: Horner over the cubic, mod P
  uint64_t s = mod_p(static_cast<uint64_t>(h.c3) * t + h.c2);
  s = mod_p(s * t + h.c1);
  s = mod_p(s * t + h.c0);
  float sg = (s & 1u) ? -1.f : 1.f;
  if (g.num_blocks > 1) {
    bk += static_cast<uint32_t>(blk_off[blk]);  // blk_off in [0, c)
    if (bk >= g.c) bk -= g.c;
    sg *= blk_sign[blk];
  }
  *bucket = bk;
  *sign = sg;
}

}  // namespace commeff
