// Region Count Sketch hash words (csrc/sketch_region.hip, ops/sketch_region.py):
// perm word of (row j, in-chunk offset o) = P_j(o) | S_j(o) << 31; cinfo word of
// (row j, chunk q) = region (bits 0-23) | shift << 24 | sigma << 31.  Shared by
// the region kernels and the fused heavy-hitter zeroing in elementwise.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include "kernels.h"

namespace commeff {
namespace rh {

constexpr uint32_t kSignBit = 0x80000000u;
constexpr uint32_t kRegionMask = 0x00ffffffu;

__device__ __forceinline__ uint32_t ci_region(uint32_t w) { return w & kRegionMask; }
__device__ __forceinline__ uint32_t ci_shift(uint32_t w) { return (w >> 24) & 0x3fu; }

// in-region bucket of lane word pw under chunk word w
__device__ __forceinline__ uint32_t in_region(uint32_t pw, uint32_t w, uint32_t m) {
  uint32_t b = (pw & ~kSignBit) + ci_shift(w);
  return b >= m ? b - m : b;
}
__device__ __forceinline__ bool neg_of(uint32_t pw, uint32_t w) { return ((pw ^ w) & kSignBit) != 0u; }

// Table layout of a region sketch (kernels.h RegionLayout): cell (group grp,
// row j, bucket t of the group) sits at (grp - g0) * gs + j * rs + t for grp in
// [g0, g1).  Row-major [r][c]: gs = g*m, rs = c, g0 = 0.  Group-major [G'][r][g*m]
// (the sharded server, parallel/server.py): gs = r*g*m, rs = g*m, and a rank's
// shard holds groups [g0, g1).
__device__ __forceinline__ size_t cell_at(uint32_t region, uint32_t t, uint32_t j, uint32_t g, uint32_t m,
                                          const RegionLayout& L) {
  const uint32_t grp = region / g;
  return static_cast<size_t>(grp - L.g0) * L.gs + static_cast<size_t>(j) * L.rs + (region - grp * g) * m + t;
}

// table cell (row j) of coordinate i under layout L (cinfo in [row][chunk]
// order); SIZE_MAX when its group is outside [g0, g1)
__device__ __forceinline__ size_t cell_of(uint64_t i, uint32_t j, uint32_t g, uint32_t m, uint32_t nch,
                                          const uint32_t* __restrict__ perm,
                                          const uint32_t* __restrict__ cinfo, const RegionLayout& L) {
  const uint32_t q = static_cast<uint32_t>(i / m), o = static_cast<uint32_t>(i - static_cast<uint64_t>(q) * m);
  const uint32_t cw = cinfo[static_cast<size_t>(j) * nch + q];
  const uint32_t region = ci_region(cw), grp = region / g;
  if (grp < L.g0 || grp >= L.g1) return ~static_cast<size_t>(0);
  return cell_at(region, in_region(perm[j * m + o], cw, m), j, g, m, L);
}

// heavy-hitter zeroing of a region sketch pair (t2 optional), r <= kZeroRows
constexpr int kZeroRows = 8;
struct RegionZero {
  float* t1;
  float* t2;
  const uint32_t* perm;
  const uint32_t* cinfo;
  uint32_t r, g, m, nch;
  uint64_t d;
  RegionLayout L;
};

}  // namespace rh
}  // namespace commeff
