// Region Count Sketch hash words (csrc/sketch_region.hip, ops/sketch_region.py):
// perm word of (row j, in-chunk offset o) = P_j(o) | S_j(o) << 31; cinfo word of
// (row j, chunk q) = region (bits 0-23) | shift << 24 | sigma << 31.  Shared by
// the region kernels and the fused heavy-hitter zeroing in elementwise.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

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

// table cell (row j) of coordinate i; cinfo in [row][chunk] order
__device__ __forceinline__ size_t cell_of(uint64_t i, uint32_t j, uint32_t c, uint32_t m, uint32_t nch,
                                          const uint32_t* __restrict__ perm,
                                          const uint32_t* __restrict__ cinfo) {
  const uint32_t q = static_cast<uint32_t>(i / m), o = static_cast<uint32_t>(i - static_cast<uint64_t>(q) * m);
  const uint32_t cw = cinfo[static_cast<size_t>(j) * nch + q];
  return static_cast<size_t>(j) * c + static_cast<size_t>(ci_region(cw)) * m + in_region(perm[j * m + o], cw, m);
}

// heavy-hitter zeroing of a region sketch pair (t2 optional), r <= kZeroRows
constexpr int kZeroRows = 8;
struct RegionZero {
  float* t1;
  float* t2;
  const uint32_t* perm;
  const uint32_t* cinfo;
  uint32_t r, c, m, nch;
  uint64_t d;
};

}  // namespace rh
}  // namespace commeff
