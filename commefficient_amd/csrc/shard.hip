// Sharded FetchSGD server helpers (parallel/server.py sharded sketch path).
//
// With the sketch table reduce-scattered by region group, every rank runs the
// momentum / error feedback, median query and top-k over ITS groups only, so
// each rank's k-list holds coordinates scattered over [0, d) (chunks are dealt
// to groups at random, ops/sketch_region.py).  The lists are all-gathered as
// packed (index << 32 | value bits) words and merged here into ascending index
// order, so the final top-k over the N*k candidates breaks |value| ties by the
// lower index exactly as the replicated unsketch does (bitwise equal results).
//
//   topk_pack     (idx, vals) -> idx << 32 | bits(vals)
//   merge_packed  N lists of k packed words, each ascending by index, disjoint
//                 -> (vals, idx) of all N*k in ascending index order
//                 (merge path: own position + lower_bound in every other list)
//   gather_i64    out[i] = src[pos[i]]
//
// Replaces the reference's single-process unsketch (/root/reference/
// CommEfficient/fed_aggregator.py:584-595) when the server state is sharded.
#include <hip/hip_runtime.h>
#include <cstdint>
#include "kernels.h"

namespace commeff {
namespace {

__global__ void __launch_bounds__(256) topk_pack_kernel(const int64_t* __restrict__ idx,
                                                        const float* __restrict__ vals, int64_t k,
                                                        const int32_t* __restrict__ cmap, int64_t m,
                                                        int64_t* __restrict__ out) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= k) return;
  int64_t g = idx[i];
  if (cmap != nullptr) {
    const int64_t q = g / m;
    g = static_cast<int64_t>(cmap[q]) * m + (g - q * m);
  }
  const uint64_t w = (static_cast<uint64_t>(g) << 32) | __float_as_uint(vals[i]);
  out[i] = static_cast<int64_t>(w);
}

constexpr int kMergeMaxLists = 64;

// NL: compile-time bound on the lists (8: the per-list search state stays in
// registers -- every loop below is unrolled -- for up to 8 ranks)
template <int NL>
__global__ void __launch_bounds__(256) merge_packed_kernel(const int64_t* __restrict__ allp, int nl, int64_t k,
                                                           float* __restrict__ vals, int64_t* __restrict__ idx) {
  const int64_t e = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (e >= nl * k) return;
  const int l = static_cast<int>(e / k);
  const int64_t i = e - static_cast<int64_t>(l) * k;
  const uint64_t v = static_cast<uint64_t>(allp[e]);
  const uint64_t key = v >> 32;
  // lower_bound of key in every other list: the searches of all lists advance
  // together (independent load chains in flight)
  int64_t lo[NL], hi[NL];
#pragma unroll
  for (int q = 0; q < NL; ++q) {
    lo[q] = 0;
    hi[q] = (q == l || q >= nl) ? 0 : k;
  }
  for (int64_t span = k; span > 0; span >>= 1) {
#pragma unroll
    for (int q = 0; q < NL; ++q) {
      if (lo[q] < hi[q]) {
        const int64_t mid = (lo[q] + hi[q]) >> 1;
        const uint64_t x = static_cast<uint64_t>(allp[static_cast<int64_t>(q) * k + mid]) >> 32;
        if (x < key) lo[q] = mid + 1; else hi[q] = mid;
      }
    }
  }
  int64_t pos = i;
#pragma unroll
  for (int q = 0; q < NL; ++q) pos += lo[q];
  vals[pos] = __uint_as_float(static_cast<uint32_t>(v));
  idx[pos] = static_cast<int64_t>(key);
}

__global__ void __launch_bounds__(256) gather_i64_kernel(const int64_t* __restrict__ src,
                                                         const int64_t* __restrict__ pos, int64_t n,
                                                         int64_t* __restrict__ out) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (i < n) out[i] = src[pos[i]];
}

inline dim3 blocks_of(int64_t n) { return dim3(static_cast<uint32_t>((n + 255) / 256)); }

}  // namespace

bool merge_packed_supported(int nl) { return nl >= 1 && nl <= kMergeMaxLists; }

void launch_topk_pack(const int64_t* idx, const float* vals, int64_t k, const int32_t* cmap, int64_t m,
                      int64_t* out, hipStream_t stream) {
  if (k <= 0) return;
  COMMEFF_LAUNCH(topk_pack_kernel, blocks_of(k), dim3(256), 0, stream, idx, vals, k, cmap, m, out);
}

void launch_merge_packed(const int64_t* allp, int nl, int64_t k, float* vals, int64_t* idx, hipStream_t stream) {
  if (nl * k <= 0) return;
  if (nl <= 8)
    COMMEFF_LAUNCH(merge_packed_kernel<8>, blocks_of(nl * k), dim3(256), 0, stream, allp, nl, k, vals, idx);
  else
    COMMEFF_LAUNCH(merge_packed_kernel<kMergeMaxLists>, blocks_of(nl * k), dim3(256), 0, stream, allp, nl, k,
                   vals, idx);
}

void launch_gather_i64(const int64_t* src, const int64_t* pos, int64_t n, int64_t* out, hipStream_t stream) {
  if (n <= 0) return;
  COMMEFF_LAUNCH(gather_i64_kernel, blocks_of(n), dim3(256), 0, stream, src, pos, n, out);
}

}  // namespace commeff
