// Region-permutation Count Sketch for gfx950: encode, median query and
// heavy-hitter zeroing with no plan arrays, no atomics and no r*d
// intermediate.  Bitwise deterministic.
//
// Hash family (ops/sketch_region.py builds the parameters from the seed):
// the d coordinates are cut into chunks of m consecutive coordinates and each
// table row into R regions of m buckets (R = c // m; the <= R - 1 leftover
// buckets of a row are never used).  In row j, chunk q goes to region
// rho_j(q) (chunks dealt evenly over the regions in a random order) and its
// coordinate o lands on bucket
//     rho_j(q) * m + (P_j(o) + shift_j(q)) mod m,   sign S_j(o) ^ sigma_j(q)
// with P_j a random permutation of [m].  Inside one chunk the map is a
// bijection (chunk-mates never collide); two coordinates of different chunks
// collide with probability (1/R) * (1/m) ~= 1/c per row, independently per
// row -- the pairwise behaviour the Count-Sketch estimates rest on, with each
// bucket receiving exactly one coordinate from each chunk of its region.
// This replaces the reference CSVec's hashed numBlocks layout
// (/root/reference/CommEfficient/fed_aggregator.py:464-467 builds the CSVec,
// fed_worker.py:313-320 encodes, fed_aggregator.py:584-595 unsketches): the
// per-chunk structure turns the encode scatter and the query gather into
// region-local LDS work.
//
// Encode (block per (region, row), W waves): each wave owns an LDS copy of
// the region and adds its share of the region's chunks into it -- within a
// chunk every lane writes a distinct bucket, and a wave's LDS accesses are
// processed in order, so plain read-add-write needs no atomics or barriers;
// the W copies are summed in a fixed order into the table.
// Query (block per chunk): the chunk's r regions -> LDS (r * m floats, 16-byte
// loads), then every coordinate gathers its r signed cells and stores the
// lower median.
#include <hip/hip_runtime.h>
#include <cstdint>
#include "kernels.h"

namespace commeff {
namespace {

constexpr uint32_t kSignBit = 0x80000000u;

// (per-coordinate permutation word, chunk shift word) -> in-region bucket, negate?
__device__ __forceinline__ uint32_t region_bucket(uint32_t pw, uint32_t shift, uint32_t m) {
  uint32_t b = (pw & ~kSignBit) + (shift & ~kSignBit);
  return b >= m ? b - m : b;
}
__device__ __forceinline__ bool region_neg(uint32_t pw, uint32_t shift) {
  return ((pw ^ shift) & kSignBit) != 0u;
}

template <int W>
__global__ void __launch_bounds__(W * 64)
cs_region_encode_kernel(float* __restrict__ table, const float* __restrict__ vec,
                        const float* __restrict__ wvec, float scale, float wscale, uint32_t d,
                        uint32_t c, uint32_t m, uint32_t R, uint32_t nch,
                        const uint32_t* __restrict__ perm, const uint2* __restrict__ cinfo,
                        const int32_t* __restrict__ lists, const int32_t* __restrict__ offs,
                        int overwrite) {
  extern __shared__ __attribute__((aligned(16))) float acc[];  // [W][m]
  const uint32_t rho = blockIdx.x, j = blockIdx.y;
  const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (uint32_t e = tid; e < W * m; e += W * 64) acc[e] = 0.f;
  __syncthreads();
  float* mine = acc + w * m;
  const uint32_t* pj = perm + static_cast<size_t>(j) * m;
  const int32_t* lj = lists + static_cast<size_t>(j) * nch;
  const int32_t l0 = offs[j * (R + 1) + rho], l1 = offs[j * (R + 1) + rho + 1];
  constexpr uint32_t U = 8;  // elements per lane in flight
  for (int32_t li = l0 + static_cast<int32_t>(w); li < l1; li += W) {
    const uint32_t q = static_cast<uint32_t>(lj[li]);
    const uint32_t shift = cinfo[static_cast<size_t>(j) * nch + q].y;
    const size_t i0 = static_cast<size_t>(q) * m;
    const uint32_t len = min(m, d - static_cast<uint32_t>(i0));
    for (uint32_t ob = lane; ob < len; ob += 64 * U) {
      float v[U];
      uint32_t pw[U];
#pragma unroll
      for (uint32_t u = 0; u < U; ++u) {
        const uint32_t o = ob + 64 * u;
        v[u] = 0.f;
        pw[u] = 0u;
        if (o < len) {
          v[u] = scale * vec[i0 + o];
          if (wvec != nullptr) v[u] += wscale * wvec[i0 + o];
          pw[u] = pj[o];
        }
      }
#pragma unroll
      for (uint32_t u = 0; u < U; ++u) {
        if (ob + 64 * u < len) {
          const uint32_t b = region_bucket(pw[u], shift, m);
          mine[b] += region_neg(pw[u], shift) ? -v[u] : v[u];
        }
      }
    }
  }
  __syncthreads();
  float* trow = table + static_cast<size_t>(j) * c;
  const uint32_t base = rho * m;
  for (uint32_t e = tid; e < m; e += W * 64) {
    float s = acc[e];
#pragma unroll
    for (int k = 1; k < W; ++k) s += acc[k * m + e];  // fixed order
    trow[base + e] = overwrite ? s : trow[base + e] + s;
  }
  if (overwrite && rho == 0)  // the unused buckets past R*m stay zero
    for (uint32_t e = R * m + tid; e < c; e += W * 64) trow[e] = 0.f;
}

template <int RT>
__device__ __forceinline__ float lower_median(float (&v)[kMaxRows], int r) {
  constexpr int N = RT > 0 ? RT : kMaxRows;
  if (RT == 0) {
#pragma unroll
    for (int q = 0; q < N; ++q)
      if (q >= r) v[q] = __builtin_huge_valf();
  }
#pragma unroll
  for (int pass = 0; pass < N; ++pass) {
#pragma unroll
    for (int q = pass & 1; q + 1 < N; q += 2) {
      const float a = v[q], b = v[q + 1];
      v[q] = fminf(a, b);
      v[q + 1] = fmaxf(a, b);
    }
  }
  if (RT > 0) return v[(N - 1) / 2];
  const int mid = (r - 1) / 2;
  float res = v[0];
#pragma unroll
  for (int q = 0; q < N; ++q)
    if (q == mid) res = v[q];
  return res;
}

template <int RT>
__global__ void __launch_bounds__(256)
cs_region_query_kernel(const float* __restrict__ table, float* __restrict__ est, uint32_t d,
                       uint32_t c, uint32_t m, uint32_t nch, uint32_t r_rt,
                       const uint32_t* __restrict__ perm, const uint2* __restrict__ cinfo,
                       uint32_t q0, int vec4) {
  extern __shared__ __attribute__((aligned(16))) float reg[];  // [r][m]
  const uint32_t r = RT > 0 ? static_cast<uint32_t>(RT) : r_rt;
  const uint32_t q = q0 + blockIdx.x;
  const uint32_t tid = threadIdx.x;
  __shared__ uint32_t sh[kMaxRows];
  if (tid < r) sh[tid] = cinfo[static_cast<size_t>(tid) * nch + q].y;
  // stage the chunk's region of every row (coalesced; 16-byte when aligned)
  for (uint32_t j = 0; j < r; ++j) {
    const uint32_t base = cinfo[static_cast<size_t>(j) * nch + q].x;
    const float* src = table + static_cast<size_t>(j) * c + base;
    float* dst = reg + j * m;
    if (vec4) {
      const float4* s4 = reinterpret_cast<const float4*>(src);
      float4* d4 = reinterpret_cast<float4*>(dst);
      for (uint32_t e = tid; e < (m >> 2); e += 256) d4[e] = s4[e];
    } else {
      for (uint32_t e = tid; e < m; e += 256) dst[e] = src[e];
    }
  }
  __syncthreads();
  const size_t i0 = static_cast<size_t>(q) * m;
  const uint32_t len = min(m, d - static_cast<uint32_t>(i0));
  const int rr = static_cast<int>(r);
  for (uint32_t o = tid; o < len; o += 256) {
    float v[kMaxRows];
    uint32_t pw[kMaxRows];
#pragma unroll
    for (int j = 0; j < (RT > 0 ? RT : kMaxRows); ++j) pw[j] = j < rr ? perm[static_cast<size_t>(j) * m + o] : 0u;
#pragma unroll
    for (int j = 0; j < (RT > 0 ? RT : kMaxRows); ++j) {
      v[j] = 0.f;
      if (j < rr) {
        const float x = reg[j * m + region_bucket(pw[j], sh[j], m)];
        v[j] = region_neg(pw[j], sh[j]) ? -x : x;
      }
    }
    est[i0 + o] = lower_median<RT>(v, rr);
  }
}

// zero cells (j, bucket_j(idx[t])) of t1 (and t2) where vals[t] != 0 (or always)
__global__ void __launch_bounds__(256)
cs_region_zero_kernel(float* __restrict__ t1, float* __restrict__ t2, const int64_t* __restrict__ idx,
                      const float* __restrict__ vals, int64_t k, uint64_t d, uint32_t r, uint32_t c,
                      uint32_t m, uint32_t nch, const uint32_t* __restrict__ perm,
                      const uint2* __restrict__ cinfo) {
  const int64_t e = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (e >= k * r) return;
  const int64_t t = e / r;
  const uint32_t j = static_cast<uint32_t>(e - t * r);
  if (vals != nullptr && vals[t] == 0.f) return;
  const uint64_t i = static_cast<uint64_t>(idx[t]);
  if (i >= d) return;  // (top-k indices are always in range)
  const uint32_t q = static_cast<uint32_t>(i / m), o = static_cast<uint32_t>(i - static_cast<uint64_t>(q) * m);
  const uint2 ci = cinfo[static_cast<size_t>(j) * nch + q];
  const size_t cell = static_cast<size_t>(j) * c + ci.x + region_bucket(perm[static_cast<size_t>(j) * m + o], ci.y, m);
  t1[cell] = 0.f;
  if (t2 != nullptr) t2[cell] = 0.f;
}

template <typename F>
void set_lds_once(F* fn, int bytes, int* done) {
  if (*done < bytes) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(fn),
                              hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    *done = bytes;
  }
}

}  // namespace

int region_encode_waves(int64_t m) {
  // W LDS copies of the region: 8 waves while they fit 2 blocks per CU
  return m * 4 * 8 <= 80 * 1024 ? 8 : (m * 4 * 4 <= 160 * 1024 ? 4 : (m * 4 * 2 <= 160 * 1024 ? 2 : 0));
}

void launch_cs_region_encode(float* table, const float* vec, const float* wvec, float scale,
                             float wscale, int64_t d, int r, int64_t c, int64_t m, int64_t R,
                             int64_t nch, const uint32_t* perm, const int32_t* cinfo,
                             const int32_t* lists, const int32_t* offs, bool overwrite,
                             hipStream_t stream) {
  const int W = region_encode_waves(m);
  const int lds = static_cast<int>(W * m * 4);
  const dim3 grid(static_cast<uint32_t>(R), static_cast<uint32_t>(r));
  const uint2* ci = reinterpret_cast<const uint2*>(cinfo);
#define COMMEFF_REGION_ENC(WW)                                                                       \
  do {                                                                                                \
    static int done = 0;                                                                              \
    set_lds_once(cs_region_encode_kernel<WW>, lds, &done);                                            \
    hipLaunchKernelGGL(cs_region_encode_kernel<WW>, grid, dim3(WW * 64), lds, stream, table, vec, wvec, \
                       scale, wscale, static_cast<uint32_t>(d), static_cast<uint32_t>(c),             \
                       static_cast<uint32_t>(m), static_cast<uint32_t>(R), static_cast<uint32_t>(nch), \
                       perm, ci, lists, offs, overwrite ? 1 : 0);                                     \
  } while (0)
  if (W == 8) COMMEFF_REGION_ENC(8);
  else if (W == 4) COMMEFF_REGION_ENC(4);
  else COMMEFF_REGION_ENC(2);
#undef COMMEFF_REGION_ENC
}

void launch_cs_region_query(const float* table, float* est, int64_t d, int r, int64_t c, int64_t m,
                            int64_t nch, const uint32_t* perm, const int32_t* cinfo, int64_t q0,
                            int64_t q1, hipStream_t stream) {
  if (q1 <= q0) return;
  const int lds = static_cast<int>(r * m * 4);
  const int vec4 = (m % 4 == 0 && c % 4 == 0) ? 1 : 0;
  const uint2* ci = reinterpret_cast<const uint2*>(cinfo);
  const dim3 grid(static_cast<uint32_t>(q1 - q0));
  if (r == 5) {
    static int done = 0;
    set_lds_once(cs_region_query_kernel<5>, lds, &done);
    hipLaunchKernelGGL(cs_region_query_kernel<5>, grid, dim3(256), lds, stream, table, est,
                       static_cast<uint32_t>(d), static_cast<uint32_t>(c), static_cast<uint32_t>(m),
                       static_cast<uint32_t>(nch), 5u, perm, ci, static_cast<uint32_t>(q0), vec4);
  } else {
    static int done = 0;
    set_lds_once(cs_region_query_kernel<0>, lds, &done);
    hipLaunchKernelGGL(cs_region_query_kernel<0>, grid, dim3(256), lds, stream, table, est,
                       static_cast<uint32_t>(d), static_cast<uint32_t>(c), static_cast<uint32_t>(m),
                       static_cast<uint32_t>(nch), static_cast<uint32_t>(r), perm, ci,
                       static_cast<uint32_t>(q0), vec4);
  }
}

void launch_cs_region_zero(float* t1, float* t2, const int64_t* idx, const float* vals, int64_t k,
                           int64_t d, int r, int64_t c, int64_t m, int64_t nch, const uint32_t* perm,
                           const int32_t* cinfo, hipStream_t stream) {
  const int64_t n = k * r;
  if (n <= 0) return;
  hipLaunchKernelGGL(cs_region_zero_kernel, dim3(static_cast<uint32_t>((n + 255) / 256)), dim3(256), 0,
                     stream, t1, t2, idx, vals, k, static_cast<uint64_t>(d), static_cast<uint32_t>(r), static_cast<uint32_t>(c),
                     static_cast<uint32_t>(m), static_cast<uint32_t>(nch), perm,
                     reinterpret_cast<const uint2*>(cinfo));
}

}  // namespace commeff
