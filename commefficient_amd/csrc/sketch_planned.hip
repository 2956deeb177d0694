// "Planned" Count-Sketch encode and query for gfx950: atomic-free and
// bitwise deterministic.
//
// Every hash is data-independent, so the scatter  table[j, h_j(i)] +=
// s_j(i) v_i  (and its transpose, the query gather) is a FIXED sparse
// pattern.  A one-time plan (ops/sketch_plan.py, built with torch sorts on
// the device) lays the r*d entries (i, j) out tile-major -- 8192-bucket table
// tiles, then coordinate chunks, then (i, j) order -- and records:
//   src_info[i*r+j] : u16  LDS staging slot of (i,j) inside its chunk | sign<<15
//   ent_info[e]     : u16  local bucket of entry e inside its tile   | sign<<15
//   perm[x], csr    : entry indices of each tile sorted by local bucket (CSR)
//   base/off [chunk][tile], seg[tile] : run starts (global / in-chunk), tile segments
// Encode  P1 (per chunk):  stage[slot] = +-v_i  (LDS, no atomics), stream the
//                          chunk's per-tile runs out contiguously -> vals[e]
//         P2 (per bucket): table[b] += sum vals[perm[csr[b]..csr[b+1])]
//                          (gathers stay inside one tile's L2-resident segment)
// Query   Q1 (per tile):   vals[e] = +-table[tile, lb(e)]  (tile staged in LDS)
//         Q2 (per chunk):  gather the chunk's runs into LDS, each thread takes
//                          its coordinate's r values from LDS, lower median.
// Replaces LDS/global atomics (measured ~220 us per pass at ResNet-9 size,
// profiles/r1_v2_bench_kernel_stats.txt) and the 33M random table gathers of
// the direct query with coalesced streams.
#include <hip/hip_runtime.h>
#include <cstdint>
#include "kernels.h"

namespace commeff {
namespace {

constexpr int kTileShift = 13;
constexpr uint32_t kTile = 1u << kTileShift;
constexpr int kStageEntries = 8960;

__device__ __forceinline__ float signed_v(float v, uint16_t info) {
  return (info & 0x8000u) ? -v : v;
}

// index of the run (tile) containing in-chunk slot e: largest t with off[t] <= e
__device__ __forceinline__ uint32_t run_of(const uint32_t* off, uint32_t num_tiles, uint32_t e) {
  uint32_t lo = 0, hi = num_tiles;  // invariant: off[lo] <= e
  while (hi - lo > 1) {
    uint32_t mid = (lo + hi) >> 1;
    if (off[mid] <= e) lo = mid; else hi = mid;
  }
  return lo;
}

// ------------------------------------------------------------- encode P1
__global__ void __launch_bounds__(256)
enc_p1_kernel(const float* __restrict__ vec, const float* __restrict__ wvec, float scale,
              float wscale, uint32_t d, uint32_t r, uint32_t chunk, uint32_t num_tiles,
              const uint16_t* __restrict__ src_info, const int32_t* __restrict__ base,
              const int32_t* __restrict__ off, float* __restrict__ vals) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* stage = reinterpret_cast<float*>(smem);
  uint32_t* soff = reinterpret_cast<uint32_t*>(stage + kStageEntries);
  uint32_t* sbase = soff + num_tiles;
  const size_t row = static_cast<size_t>(blockIdx.x) * num_tiles;
  for (uint32_t t = threadIdx.x; t < num_tiles; t += blockDim.x) {
    soff[t] = static_cast<uint32_t>(off[row + t]);
    sbase[t] = static_cast<uint32_t>(base[row + t]);
  }
  const uint32_t i0 = blockIdx.x * chunk;
  const uint32_t i1 = min(d, i0 + chunk);
  for (uint32_t i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
    float v = scale * vec[i];
    if (wvec != nullptr) v += wscale * wvec[i];
    const uint16_t* si = src_info + static_cast<size_t>(i) * r;
    for (uint32_t j = 0; j < r; ++j) {
      const uint16_t info = si[j];
      stage[info & 0x3fffu] = signed_v(v, info);
    }
  }
  __syncthreads();
  const uint32_t total = (i1 - i0) * r;
  for (uint32_t e = threadIdx.x; e < total; e += blockDim.x) {
    const uint32_t t = run_of(soff, num_tiles, e);
    vals[static_cast<size_t>(sbase[t]) + (e - soff[t])] = stage[e];
  }
}

// ------------------------------------------------------------- encode P2
// grid = num_tiles * splits, block 256; each thread owns whole buckets.
__global__ void __launch_bounds__(256)
enc_p2_kernel(float* __restrict__ table, const float* __restrict__ vals,
              const int32_t* __restrict__ perm, const int32_t* __restrict__ csr,
              uint32_t total_buckets, uint32_t splits) {
  const uint32_t t = blockIdx.x / splits;
  const uint32_t s = blockIdx.x - t * splits;
  const uint32_t per = kTile / splits;
  for (uint32_t lb = s * per + threadIdx.x; lb < (s + 1) * per; lb += blockDim.x) {
    const uint32_t gb = (t << kTileShift) + lb;
    if (gb >= total_buckets) break;
    const int32_t a = csr[gb], b = csr[gb + 1];
    float acc = 0.f;
    int32_t x = a;
    for (; x + 3 < b; x += 4) {  // 4 independent gathers in flight
      const float v0 = vals[perm[x]], v1 = vals[perm[x + 1]];
      const float v2 = vals[perm[x + 2]], v3 = vals[perm[x + 3]];
      acc += (v0 + v1) + (v2 + v3);
    }
    for (; x < b; ++x) acc += vals[perm[x]];
    if (b > a) table[gb] += acc;
  }
}

// -------------------------------------------------------------- query Q1
// grid = num_tiles * splits; the tile is staged in LDS, each block converts
// its share of the tile's entries into signed cell values (entry order).
__global__ void __launch_bounds__(256)
qry_q1_kernel(const float* __restrict__ table, const uint16_t* __restrict__ ent_info,
              const int32_t* __restrict__ seg, float* __restrict__ vals,
              uint32_t total_buckets, uint32_t splits) {
  __shared__ float tile[kTile];
  const uint32_t t = blockIdx.x / splits;
  const uint32_t s = blockIdx.x - t * splits;
  const uint32_t tb = t << kTileShift;
  for (uint32_t b = threadIdx.x; b < kTile; b += blockDim.x) {
    const uint32_t gb = tb + b;
    tile[b] = gb < total_buckets ? table[gb] : 0.f;
  }
  __syncthreads();
  const uint32_t lo = static_cast<uint32_t>(seg[t]), hi = static_cast<uint32_t>(seg[t + 1]);
  const uint32_t n = hi - lo;
  const uint32_t e0 = lo + static_cast<uint32_t>(static_cast<uint64_t>(n) * s / splits);
  const uint32_t e1 = lo + static_cast<uint32_t>(static_cast<uint64_t>(n) * (s + 1) / splits);
  for (uint32_t e = e0 + threadIdx.x; e < e1; e += blockDim.x) {
    const uint16_t info = ent_info[e];
    vals[e] = signed_v(tile[info & 0x1fffu], info);
  }
}

// -------------------------------------------------------------- query Q2
template <int R>
__device__ __forceinline__ float lower_median_r(float (&v)[kMaxRows], int r) {
  constexpr int N = R > 0 ? R : kMaxRows;
  if (R == 0) {
#pragma unroll
    for (int q = 0; q < N; ++q)
      if (q >= r) v[q] = __builtin_huge_valf();
  }
#pragma unroll
  for (int pass = 0; pass < N; ++pass) {
#pragma unroll
    for (int q = pass & 1; q + 1 < N; q += 2) {
      float a = v[q], b = v[q + 1];
      v[q] = fminf(a, b);
      v[q + 1] = fmaxf(a, b);
    }
  }
  if (R > 0) return v[(N - 1) / 2];
  const int m = (r - 1) / 2;
  float res = v[0];
#pragma unroll
  for (int q = 0; q < N; ++q)
    if (q == m) res = v[q];
  return res;
}

template <int R>
__global__ void __launch_bounds__(256)
qry_q2_kernel(const float* __restrict__ vals, uint32_t d, uint32_t r, uint32_t chunk,
              uint32_t num_tiles, const uint16_t* __restrict__ src_info,
              const int32_t* __restrict__ base, const int32_t* __restrict__ off,
              float* __restrict__ est) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* stage = reinterpret_cast<float*>(smem);
  uint32_t* soff = reinterpret_cast<uint32_t*>(stage + kStageEntries);
  uint32_t* sbase = soff + num_tiles;
  const size_t row = static_cast<size_t>(blockIdx.x) * num_tiles;
  for (uint32_t t = threadIdx.x; t < num_tiles; t += blockDim.x) {
    soff[t] = static_cast<uint32_t>(off[row + t]);
    sbase[t] = static_cast<uint32_t>(base[row + t]);
  }
  __syncthreads();
  const uint32_t i0 = blockIdx.x * chunk;
  const uint32_t i1 = min(d, i0 + chunk);
  const uint32_t total = (i1 - i0) * r;
  for (uint32_t e = threadIdx.x; e < total; e += blockDim.x) {
    const uint32_t t = run_of(soff, num_tiles, e);
    stage[e] = vals[static_cast<size_t>(sbase[t]) + (e - soff[t])];
  }
  __syncthreads();
  for (uint32_t i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
    float v[kMaxRows];
    const uint16_t* si = src_info + static_cast<size_t>(i) * r;
    const int rr = R > 0 ? R : static_cast<int>(r);
#pragma unroll
    for (int j = 0; j < (R > 0 ? R : kMaxRows); ++j) {
      v[j] = 0.f;
      if (j < rr) v[j] = stage[si[j] & 0x3fffu];
    }
    est[i] = lower_median_r<R>(v, rr);
  }
}

// ---------------------------------------------------------------- hashes
// bucket|neg<<31 for every (i, j), laid out [d, r] (src order), for the plan
__global__ void __launch_bounds__(256)
hash_all_kernel(RowHashes h, SketchGeom g, const int32_t* __restrict__ blk_off,
                const float* __restrict__ blk_sign, int32_t* __restrict__ out) {
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < g.d; i += stride) {
    uint32_t blk, t;
    split_block(i, g, &blk, &t);
    for (uint32_t j = 0; j < g.r; ++j) {
      uint32_t bk;
      float s;
      hash_t(h.row[j], t, blk, g, blk_off + j * g.num_blocks, blk_sign + j * g.num_blocks, &bk,
             &s);
      out[static_cast<size_t>(i) * g.r + j] =
          static_cast<int32_t>(bk | (s < 0.f ? 0x80000000u : 0u));
    }
  }
}

size_t stage_lds(uint32_t num_tiles) {
  return kStageEntries * sizeof(float) + 2 * num_tiles * sizeof(uint32_t);
}

void set_lds_attr(const void* fn) {
  (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
}

}  // namespace

void launch_cs_hash_all(const RowHashes& h, const SketchGeom& g, const int32_t* blk_off,
                        const float* blk_sign, int32_t* out, hipStream_t stream) {
  if (g.d == 0) return;
  int64_t blocks = (static_cast<int64_t>(g.d) + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(hash_all_kernel, dim3(static_cast<uint32_t>(blocks)), dim3(256), 0, stream,
                     h, g, blk_off, blk_sign, out);
}

void launch_cs_encode_planned(float* table, const float* vec, const float* wvec, float scale,
                              float wscale, const SketchGeom& g, const BinPlan& p,
                              const PlannedArgs& a, hipStream_t stream) {
  if (g.d == 0) return;
  static bool attr = false;
  if (!attr) {
    set_lds_attr(reinterpret_cast<const void*>(enc_p1_kernel));
    attr = true;
  }
  const uint32_t nt = static_cast<uint32_t>(p.num_tiles);
  hipLaunchKernelGGL(enc_p1_kernel, dim3(static_cast<uint32_t>(p.num_chunks)), dim3(256),
                     stage_lds(nt), stream, vec, wvec, scale, wscale, g.d, g.r,
                     static_cast<uint32_t>(p.chunk), nt, a.src_info, a.base, a.off, a.vals);
  const uint32_t splits = 8;  // 1024 buckets per block, 4 per thread
  hipLaunchKernelGGL(enc_p2_kernel, dim3(nt * splits), dim3(256), 0, stream, table, a.vals,
                     a.perm, a.csr, static_cast<uint32_t>(static_cast<int64_t>(g.r) * g.c),
                     splits);
}

void launch_cs_query_planned(const float* table, float* est, const SketchGeom& g,
                             const BinPlan& p, const PlannedArgs& a, hipStream_t stream) {
  if (g.d == 0) return;
  static bool attr = false;
  const uint32_t nt = static_cast<uint32_t>(p.num_tiles);
  const uint32_t splits = 4;
  hipLaunchKernelGGL(qry_q1_kernel, dim3(nt * splits), dim3(256), 0, stream, table, a.ent_info,
                     a.seg, a.vals, static_cast<uint32_t>(static_cast<int64_t>(g.r) * g.c),
                     splits);
  const dim3 grid(static_cast<uint32_t>(p.num_chunks));
  const size_t lds = stage_lds(nt);
  const uint32_t ch = static_cast<uint32_t>(p.chunk);
  if (!attr) {
    set_lds_attr(reinterpret_cast<const void*>(qry_q2_kernel<5>));
    set_lds_attr(reinterpret_cast<const void*>(qry_q2_kernel<3>));
    set_lds_attr(reinterpret_cast<const void*>(qry_q2_kernel<1>));
    set_lds_attr(reinterpret_cast<const void*>(qry_q2_kernel<0>));
    attr = true;
  }
  switch (g.r) {
    case 5: hipLaunchKernelGGL(qry_q2_kernel<5>, grid, dim3(256), lds, stream, a.vals, g.d, g.r, ch, nt, a.src_info, a.base, a.off, est); break;
    case 3: hipLaunchKernelGGL(qry_q2_kernel<3>, grid, dim3(256), lds, stream, a.vals, g.d, g.r, ch, nt, a.src_info, a.base, a.off, est); break;
    case 1: hipLaunchKernelGGL(qry_q2_kernel<1>, grid, dim3(256), lds, stream, a.vals, g.d, g.r, ch, nt, a.src_info, a.base, a.off, est); break;
    default: hipLaunchKernelGGL(qry_q2_kernel<0>, grid, dim3(256), lds, stream, a.vals, g.d, g.r, ch, nt, a.src_info, a.base, a.off, est); break;
  }
}

}  // namespace commeff
