// "Planned" Count-Sketch encode and query for gfx950: no atomics anywhere,
// bitwise deterministic, every global access a coalesced stream or a short
// contiguous run.
//
// The hashes are data-independent, so the scatter table[j, h_j(i)] +=
// s_j(i) v_i (and its transpose, the query gather) is a FIXED sparse pattern.
// A one-time plan (ops/sketch_plan.py, built with device sorts) lays the r*d
// entries (i, j) out tile-major -- T-bucket table tiles (T = 512..4096), then
// coordinate chunks, then (i, j) order -- so that
//   * a coordinate chunk's entries for one tile are a contiguous RUN of the
//     tile's segment (runs of ~30 entries), and
//   * a tile's whole segment (<= 32767 entries) fits in LDS.
// Plan arrays:
//   src_info[i*r+j] u16  slot of entry (i,j) in its chunk's LDS stage
//   ent_info[e]     u16  in-tile bucket of entry e | sign << 15 (entry order)
//   perm[cm]        u16  at an entry's chunk-major position (P1's output):
//                        its segment-local bucket-order index | sign << 15
//   csr[gb]         i32  bucket start in perm (global bucket gb = j*c + h)
//   base/off        i32  run starts per (chunk, tile): global / in-chunk
//   seg[t]          i32  tile segment starts
//   p2_src/p2_pos   i32  the same runs, tile-major (for encode P2)
//   vals            f32  d*r scratch shared by encode and query
// Encode  P1 (block per chunk): stage[slot] = v_i (LDS, no atomics); the
//            stage (tile-ordered inside the chunk) is written out chunk-major
//            with full-line stores
//         P2 (block per tile):  gather the tile's run of every chunk and
//            scatter each value (signed) to its bucket-order LDS slot;
//            lane per bucket sums its contiguous range; table tile += sums
// Query   Q1 (block per tile):  tile -> LDS; vals[e] = +-tile[lb(e)]
//         Q2 (block per chunk): runs -> LDS stage; per coordinate the
//            lower median of its r staged values
// Every run-structured access is a READ (partial-line writes would be
// read-modify-written); loads are batched 8-16 deep per thread because one
// 150 KB block per CU leaves little occupancy to hide HBM latency.
// History (ResNet-9 size, profiles/): a global-gather P2 took 603 us; LDS
// float atomics (binned encode, 229+215 us) retire ~0.4 lanes/clk/CU.
#include <hip/hip_runtime.h>
#include <cstdint>
#include "kernels.h"

namespace commeff {
namespace {

constexpr int kLdsBytes = 160 * 1024;

// Logical block order for the run-gathering passes: blocks are dealt
// round-robin over the 8 XCDs, so neighbouring tiles (encode P2) or chunks
// (query Q2) -- whose runs share 128-byte lines -- would read those lines
// through different L2s; remapped, logical blocks l and l+1 run on one XCD.
__device__ __forceinline__ uint32_t xcd_block(uint32_t bid, uint32_t nwg) {
  const uint32_t xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

__device__ __forceinline__ float signed_v(float v, uint32_t info) {
  return (info & 0x8000u) ? -v : v;
}

// ------------------------------------------------------------- encode P1
template <int R>
__global__ void __launch_bounds__(1024)
enc_p1_kernel(const float* __restrict__ vec, const float* __restrict__ wvec, float scale,
              float wscale, uint32_t d, uint32_t r_rt, uint32_t chunk,
              const uint16_t* __restrict__ src_info, float* __restrict__ vals, bool vec16,
              float* __restrict__ bmax) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const uint32_t r = R > 0 ? static_cast<uint32_t>(R) : r_rt;
  uint32_t amax = 0u;  // max |v| bits (as unsigned: NaN > Inf > finite)
  const uint32_t i0 = blockIdx.x * chunk;
  const uint32_t i1 = min(d, i0 + chunk);
  const uint32_t total = (i1 - i0) * r;
  float* stage = reinterpret_cast<float*>(smem);
  const uint32_t nt = blockDim.x;
  uint32_t iscalar = i0;  // first coordinate left to the per-coordinate loop
  if constexpr (R > 0) {
    if (vec16) {
      // 8 consecutive coordinates per lane: their values in two 16-byte loads
      // (per operand), their 8R u16 slots in R 16-byte loads (chunk % 64 == 0:
      // every unit is 16-byte aligned); kU units per lane in flight
      constexpr uint32_t kU = 2;
      const uint32_t ua = i0 >> 3, ue = ua + ((i1 - i0) >> 3);
      const float4* v4 = reinterpret_cast<const float4*>(vec);
      const float4* w4 = reinterpret_cast<const float4*>(wvec);
      const uint4* s4 = reinterpret_cast<const uint4*>(src_info);
      for (uint32_t ub = ua + threadIdx.x; ub < ue; ub += kU * nt) {
        float v[kU][8];
        uint4 sw[kU][R];
#pragma unroll
        for (uint32_t q = 0; q < kU; ++q) {
          const uint32_t u = ub + q * nt;
          if (u < ue) {
            const float4 a = v4[2 * u], b = v4[2 * u + 1];
            v[q][0] = scale * a.x; v[q][1] = scale * a.y; v[q][2] = scale * a.z; v[q][3] = scale * a.w;
            v[q][4] = scale * b.x; v[q][5] = scale * b.y; v[q][6] = scale * b.z; v[q][7] = scale * b.w;
            if (wvec != nullptr) {
              const float4 c = w4[2 * u], e = w4[2 * u + 1];
              v[q][0] += wscale * c.x; v[q][1] += wscale * c.y; v[q][2] += wscale * c.z; v[q][3] += wscale * c.w;
              v[q][4] += wscale * e.x; v[q][5] += wscale * e.y; v[q][6] += wscale * e.z; v[q][7] += wscale * e.w;
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) amax = max(amax, __float_as_uint(v[q][k]) & 0x7fffffffu);
#pragma unroll
            for (int k = 0; k < R; ++k) sw[q][k] = s4[static_cast<size_t>(u) * R + k];
          }
        }
#pragma unroll
        for (uint32_t q = 0; q < kU; ++q) {
          if (ub + q * nt < ue) {
#pragma unroll
            for (int x = 0; x < 8 * R; ++x) {  // entry (coordinate x / R, row x % R)
              const uint4 wv = sw[q][x >> 3];
              const uint32_t word = (x & 7) < 2 ? wv.x : (x & 7) < 4 ? wv.y : (x & 7) < 6 ? wv.z : wv.w;
              stage[(word >> (16 * (x & 1))) & 0xffffu] = v[q][x / R];
            }
          }
        }
      }
      iscalar = i0 + ((i1 - i0) & ~7u);
    }
  }
  // thread per coordinate, kB coordinates per thread in flight: v_i loaded
  // once, its r slots read from the (i, j)-ordered src_info stream
  constexpr uint32_t kB = 4;
  constexpr uint32_t RR = R > 0 ? static_cast<uint32_t>(R) : kMaxRows;
  for (uint32_t ib = iscalar + threadIdx.x; ib < i1; ib += kB * nt) {
    float v[kB];
    uint32_t sl[kB][RR];
#pragma unroll
    for (uint32_t u = 0; u < kB; ++u) {
      const uint32_t i = ib + u * nt;
      v[u] = 0.f;
      if (i < i1) {
        v[u] = scale * vec[i];
        if (wvec != nullptr) v[u] += wscale * wvec[i];
        amax = max(amax, __float_as_uint(v[u]) & 0x7fffffffu);
        const uint16_t* s = src_info + static_cast<size_t>(i) * r;
#pragma unroll
        for (uint32_t j = 0; j < RR; ++j) sl[u][j] = j < r ? s[j] : 0u;
      }
    }
#pragma unroll
    for (uint32_t u = 0; u < kB; ++u) {
      if (ib + u * nt < i1) {
#pragma unroll
        for (uint32_t j = 0; j < RR; ++j)
          if (j < r) stage[sl[u][j]] = v[u];
      }
    }
  }
  __syncthreads();
  // the stage (already tile-ordered inside the chunk) goes out contiguously,
  // chunk-major: full-line 16-byte stores; P2 gathers the runs (partial-line
  // READS are cheap, partial-line writes are not)
  float4* dst = reinterpret_cast<float4*>(vals + static_cast<size_t>(i0) * r);
  const float4* src = reinterpret_cast<const float4*>(stage);
  const uint32_t n4 = total / 4;
  for (uint32_t k = threadIdx.x; k < n4; k += nt) dst[k] = src[k];
  for (uint32_t k = n4 * 4 + threadIdx.x; k < total; k += nt)
    vals[static_cast<size_t>(i0) * r + k] = stage[k];
  if (bmax != nullptr) {
    // chunk max |v| for the fixed-point encode P2 (dense plans): wave max,
    // then an LDS max over the waves (the stage is free again)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) amax = max(amax, static_cast<uint32_t>(__shfl_xor(static_cast<int>(amax), o)));
    __syncthreads();
    uint32_t* red = reinterpret_cast<uint32_t*>(smem);
    if (threadIdx.x == 0) red[0] = 0u;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) atomicMax(red, amax);
    __syncthreads();
    if (threadIdx.x == 0) bmax[blockIdx.x] = __uint_as_float(red[0]);
  }
}

// ----------------------------------------------- encode P2 (dense, fixed point)
// gfx950 retires LDS float atomics at ~0.33 lanes/clk/CU but 64-bit integer
// ones at ~5.9 (scripts/experiments/lds_atomic_bench.hip, measured), so the dense P2
// accumulates in 64-bit fixed point: every value is scaled by the same power
// of two 2^shift with max|v| * 2^shift < 2^46 (18 bits of headroom: buckets of
// up to 65536 entries, checked when the plan is built), rounded to an integer
// and added with ds_add_u64.  Integer sums are order independent, so the
// encode is bitwise deterministic; the quantum max|v| * 2^-46 lies far below
// the fp32 resolution of every value within 2^22 of the maximum.  A NaN/Inf
// anywhere in the vector makes the whole table NaN (detected downstream).
constexpr int kFxBits = 46;
constexpr double kFxMagic = 6755399441055744.0;  // 1.5 * 2^52

__device__ __forceinline__ int fx_shift(float m) {
  int ex = 0;
  (void)frexpf(m, &ex);  // m = f * 2^ex, f in [0.5, 1); m == 0 -> ex = 0
  return kFxBits - ex;
}

__device__ __forceinline__ bool fx_finite(float m) {
  return (__float_as_uint(m) & 0x7fffffffu) < 0x7f800000u;
}

__global__ void __launch_bounds__(1024) fx_max_kernel(const float* __restrict__ bmax, uint32_t n,
                                                      float* __restrict__ gmax) {
  __shared__ uint32_t red;
  if (threadIdx.x == 0) red = 0u;
  __syncthreads();
  uint32_t m = 0u;
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) m = max(m, __float_as_uint(bmax[i]));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = max(m, static_cast<uint32_t>(__shfl_xor(static_cast<int>(m), o)));
  if ((threadIdx.x & 63) == 0) atomicMax(&red, m);
  __syncthreads();
  if (threadIdx.x == 0) gmax[0] = __uint_as_float(red);
}

__global__ void __launch_bounds__(1024)
enc_p2_dense_fx_kernel(float* __restrict__ table, long long* __restrict__ slab,
                       const float* __restrict__ gmax, const float* __restrict__ vals,
                       const uint16_t* __restrict__ cm_info, const int32_t* __restrict__ p2_src,
                       const int32_t* __restrict__ p2_pos, uint32_t tile, uint32_t total_buckets,
                       uint32_t num_chunks, uint32_t splits, bool overwrite) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned long long* T = reinterpret_cast<unsigned long long*>(smem);
  const uint32_t lb = xcd_block(blockIdx.x, gridDim.x);
  const uint32_t t = lb / splits, s = lb - t * splits;
  const uint32_t nt = blockDim.x;
  const float m = gmax[0];
  const bool finite = fx_finite(m);
  const int shift = fx_shift(m);
  for (uint32_t b = threadIdx.x; b < tile; b += nt) T[b] = 0ull;
  __syncthreads();
  const uint32_t c0 = static_cast<uint32_t>(static_cast<uint64_t>(num_chunks) * s / splits);
  const uint32_t c1 = static_cast<uint32_t>(static_cast<uint64_t>(num_chunks) * (s + 1) / splits);
  const int32_t* psrc = p2_src + static_cast<size_t>(t) * num_chunks;
  const int32_t* ppos = p2_pos + static_cast<size_t>(t) * (num_chunks + 1);
  const uint32_t mask = tile - 1;
  constexpr uint32_t kB = 8;
  const uint32_t hw = threadIdx.x >> 5, l32 = threadIdx.x & 31, nhw = nt >> 5;
  for (uint32_t cb = c0 + hw * kB; finite && cb < c1; cb += nhw * kB) {
    uint32_t src[kB], len[kB];
#pragma unroll
    for (uint32_t q = 0; q < kB; ++q) {
      const uint32_t ch = cb + q;
      src[q] = ch < c1 ? static_cast<uint32_t>(psrc[ch]) : 0u;
      len[q] = ch < c1 ? static_cast<uint32_t>(ppos[ch + 1] - ppos[ch]) : 0u;
    }
    for (uint32_t k0 = 0;; k0 += 128) {
      float v[kB][4];
      uint32_t info[kB][4];
#pragma unroll
      for (uint32_t q = 0; q < kB; ++q) {
#pragma unroll
        for (uint32_t u = 0; u < 4; ++u) {
          const uint32_t k = k0 + u * 32 + l32;
          info[q][u] = 0xffffffffu;
          v[q][u] = 0.f;
          if (k < len[q]) {
            v[q][u] = vals[src[q] + k];
            info[q][u] = cm_info[src[q] + k];
          }
        }
      }
#pragma unroll
      for (uint32_t q = 0; q < kB; ++q) {
#pragma unroll
        for (uint32_t u = 0; u < 4; ++u)
          if (info[q][u] != 0xffffffffu) {
            // round(v * 2^shift) to an integer through the double magic number
            // 1.5 * 2^52 (|.| < 2^46): 4 VALU ops instead of the ~20 of a
            // generic f32 -> i64 conversion
            const double x = ldexp(static_cast<double>(signed_v(v[q][u], info[q][u])), shift) +
                             kFxMagic;
            const long long qi = __double_as_longlong(x) - __double_as_longlong(kFxMagic);
            atomicAdd(T + (info[q][u] & mask), static_cast<unsigned long long>(qi));
          }
      }
      bool more = false;
#pragma unroll
      for (uint32_t q = 0; q < kB; ++q) more |= k0 + 128 < len[q];
      if (!more) break;
    }
  }
  __syncthreads();
  const uint32_t gb0 = t * tile;
  for (uint32_t b = threadIdx.x; b < tile; b += nt) {
    const uint32_t gb = gb0 + b;
    if (gb >= total_buckets) break;
    if (splits == 1) {
      const float f = finite ? static_cast<float>(ldexp(static_cast<double>(static_cast<long long>(T[b])), -shift))
                             : __builtin_nanf("");
      table[gb] = overwrite ? f : table[gb] + f;
    } else {
      slab[static_cast<size_t>(s) * gridDim.x / splits * tile + gb] = static_cast<long long>(T[b]);
    }
  }
}

// the splits' partial tiles, summed in integers (order free) and scaled back
__global__ void __launch_bounds__(256)
enc_fx_reduce_kernel(float* __restrict__ table, const long long* __restrict__ slab,
                     const float* __restrict__ gmax, uint32_t total_buckets, size_t stride,
                     uint32_t splits, bool overwrite) {
  const float m = gmax[0];
  const bool finite = fx_finite(m);
  const int shift = fx_shift(m);
  for (uint32_t gb = blockIdx.x * blockDim.x + threadIdx.x; gb < total_buckets;
       gb += gridDim.x * blockDim.x) {
    long long acc = 0;
    for (uint32_t s = 0; s < splits; ++s) acc += slab[s * stride + gb];
    const float f = finite ? static_cast<float>(ldexp(static_cast<double>(acc), -shift))
                           : __builtin_nanf("");
    table[gb] = overwrite ? f : table[gb] + f;
  }
}

// ------------------------------------------------------------- encode P2
__global__ void __launch_bounds__(1024)
enc_p2_kernel(float* __restrict__ table, const float* __restrict__ vals,
              const uint16_t* __restrict__ perm, const int32_t* __restrict__ csr,
              const int32_t* __restrict__ seg, const int32_t* __restrict__ p2_src,
              const int32_t* __restrict__ p2_pos, uint32_t tile, uint32_t total_buckets,
              uint32_t num_chunks, bool overwrite) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  // LDS: bucket-ordered segment S [kPlanSegCap] | run metadata [2*num_chunks+1]
  float* S = reinterpret_cast<float*>(smem);
  int32_t* msrc = reinterpret_cast<int32_t*>(S + kPlanSegCap);
  int32_t* mpos = msrc + num_chunks;
  const uint32_t t = xcd_block(blockIdx.x, gridDim.x);
  const uint32_t nt = blockDim.x;
  const int32_t* psrc = p2_src + static_cast<size_t>(t) * num_chunks;
  const int32_t* ppos = p2_pos + static_cast<size_t>(t) * (num_chunks + 1);
  for (uint32_t k = threadIdx.x; k < num_chunks; k += nt) msrc[k] = psrc[k];
  for (uint32_t k = threadIdx.x; k <= num_chunks; k += nt) mpos[k] = ppos[k];
  __syncthreads();
  // the tile's run in every chunk (chunk-major vals from P1) is read together
  // with perm at the same positions and scattered (signed) straight into its
  // bucket-order slot; a half-wave per run, kB runs per half-wave in flight
  {
    constexpr uint32_t kB = 16;
    const uint32_t hw = threadIdx.x >> 5, l32 = threadIdx.x & 31, nhw = nt >> 5;
    for (uint32_t c0 = hw * kB; c0 < num_chunks; c0 += nhw * kB) {
      // entries l32 and l32 + 32 of every run in flight at once (runs average
      // ~26 entries; a serial second round trip for the ~10 % of runs longer
      // than 32 used to stall the whole batch)
      float v[kB], v2[kB];
      uint32_t pl[kB], pl2[kB];
#pragma unroll
      for (uint32_t q = 0; q < kB; ++q) {
        const uint32_t ch = c0 + q;
        v[q] = v2[q] = 0.f;
        pl[q] = pl2[q] = 0xffffffffu;
        const uint32_t len = ch < num_chunks ? static_cast<uint32_t>(mpos[ch + 1] - mpos[ch]) : 0u;
        if (l32 < len) {
          v[q] = vals[msrc[ch] + l32];
          pl[q] = perm[msrc[ch] + l32];
        }
        if (l32 + 32 < len) {
          v2[q] = vals[msrc[ch] + l32 + 32];
          pl2[q] = perm[msrc[ch] + l32 + 32];
        }
      }
#pragma unroll
      for (uint32_t q = 0; q < kB; ++q) {
        if (pl[q] != 0xffffffffu) S[pl[q] & 0x7fffu] = signed_v(v[q], pl[q]);
        if (pl2[q] != 0xffffffffu) S[pl2[q] & 0x7fffu] = signed_v(v2[q], pl2[q]);
        const uint32_t ch = c0 + q;
        if (ch < num_chunks) {
          const uint32_t len = mpos[ch + 1] - mpos[ch];
          for (uint32_t k = l32 + 64; k < len; k += 32) {
            const uint32_t x = msrc[ch] + k, p = perm[x];
            S[p & 0x7fffu] = signed_v(vals[x], p);
          }
        }
      }
    }
  }
  __syncthreads();
  // bucket sums: contiguous LDS ranges
  const uint32_t lo = static_cast<uint32_t>(seg[t]);
  const uint32_t gb0 = t * tile;
  for (uint32_t b = threadIdx.x; b < tile; b += nt) {
    const uint32_t gb = gb0 + b;
    if (gb >= total_buckets) break;
    const uint32_t x0 = static_cast<uint32_t>(csr[gb]) - lo, x1 = static_cast<uint32_t>(csr[gb + 1]) - lo;
    float acc = 0.f;
    for (uint32_t x = x0; x < x1; ++x) acc += S[x];
    if (overwrite) table[gb] = acc;
    else if (x1 > x0) table[gb] += acc;
  }
}

// ------------------------------------------------------ encode P2 (dense)
// Many entries per bucket (GPT-2: ~249): a tile's segment (2M entries for
// 8192 buckets) cannot sit in LDS in bucket order, so the tile accumulates
// in LDS with float atomics instead.  grid = num_tiles x splits; block (t, s)
// takes the runs of its 1/splits share of the chunks (read straight from the
// tile's metadata rows in global memory), a half-wave per run with kB runs in
// flight, and adds its partial tile to the table (plain stores when it owns
// the tile, else contiguous 256-B-per-wave global atomics).  Not bitwise
// deterministic (LDS atomic order) -- client-side encode only; every rank
// still receives the identical all-reduced table.
__global__ void __launch_bounds__(1024)
enc_p2_dense_kernel(float* __restrict__ table, const float* __restrict__ vals,
                    const uint16_t* __restrict__ cm_info, const int32_t* __restrict__ p2_src,
                    const int32_t* __restrict__ p2_pos, uint32_t tile, uint32_t total_buckets,
                    uint32_t num_chunks, uint32_t splits, bool overwrite) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* T = reinterpret_cast<float*>(smem);
  const uint32_t lb = xcd_block(blockIdx.x, gridDim.x);
  const uint32_t t = lb / splits, s = lb - t * splits;
  const uint32_t nt = blockDim.x;
  for (uint32_t b = threadIdx.x; b < tile; b += nt) T[b] = 0.f;
  __syncthreads();
  const uint32_t c0 = static_cast<uint32_t>(static_cast<uint64_t>(num_chunks) * s / splits);
  const uint32_t c1 = static_cast<uint32_t>(static_cast<uint64_t>(num_chunks) * (s + 1) / splits);
  const int32_t* psrc = p2_src + static_cast<size_t>(t) * num_chunks;
  const int32_t* ppos = p2_pos + static_cast<size_t>(t) * (num_chunks + 1);
  const uint32_t mask = tile - 1;
  constexpr uint32_t kB = 8;
  const uint32_t hw = threadIdx.x >> 5, l32 = threadIdx.x & 31, nhw = nt >> 5;
  for (uint32_t cb = c0 + hw * kB; cb < c1; cb += nhw * kB) {
    uint32_t src[kB], len[kB];
#pragma unroll
    for (uint32_t q = 0; q < kB; ++q) {
      const uint32_t ch = cb + q;
      src[q] = ch < c1 ? static_cast<uint32_t>(psrc[ch]) : 0u;
      len[q] = ch < c1 ? static_cast<uint32_t>(ppos[ch + 1] - ppos[ch]) : 0u;
    }
    // runs average ~127 entries at GPT-2 size: 4 entries per lane in flight
    for (uint32_t k0 = 0;; k0 += 128) {
      float v[kB][4];
      uint32_t info[kB][4];
#pragma unroll
      for (uint32_t q = 0; q < kB; ++q) {
#pragma unroll
        for (uint32_t u = 0; u < 4; ++u) {
          const uint32_t k = k0 + u * 32 + l32;
          info[q][u] = 0xffffffffu;
          v[q][u] = 0.f;
          if (k < len[q]) {
            v[q][u] = vals[src[q] + k];
            info[q][u] = cm_info[src[q] + k];
          }
        }
      }
#pragma unroll
      for (uint32_t q = 0; q < kB; ++q) {
#pragma unroll
        for (uint32_t u = 0; u < 4; ++u)
          if (info[q][u] != 0xffffffffu)
            atomicAdd(T + (info[q][u] & mask), signed_v(v[q][u], info[q][u]));
      }
      // half-wave-uniform exit: every lane of the half-wave sees the same len[]
      bool more = false;
#pragma unroll
      for (uint32_t q = 0; q < kB; ++q) more |= k0 + 128 < len[q];
      if (!more) break;
    }
  }
  __syncthreads();
  const uint32_t gb0 = t * tile;
  for (uint32_t b = threadIdx.x; b < tile; b += nt) {
    const uint32_t gb = gb0 + b;
    if (gb >= total_buckets) break;
    if (splits == 1) {
      if (overwrite) table[gb] = T[b];
      else table[gb] += T[b];
    } else if (T[b] != 0.f) {
      atomicAdd(table + gb, T[b]);
    }
  }
}

// -------------------------------------------------------------- query Q1
__global__ void __launch_bounds__(256)
qry_q1_kernel(const float* __restrict__ table, const uint16_t* __restrict__ ent_info,
              const int32_t* __restrict__ seg, float* __restrict__ vals, uint32_t tile,
              uint32_t total_buckets, uint32_t splits, const int32_t* __restrict__ base,
              uint32_t num_tiles, uint32_t c0, uint32_t c1, uint32_t num_chunks) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* T = reinterpret_cast<float*>(smem);
  const uint32_t t = blockIdx.x / splits;
  const uint32_t s = blockIdx.x - t * splits;
  const uint32_t tb = t * tile;
  for (uint32_t b = threadIdx.x; b < tile; b += blockDim.x) {
    const uint32_t gb = tb + b;
    T[b] = gb < total_buckets ? table[gb] : 0.f;
  }
  __syncthreads();
  // entries of coordinate chunks [c0, c1) only (a rank's shard of the query):
  // a tile's segment is chunk-major, so they are one contiguous sub-range
  const uint32_t lo = static_cast<uint32_t>(c0 == 0 ? seg[t] : base[static_cast<size_t>(c0) * num_tiles + t]);
  const uint32_t hi = static_cast<uint32_t>(c1 >= num_chunks ? seg[t + 1]
                                                             : base[static_cast<size_t>(c1) * num_tiles + t]);
  const uint32_t n = hi - lo;
  const uint32_t e0 = lo + static_cast<uint32_t>(static_cast<uint64_t>(n) * s / splits);
  const uint32_t e1 = lo + static_cast<uint32_t>(static_cast<uint64_t>(n) * (s + 1) / splits);
  const uint32_t mask = tile - 1;
  const uint32_t nt = blockDim.x;
  // 8 consecutive entries per lane: one 16-byte load of their u16 infos and
  // two 16-byte stores of their values (2-byte loads / 4-byte stores per lane
  // left this pass latency-bound at ~2.3 TB/s, profiles/r2_pmc_gpt2.txt);
  // kU such units per lane in flight.  Unaligned head / tail: scalar.
  const uint32_t ea = min(e1, (e0 + 7u) & ~7u), eb = max(ea, e1 & ~7u);
  for (uint32_t e = e0 + threadIdx.x; e < ea; e += nt) vals[e] = signed_v(T[ent_info[e] & mask], ent_info[e]);
  for (uint32_t e = eb + threadIdx.x; e < e1; e += nt) vals[e] = signed_v(T[ent_info[e] & mask], ent_info[e]);
  constexpr uint32_t kU = 4;
  const uint32_t u0 = ea >> 3, u1 = eb >> 3;
  const uint4* info4 = reinterpret_cast<const uint4*>(ent_info);
  float4* out4 = reinterpret_cast<float4*>(vals);
  for (uint32_t ub = u0 + threadIdx.x; ub < u1; ub += kU * nt) {
    uint4 w[kU];
#pragma unroll
    for (uint32_t q = 0; q < kU; ++q) {
      const uint32_t u = ub + q * nt;
      if (u < u1) w[q] = info4[u];
    }
#pragma unroll
    for (uint32_t q = 0; q < kU; ++q) {
      const uint32_t u = ub + q * nt;
      if (u < u1) {
        const uint32_t h[4] = {w[q].x, w[q].y, w[q].z, w[q].w};
        float o[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const uint32_t inf = (h[k >> 1] >> (16 * (k & 1))) & 0xffffu;
          o[k] = signed_v(T[inf & mask], inf);
        }
        out4[2 * u] = make_float4(o[0], o[1], o[2], o[3]);
        out4[2 * u + 1] = make_float4(o[4], o[5], o[6], o[7]);
      }
    }
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
      const float a = v[q], b = v[q + 1];
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

template <int R, int DEEP>
__global__ void __launch_bounds__(1024)
qry_q2_kernel(const float* __restrict__ vals, uint32_t d, uint32_t r_rt, uint32_t chunk,
              uint32_t num_tiles, const uint16_t* __restrict__ src_info,
              const int32_t* __restrict__ base, const int32_t* __restrict__ off,
              float* __restrict__ est, bool vec16, uint32_t c0) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const uint32_t r = R > 0 ? static_cast<uint32_t>(R) : r_rt;
  const uint32_t cb = xcd_block(blockIdx.x, gridDim.x) + c0;  // coordinate chunk of this block
  const uint32_t i0 = cb * chunk;
  const uint32_t i1 = min(d, i0 + chunk);
  float* stage = reinterpret_cast<float*>(smem);
  uint32_t* soff = reinterpret_cast<uint32_t*>(stage + chunk * r);
  uint32_t* sbase = soff + num_tiles + 1;
  const size_t orow = static_cast<size_t>(cb) * (num_tiles + 1);
  const size_t brow = static_cast<size_t>(cb) * num_tiles;
  for (uint32_t t = threadIdx.x; t <= num_tiles; t += blockDim.x) soff[t] = off[orow + t];
  for (uint32_t t = threadIdx.x; t < num_tiles; t += blockDim.x) sbase[t] = base[brow + t];
  __syncthreads();
  // runs -> stage: a half-wave per run (runs average ~30), kB runs per
  // half-wave in flight at once
  // DEEP x 32 entries of every run in flight before the serial tail (exact
  // plans: runs of ~30 -> 2; dense plans: runs of ~127 -> 4; 4 on the exact
  // plan measured 97 -> 107 us at ResNet-9 size)
  constexpr uint32_t kB = 16;
  const uint32_t hw = threadIdx.x >> 5, l32 = threadIdx.x & 31, nhw = blockDim.x >> 5;
  for (uint32_t t0 = hw * kB; t0 < num_tiles; t0 += nhw * kB) {
    float v[kB][DEEP];
#pragma unroll
    for (uint32_t q = 0; q < kB; ++q) {
      const uint32_t t = t0 + q;
      const uint32_t len = t < num_tiles ? soff[t + 1] - soff[t] : 0u;
#pragma unroll
      for (uint32_t u = 0; u < DEEP; ++u) {
        v[q][u] = 0.f;
        if (l32 + 32 * u < len) v[q][u] = vals[sbase[t] + l32 + 32 * u];
      }
    }
#pragma unroll
    for (uint32_t q = 0; q < kB; ++q) {
      const uint32_t t = t0 + q;
      if (t < num_tiles) {
        const uint32_t o = soff[t], len = soff[t + 1] - o;
#pragma unroll
        for (uint32_t u = 0; u < DEEP; ++u)
          if (l32 + 32 * u < len) stage[o + l32 + 32 * u] = v[q][u];
        for (uint32_t k = l32 + 32 * DEEP; k < len; k += 32) stage[o + k] = vals[sbase[t] + k];
      }
    }
  }
  __syncthreads();
  const int rr = static_cast<int>(r);
  uint32_t iscalar = i0;
  if constexpr (R > 0) {
    if (vec16) {
      // 8 consecutive coordinates per lane: R 16-byte loads of their slots,
      // two 16-byte stores of their medians
      const uint32_t ua = i0 >> 3, ue = ua + ((i1 - i0) >> 3);
      const uint4* s4 = reinterpret_cast<const uint4*>(src_info);
      float4* e4 = reinterpret_cast<float4*>(est);
      for (uint32_t u = ua + threadIdx.x; u < ue; u += blockDim.x) {
        uint4 sw[R];
#pragma unroll
        for (int k = 0; k < R; ++k) sw[k] = s4[static_cast<size_t>(u) * R + k];
        float m[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          float v[kMaxRows];
#pragma unroll
          for (int j = 0; j < R; ++j) {
            const int x = c * R + j;
            const uint4 wv = sw[x >> 3];
            const uint32_t word = (x & 7) < 2 ? wv.x : (x & 7) < 4 ? wv.y : (x & 7) < 6 ? wv.z : wv.w;
            v[j] = stage[(word >> (16 * (x & 1))) & 0xffffu];
          }
          m[c] = lower_median_r<R>(v, rr);
        }
        e4[2 * u] = make_float4(m[0], m[1], m[2], m[3]);
        e4[2 * u + 1] = make_float4(m[4], m[5], m[6], m[7]);
      }
      iscalar = i0 + ((i1 - i0) & ~7u);
    }
  }
  for (uint32_t i = iscalar + threadIdx.x; i < i1; i += blockDim.x) {
    float v[kMaxRows];
    uint32_t sl[kMaxRows];
    const uint16_t* si = src_info + static_cast<size_t>(i) * r;
#pragma unroll
    for (int j = 0; j < (R > 0 ? R : kMaxRows); ++j) sl[j] = j < rr ? si[j] : 0u;
#pragma unroll
    for (int j = 0; j < (R > 0 ? R : kMaxRows); ++j) v[j] = j < rr ? stage[sl[j]] : 0.f;
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

size_t stage_lds(const PlanGeom& p, int r) {
  return static_cast<size_t>(p.chunk) * r * 4 + (2 * p.num_tiles + 1) * 4;
}

void set_lds_attr(const void* fn) {
  (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes);
}

int64_t device_cus() {
  static const int64_t cus = [] {
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess &&
        prop.multiProcessorCount > 0)
      return static_cast<int64_t>(prop.multiProcessorCount);
    return int64_t{256};  // MI355X (CPU-side plan checks)
  }();
  return cus;
}

}  // namespace

bool planned_geometry(int64_t d, int64_t r, int64_t c, PlanGeom* out) {
  if (d <= 0 || r < 1 || r > kMaxRows || c < 1 || d * r >= (int64_t{1} << 31)) return false;
  for (int64_t tile = 4096; tile >= 512; tile >>= 1) {
    PlanGeom p;
    p.tile = tile;
    p.num_tiles = (r * c + tile - 1) / tile;
    // expected segment d*r/(r*c) entries per bucket, 12 % headroom
    const double seg = static_cast<double>(d) / static_cast<double>(c) * static_cast<double>(tile);
    if (seg * 1.12 + 256 > kPlanSegCap) continue;
    const int64_t tables = (2 * p.num_tiles + 1) * 4;
    const int64_t stage_bytes = kLdsBytes - 1024 - tables;
    if (stage_bytes < 64 * r * 4 * 16) continue;
    int64_t chunk = (stage_bytes / 4 / r) / 64 * 64;
    if (chunk > kPlanStageCap / r / 64 * 64) chunk = kPlanStageCap / r / 64 * 64;
    if (chunk < 64) continue;
    // P1 / Q2 run one LDS-filling block per CU: shrink the chunk so the
    // chunk count is just under a whole number of block rounds (863 chunks
    // on 256 CUs would leave the 4th round 37 % busy; 1017 fills it)
    {
      const int64_t cus = device_cus();
      const int64_t rounds = (d + cus * chunk - 1) / (cus * chunk);
      const int64_t bal = ((d + cus * rounds - 1) / (cus * rounds) + 63) / 64 * 64;
      if (bal >= 64 && bal < chunk) chunk = bal;
    }
    p.chunk = chunk;
    p.num_chunks = (d + chunk - 1) / chunk;
    // encode P2 keeps a tile's run metadata (2 words per chunk) beside the
    // segment in LDS
    if (kPlanSegCap * 4 + (2 * p.num_chunks + 1) * 4 > kLdsBytes) continue;
    *out = p;
    return true;
  }
  return false;
}

bool planned_geometry_dense(int64_t d, int64_t r, int64_t c, PlanGeom* out) {
  if (d <= 0 || r < 1 || r > kMaxRows || c < 1 || d * r >= (int64_t{1} << 31)) return false;
  PlanGeom p;
  p.dense = true;
  p.tile = 8192;  // in-tile bucket in 13 bits of the u16 entry info (sign: bit 15)
  p.num_tiles = (r * c + p.tile - 1) / p.tile;
  const int64_t tables = (2 * p.num_tiles + 1) * 4;
  const int64_t stage_bytes = kLdsBytes - 1024 - tables;
  if (stage_bytes < 64 * r * 4 * 16) return false;
  int64_t chunk = (stage_bytes / 4 / r) / 64 * 64;
  if (chunk > kPlanStageCap / r / 64 * 64) chunk = kPlanStageCap / r / 64 * 64;
  if (chunk < 64) return false;
  {
    const int64_t cus = device_cus();
    const int64_t rounds = (d + cus * chunk - 1) / (cus * chunk);
    const int64_t bal = ((d + cus * rounds - 1) / (cus * rounds) + 63) / 64 * 64;
    if (bal >= 64 && bal < chunk) chunk = bal;
  }
  p.chunk = chunk;
  p.num_chunks = (d + chunk - 1) / chunk;
  // encode P2: enough blocks for every CU -> split each tile's chunk range
  p.p2_splits = 1;
  while (p.num_tiles * p.p2_splits < 4 * device_cus() && p.p2_splits < 64) p.p2_splits *= 2;
  *out = p;
  return true;
}

void launch_cs_hash_all(const RowHashes& h, const SketchGeom& g, const int32_t* blk_off,
                        const float* blk_sign, int32_t* out, hipStream_t stream) {
  if (g.d == 0) return;
  int64_t blocks = (static_cast<int64_t>(g.d) + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  COMMEFF_LAUNCH(hash_all_kernel, dim3(static_cast<uint32_t>(blocks)), dim3(256), 0, stream,
                     h, g, blk_off, blk_sign, out);
}

void launch_cs_encode_planned(float* table, const float* vec, const float* wvec, float scale,
                              float wscale, int64_t d, int r, int64_t c, const PlanGeom& p,
                              const PlannedArgs& a, bool overwrite, hipStream_t stream) {
  if (d == 0) return;
  static bool attr = false;
  if (!attr) {
    set_lds_attr(reinterpret_cast<const void*>(enc_p1_kernel<5>));
    set_lds_attr(reinterpret_cast<const void*>(enc_p1_kernel<3>));
    set_lds_attr(reinterpret_cast<const void*>(enc_p1_kernel<1>));
    set_lds_attr(reinterpret_cast<const void*>(enc_p1_kernel<0>));
    set_lds_attr(reinterpret_cast<const void*>(enc_p2_kernel));
    set_lds_attr(reinterpret_cast<const void*>(enc_p2_dense_fx_kernel));
    attr = true;
  }
  const uint32_t nt = static_cast<uint32_t>(p.num_tiles), ch = static_cast<uint32_t>(p.chunk);
  const dim3 g1(static_cast<uint32_t>(p.num_chunks));
  const size_t l1 = static_cast<size_t>(p.chunk) * r * 4;
  const uint32_t dd = static_cast<uint32_t>(d), rr = static_cast<uint32_t>(r);
  const bool v16 = (reinterpret_cast<uintptr_t>(vec) % 16 == 0) &&
                   (reinterpret_cast<uintptr_t>(wvec) % 16 == 0) &&
                   (reinterpret_cast<uintptr_t>(a.src_info) % 16 == 0) && ch % 8 == 0;
  const bool fxp = p.dense && a.fx != nullptr;  // fixed-point dense P2
  switch (r) {
    case 5: COMMEFF_LAUNCH(enc_p1_kernel<5>, g1, dim3(1024), l1, stream, vec, wvec, scale, wscale, dd, rr, ch, a.src_info, a.vals, v16, fxp ? a.bmax : nullptr); break;
    case 3: COMMEFF_LAUNCH(enc_p1_kernel<3>, g1, dim3(1024), l1, stream, vec, wvec, scale, wscale, dd, rr, ch, a.src_info, a.vals, v16, fxp ? a.bmax : nullptr); break;
    case 1: COMMEFF_LAUNCH(enc_p1_kernel<1>, g1, dim3(1024), l1, stream, vec, wvec, scale, wscale, dd, rr, ch, a.src_info, a.vals, v16, fxp ? a.bmax : nullptr); break;
    default: COMMEFF_LAUNCH(enc_p1_kernel<0>, g1, dim3(1024), l1, stream, vec, wvec, scale, wscale, dd, rr, ch, a.src_info, a.vals, v16, fxp ? a.bmax : nullptr); break;
  }
  if (fxp) {
    const uint32_t splits = static_cast<uint32_t>(p.p2_splits);
    const uint32_t total = static_cast<uint32_t>(r * c);
    COMMEFF_LAUNCH(fx_max_kernel, dim3(1), dim3(1024), 0, stream, a.bmax,
                       static_cast<uint32_t>(p.num_chunks), a.gmax);
    COMMEFF_LAUNCH(enc_p2_dense_fx_kernel, dim3(nt * splits), dim3(1024), p.tile * 8, stream,
                       table, reinterpret_cast<long long*>(a.fx), a.gmax, a.vals, a.perm, a.p2_src,
                       a.p2_pos, static_cast<uint32_t>(p.tile), total,
                       static_cast<uint32_t>(p.num_chunks), splits, overwrite);
    if (splits > 1) {
      const uint32_t blocks = (total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096;
      COMMEFF_LAUNCH(enc_fx_reduce_kernel, dim3(blocks), dim3(256), 0, stream, table,
                         reinterpret_cast<const long long*>(a.fx), a.gmax, total,
                         static_cast<size_t>(p.num_tiles) * p.tile, splits, overwrite);
    }
    return;
  }
  if (p.dense) {
    // enough blocks for every CU: split each tile's chunk range
    uint32_t splits = static_cast<uint32_t>(p.p2_splits);
    if (overwrite && splits > 1) {
      tape_memset(table, 0, static_cast<size_t>(r) * c * sizeof(float), stream);
    }
    COMMEFF_LAUNCH(enc_p2_dense_kernel, dim3(nt * splits), dim3(1024), p.tile * 4, stream, table,
                       a.vals, a.perm, a.p2_src, a.p2_pos, static_cast<uint32_t>(p.tile),
                       static_cast<uint32_t>(r * c), static_cast<uint32_t>(p.num_chunks), splits,
                       overwrite);
    return;
  }
  const size_t l2 = static_cast<size_t>(kPlanSegCap) * 4 + (2 * p.num_chunks + 1) * 4;
  COMMEFF_LAUNCH(enc_p2_kernel, dim3(nt), dim3(1024), l2, stream, table, a.vals, a.perm,
                     a.csr, a.seg, a.p2_src, a.p2_pos, static_cast<uint32_t>(p.tile),
                     static_cast<uint32_t>(r * c), static_cast<uint32_t>(p.num_chunks), overwrite);
}

void launch_cs_query_planned(const float* table, float* est, int64_t d, int r, int64_t c,
                             const PlanGeom& p, const PlannedArgs& a, hipStream_t stream,
                             int64_t c0, int64_t c1) {
  if (d == 0) return;
  if (c1 < 0 || c1 > p.num_chunks) c1 = p.num_chunks;
  if (c0 < 0) c0 = 0;
  if (c0 >= c1) return;
  static bool attr = false;
  if (!attr) {
    set_lds_attr(reinterpret_cast<const void*>(qry_q2_kernel<5, 2>));
    set_lds_attr(reinterpret_cast<const void*>(qry_q2_kernel<3, 2>));
    set_lds_attr(reinterpret_cast<const void*>(qry_q2_kernel<1, 2>));
    set_lds_attr(reinterpret_cast<const void*>(qry_q2_kernel<0, 2>));
    set_lds_attr(reinterpret_cast<const void*>(qry_q2_kernel<5, 4>));
    set_lds_attr(reinterpret_cast<const void*>(qry_q2_kernel<0, 4>));
    attr = true;
  }
  const uint32_t nt = static_cast<uint32_t>(p.num_tiles), ch = static_cast<uint32_t>(p.chunk);
  // >= 8 blocks per CU (dense plans have few, long tiles)
  uint32_t splits = 4;
  while (nt * splits < 8 * static_cast<uint32_t>(device_cus()) && splits < 64) splits *= 2;
  COMMEFF_LAUNCH(qry_q1_kernel, dim3(nt * splits), dim3(256), p.tile * 4, stream, table,
                     a.ent_info, a.seg, a.vals, static_cast<uint32_t>(p.tile),
                     static_cast<uint32_t>(r * c), splits, a.base, nt, static_cast<uint32_t>(c0),
                     static_cast<uint32_t>(c1), static_cast<uint32_t>(p.num_chunks));
  const dim3 g2(static_cast<uint32_t>(c1 - c0));
  const uint32_t cc0 = static_cast<uint32_t>(c0);
  const size_t l2 = stage_lds(p, r);
  const uint32_t dd = static_cast<uint32_t>(d), rr = static_cast<uint32_t>(r);
  const bool v16 = (reinterpret_cast<uintptr_t>(est) % 16 == 0) &&
                   (reinterpret_cast<uintptr_t>(a.src_info) % 16 == 0) && ch % 8 == 0;
  if (p.dense) {
    if (r == 5) COMMEFF_LAUNCH((qry_q2_kernel<5, 4>), g2, dim3(1024), l2, stream, a.vals, dd, rr, ch, nt, a.src_info, a.base, a.off, est, v16, cc0);
    else COMMEFF_LAUNCH((qry_q2_kernel<0, 4>), g2, dim3(1024), l2, stream, a.vals, dd, rr, ch, nt, a.src_info, a.base, a.off, est, v16, cc0);
    return;
  }
  switch (r) {
    case 5: COMMEFF_LAUNCH((qry_q2_kernel<5, 2>), g2, dim3(1024), l2, stream, a.vals, dd, rr, ch, nt, a.src_info, a.base, a.off, est, v16, cc0); break;
    case 3: COMMEFF_LAUNCH((qry_q2_kernel<3, 2>), g2, dim3(1024), l2, stream, a.vals, dd, rr, ch, nt, a.src_info, a.base, a.off, est, v16, cc0); break;
    case 1: COMMEFF_LAUNCH((qry_q2_kernel<1, 2>), g2, dim3(1024), l2, stream, a.vals, dd, rr, ch, nt, a.src_info, a.base, a.off, est, v16, cc0); break;
    default: COMMEFF_LAUNCH((qry_q2_kernel<0, 2>), g2, dim3(1024), l2, stream, a.vals, dd, rr, ch, nt, a.src_info, a.base, a.off, est, v16, cc0); break;
  }
}

}  // namespace commeff
