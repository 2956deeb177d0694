// Region Count Sketch for gfx950: encode, median query and heavy-hitter
// zeroing with no atomics and no r*d intermediate; bitwise deterministic.
//
// Hash family (ops/sketch_region.py builds the parameters from the seed):
// the d coordinates are cut into chunks of m = 64 consecutive coordinates
// (one wavefront) and each table row into regions of m buckets, g = 32
// regions per GROUP (G = c // (g m) groups; leftover buckets unused).  Chunks
// are dealt to groups (random balanced order); inside its group a chunk sits
// in a batch of W = 32 chunks, and in row j the batch's chunks take W distinct
// regions of the group (a random injection per (row, batch); W = 32 when
// g >= 32: two chunks per wave per batch).  Coordinate o
// of chunk q lands in row j on bucket
//     region_j(q) * m + (P_j(o) + shift_j(q)) mod m,   sign S_j(o) ^ sigma_j(q)
// with P_j a random permutation of [m].  Inside a chunk the map is a
// bijection; two coordinates of one group collide in row j with probability
// G/c, independently across rows, of different groups never: ~1/c per row,
// like uniform hashing.  A chunk of large values (a "hot" layer) meets a
// different random 1/g of its group in every row, so the median filters it.
// Replaces the reference CSVec's hashed numBlocks layout
// (/root/reference/CommEfficient/fed_aggregator.py:464-467 builds the CSVec,
// fed_worker.py:313-320 encodes, fed_aggregator.py:584-595 unsketches).
//
// Encode (block per group, one wave per chunk of a batch): the group's r x g
// regions accumulate in LDS (40 KB); every chunk is read once; a batch's
// chunks own distinct regions in every row and a chunk's lanes distinct
// buckets, so plain read-add-writes need no atomics; one barrier separates
// batches (a fixed order: deterministic).  Several batches' values are in
// flight at once.
// Query (block per group): the group's r x g regions -> LDS once, then one wave
// per chunk gathers each lane's r signed cells and stores the lower median.
// cinfo word of (row, chunk): region (bits 0-23) | shift << 24 | sigma << 31;
// the encode and query read them in list order ([list position][row]: one
// contiguous 4r-byte run per chunk), the zeroing by chunk ([row][chunk]).
#include <hip/hip_runtime.h>
#include <cstdint>
#include "kernels.h"
#include "region_hash.h"

namespace commeff {
namespace {

using rh::ci_region;
using rh::ci_shift;
using rh::in_region;
using rh::kRegionMask;
using rh::kSignBit;
using rh::neg_of;

// RT rows (0: runtime r <= kMaxRows), SL = chunk slots per wave per pipelined
// group, K slots per batch (batch = K * W chunks, W = blockDim / 64 waves:
// one barrier per K chunks per wave), HW: a weight-decay operand
template <int RT, int SL, int K, bool HW>
__global__ void __launch_bounds__(1024)
cs_region_encode_kernel(float* __restrict__ table, const float* __restrict__ vec,
                        const float* __restrict__ wvec, float scale, float wscale, uint32_t d,
                        uint32_t c, uint32_t m, uint32_t g, uint32_t G, uint32_t nch, uint32_t r_rt,
                        const uint32_t* __restrict__ perm, const uint32_t* __restrict__ cinfo,
                        const int32_t* __restrict__ lists, const int32_t* __restrict__ goffs,
                        int overwrite, float* __restrict__ zero_vec, RegionLayout L) {
  constexpr int NR = RT > 0 ? RT : kMaxRows;
  extern __shared__ __attribute__((aligned(16))) float acc[];  // [r][g * m]
  const uint32_t r = RT > 0 ? static_cast<uint32_t>(RT) : r_rt;
  const uint32_t grp = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint32_t W = blockDim.x >> 6, gm = g * m, rbase = grp * g;
  for (uint32_t e = tid; e < r * gm; e += blockDim.x) acc[e] = 0.f;
  uint32_t pw[NR];  // this lane's permutation words, the same in every chunk
#pragma unroll
  for (int j = 0; j < NR; ++j) pw[j] = (j < static_cast<int>(r) && lane < m) ? perm[j * m + lane] : 0u;
  const int32_t l0 = goffs[grp], l1 = goffs[grp + 1];
  const int32_t step = static_cast<int32_t>(SL * W);
  // software pipeline over groups of SL / K batches: while group k is added into
  // LDS, the values and chunk words of group k + 1 and the chunk ids of group
  // k + 2 are in flight.  Every load is unconditional (indices clamped into
  // range, validity applied at use): a load under a lane or list-end branch
  // is waited for inside the branch.  The chunk words are VECTOR loads (lane
  // j < r fetches row j's word, broadcast with readlane): a scalar load's
  // wait would also wait for the LDS traffic.
  uint32_t q1[SL], q2[SL], word[SL], wordn[SL];
  float x[SL], xn[SL], y[SL], yn[SL];
  const int32_t llast = l1 > l0 ? l1 - 1 : l0;
  const uint32_t lr = lane < r ? lane : r - 1;
  auto ids = [&](int32_t lb, uint32_t (&q)[SL]) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < SL; ++u) q[u] = static_cast<uint32_t>(lists[min(lb + static_cast<int32_t>(u * W + w), llast)]);
  };
  auto values = [&](int32_t lb, const uint32_t (&q)[SL], float (&xx)[SL], float (&yy)[SL], uint32_t (&ww)[SL])
      __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < SL; ++u) {
      ww[u] = cinfo[static_cast<size_t>(min(lb + static_cast<int32_t>(u * W + w), llast)) * r + lr];
      const size_t i = static_cast<size_t>(q[u]) * m + min(lane, d - q[u] * m - 1);
      xx[u] = vec[i];
      if constexpr (HW) yy[u] = wvec[i];
    }
  };
  if (l1 > l0) {
    ids(l0, q1);
    values(l0, q1, x, y, word);
    ids(l0 + step, q2);
  }
  __syncthreads();
  for (int32_t lb = l0; lb < l1; lb += step) {
    uint32_t qc[SL];
#pragma unroll
    for (int u = 0; u < SL; ++u) qc[u] = q1[u];
    // (unconditional even past the end -- clamped loads: a load under a
    // branch is waited for where the branch joins)
    values(lb + step, q2, xn, yn, wordn);
#pragma unroll
    for (int u = 0; u < SL; ++u) q1[u] = q2[u];
    ids(lb + 2 * step, q2);
#pragma unroll
    for (int u = 0; u < SL; ++u) {
      const bool live = lb + static_cast<int32_t>(u * W + w) < l1 && lane < min(m, d - qc[u] * m);
      float v = scale * x[u];
      if constexpr (HW) v += wscale * y[u];
      uint32_t cw[NR];
#pragma unroll
      for (int j = 0; j < NR; ++j) cw[j] = j < static_cast<int>(r) ? __builtin_amdgcn_readlane(word[u], j) : 0u;
      // the previous batch's read-add-writes are done (LDS only: the loads of
      // the groups ahead stay in flight -- __syncthreads would drain them)
      if (u % K == 0) {  // a new batch
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
      }
      if (live) {
        // zero_vec (== vec): the encode is the vector's last reader -- clear
        // it for the next accumulation (each element is read exactly once)
        if (zero_vec != nullptr) zero_vec[static_cast<size_t>(qc[u]) * m + lane] = 0.f;
        uint32_t b[NR];
        float a[NR];
#pragma unroll
        for (int j = 0; j < NR; ++j) {  // distinct cells: every read before the writes
          b[j] = 0u;
          a[j] = 0.f;
          if (j < static_cast<int>(r)) {
            b[j] = j * gm + (ci_region(cw[j]) - rbase) * m + in_region(pw[j], cw[j], m);
            a[j] = acc[b[j]];
          }
        }
#pragma unroll
        for (int j = 0; j < NR; ++j)
          if (j < static_cast<int>(r)) acc[b[j]] = a[j] + (neg_of(pw[j], cw[j]) ? -v : v);
      }
    }
#pragma unroll
    for (int u = 0; u < SL; ++u) {
      x[u] = xn[u];
      if constexpr (HW) y[u] = yn[u];
      word[u] = wordn[u];
    }
  }
  __syncthreads();
  for (uint32_t j = 0; j < r; ++j) {
    float* trow = table + static_cast<size_t>(grp - L.g0) * L.gs + static_cast<size_t>(j) * L.rs;
    for (uint32_t e = tid; e < gm; e += blockDim.x) trow[e] = overwrite ? acc[j * gm + e] : trow[e] + acc[j * gm + e];
    if (overwrite && grp == 0 && L.rs == c)  // row-major: the unused buckets past G*g*m stay zero
      for (uint32_t e = G * gm + tid; e < c; e += blockDim.x) table[static_cast<size_t>(j) * c + e] = 0.f;
  }
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

// est for the chunks of group blockIdx.x inside [q0, q1); blockDim = 64 * W.
// HIST: also the top-k's first histogram of the estimates (csrc/topk.hip
// pass 0: keys = bits & 0x7fffffff >= hint[0], bin = key >> 20) -- LDS
// privatised, non-empty bins added to hist0: integer counts, deterministic
// Server momentum fused into the staging (MOM, csrc/elementwise.hip
// momentum_ef semantics on this group's regions, which no other block
// touches): 1 = virtual error feedback, V = rho V + gscale G, E += V, the
// query reads E (= table); 2 = V = rho V + gscale G, the query reads V (=
// table).  The regions of every group are staged (and updated) even when the
// query covers only a chunk range; the unused tail buckets stay zero.
struct RegionMom {
  float* V;
  const float* G;
  float rho, gscale;
  int mode;
};

template <int RT, bool HIST>
__global__ void __launch_bounds__(1024)
cs_region_query_kernel(float* __restrict__ table, float* __restrict__ est, uint32_t d,
                       RegionLayout L, uint32_t m, uint32_t g, uint32_t nch, uint32_t r_rt,
                       const uint32_t* __restrict__ perm, const uint32_t* __restrict__ cinfo,
                       const int32_t* __restrict__ lists, const int32_t* __restrict__ goffs,
                       uint32_t q0, uint32_t q1, int vec4, const uint32_t* __restrict__ hint,
                       uint32_t* __restrict__ hist0, RegionMom mom, uint64_t* __restrict__ ballots,
                       uint32_t* __restrict__ segtot, const int32_t* __restrict__ cpos, uint32_t bpg) {
  // ballots (m == 64): per chunk of est the mask of keys >= hint, and the
  // per-segment (1,024 chunks) popcount totals: the top-k's candidate list
  // (csrc/topk.hip cand_compact_kernel)
  __shared__ uint32_t hh[HIST ? 2048 : 1];
  __shared__ uint32_t sh[HIST ? 2048 : 1];
  if constexpr (HIST)
    for (uint32_t b = threadIdx.x; b < 2048; b += blockDim.x) {
      hh[b] = 0u;
      sh[b] = 0u;
    }
  const uint32_t hlb = (HIST && hint != nullptr) ? hint[0] : 0u;
  constexpr int NR = RT > 0 ? RT : kMaxRows;
  extern __shared__ __attribute__((aligned(16))) float reg[];  // [r][g * m]
  const uint32_t r = RT > 0 ? static_cast<uint32_t>(RT) : r_rt;
  // bpg blocks per group (a shard of few groups): each stages the group's
  // regions (read-only: the momentum ran in its own pass) and gathers its
  // 1/bpg of the group's chunk list
  const uint32_t gl = blockIdx.x / bpg, part = blockIdx.x - gl * bpg;
  const uint32_t grp = gl + L.g0, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint32_t W = blockDim.x >> 6, gm = g * m, rbase = grp * g;
  if (vec4) {
    // every row's staging loads of a pass issued before its stores (SU float4
    // of table, G and V per thread in flight): one dependent HBM round trip per
    // pass instead of one per row -- the rows' loads were serialised behind
    // the previous row's stores (table / V may alias G as far as the compiler
    // knows)
    constexpr int SU = 4;
    const uint32_t q4 = gm >> 2, n4 = r * q4;
    for (uint32_t e0 = tid; e0 < n4; e0 += SU * blockDim.x) {
      float4 t[SU], gg[SU], vv[SU];
      size_t o[SU];
      uint32_t di[SU];
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        const uint32_t e = min(e0 + u * blockDim.x, n4 - 1);  // (clamped: loads unconditional)
        const uint32_t j = e / q4, ee = e - j * q4;
        o[u] = static_cast<size_t>(gl) * L.gs + static_cast<size_t>(j) * L.rs + 4 * ee;
        di[u] = j * gm + 4 * ee;
        t[u] = *reinterpret_cast<const float4*>(table + o[u]);
        if (mom.mode != 0) {
          gg[u] = *reinterpret_cast<const float4*>(mom.G + o[u]);
          vv[u] = mom.mode == 1 ? *reinterpret_cast<const float4*>(mom.V + o[u]) : t[u];
        }
      }
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        if (e0 + u * blockDim.x >= n4) break;
        float4 tt = t[u];
        if (mom.mode != 0) {
          float4 v = vv[u];
          // (explicit fmaf, as in momentum_ef: identical rounding)
          v.x = fmaf(mom.rho, v.x, mom.gscale * gg[u].x);
          v.y = fmaf(mom.rho, v.y, mom.gscale * gg[u].y);
          v.z = fmaf(mom.rho, v.z, mom.gscale * gg[u].z);
          v.w = fmaf(mom.rho, v.w, mom.gscale * gg[u].w);
          if (mom.mode == 1) {
            *reinterpret_cast<float4*>(mom.V + o[u]) = v;
            tt.x += v.x; tt.y += v.y; tt.z += v.z; tt.w += v.w;
          } else {
            tt = v;
          }
          *reinterpret_cast<float4*>(table + o[u]) = tt;
        }
        *reinterpret_cast<float4*>(reg + di[u]) = tt;
      }
    }
  } else {
  for (uint32_t j = 0; j < r; ++j) {
    const size_t o = static_cast<size_t>(gl) * L.gs + static_cast<size_t>(j) * L.rs;
    float* src = table + o;
    float* dst = reg + j * gm;
    {
      for (uint32_t e = tid; e < gm; e += blockDim.x) {
        float t = src[e];
        if (mom.mode != 0) {
          float v = fmaf(mom.rho, mom.mode == 1 ? mom.V[o + e] : t, mom.gscale * mom.G[o + e]);
          if (mom.mode == 1) {
            mom.V[o + e] = v;
            t += v;
          } else {
            t = v;
          }
          src[e] = t;
        }
        dst[e] = t;
      }
    }
  }
  }
  uint32_t pw[NR];
#pragma unroll
  for (int j = 0; j < NR; ++j) pw[j] = (j < static_cast<int>(r) && lane < m) ? perm[j * m + lane] : 0u;
  __syncthreads();
  const int rr = static_cast<int>(r);
  const int32_t ga = goffs[grp], gb = goffs[grp + 1], gn = gb - ga;
  const int32_t l0 = ga + static_cast<int32_t>((static_cast<int64_t>(gn) * part) / bpg);
  const int32_t l1 = ga + static_cast<int32_t>((static_cast<int64_t>(gn) * (part + 1)) / bpg);
  // chunk ids and words of the next UQ chunks of this wave are in flight
  // while the current UQ are gathered (VECTOR loads for the words: lane j < r
  // fetches row j's word, readlane broadcasts -- a scalar load's wait would
  // also wait for the LDS gathers)
  constexpr int UQ = 8;
  const int32_t step = static_cast<int32_t>(UQ * W);
  uint32_t q[UQ], word[UQ], qn[UQ], wn[UQ];
  // (unconditional loads at clamped positions: a load under a branch is
  // waited for inside the branch)
  const int32_t llast = l1 > l0 ? l1 - 1 : l0;
  const uint32_t lr = lane < r ? lane : r - 1;
  auto fetch = [&](int32_t lb, uint32_t (&qq)[UQ], uint32_t (&ww)[UQ]) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < UQ; ++u) {
      const int32_t li = min(lb + static_cast<int32_t>(u * W + w), llast);
      qq[u] = static_cast<uint32_t>(lists[li]);
      ww[u] = cinfo[static_cast<size_t>(li) * r + lr];
    }
  };
  if (l1 > l0) fetch(l0, q, word);
  for (int32_t lb = l0; lb < l1; lb += step) {
    fetch(lb + step, qn, wn);  // (unconditional, clamped: see the encode)
#pragma unroll
    for (int u = 0; u < UQ; ++u) {
      // (wave-uniform) past the list end / another rank's shard
      if (lb + static_cast<int32_t>(u * W + w) >= l1 || q[u] < q0 || q[u] >= q1) continue;
      const uint32_t len = min(m, d - q[u] * m);
      uint32_t cw[NR];
#pragma unroll
      for (int j = 0; j < NR; ++j) cw[j] = j < rr ? __builtin_amdgcn_readlane(word[u], j) : 0u;
      bool cand = false;
      if (lane < len) {
        float v[kMaxRows];
#pragma unroll
        for (int j = 0; j < kMaxRows; ++j) {
          v[j] = 0.f;
          if (j < NR && j < rr) {
            const float x = reg[j * gm + (ci_region(cw[j]) - rbase) * m + in_region(pw[j], cw[j], m)];
            v[j] = neg_of(pw[j], cw[j]) ? -x : x;
          }
        }
        const float e = lower_median<RT>(v, rr);
        // (cpos: a sharded query's compact chunk positions, ascending in q)
        const uint32_t qo = cpos != nullptr ? static_cast<uint32_t>(cpos[q[u]]) : q[u];
        est[static_cast<size_t>(qo) * m + lane] = e;
        if constexpr (HIST) {
          const uint32_t key = __float_as_uint(e) & 0x7fffffffu;
          cand = key >= hlb;
          if (cand) atomicAdd(hh + (key >> 20), 1u);
        }
      }
      if constexpr (HIST) {
        if (ballots != nullptr) {
          const uint64_t bal = __ballot(cand);
          if (lane == 0) {
            const uint32_t qb = (cpos != nullptr ? static_cast<uint32_t>(cpos[q[u]]) : q[u]) - q0;
            ballots[qb] = bal;
            atomicAdd(sh + (qb >> 10), static_cast<uint32_t>(__popcll(bal)));
          }
        }
      }
    }
#pragma unroll
    for (int u = 0; u < UQ; ++u) {
      q[u] = qn[u];
      word[u] = wn[u];
    }
  }
  if constexpr (HIST) {
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < 2048; b += blockDim.x) {
      if (hh[b] != 0u) atomicAdd(hist0 + b, hh[b]);
      if (ballots != nullptr && sh[b] != 0u) atomicAdd(segtot + b, sh[b]);
    }
  }
}

// zero cells (j, bucket_j(idx[t])) of t1 (and t2) where vals[t] != 0 (or always)
__global__ void __launch_bounds__(256)
cs_region_zero_kernel(float* __restrict__ t1, float* __restrict__ t2, const int64_t* __restrict__ idx,
                      const float* __restrict__ vals, int64_t k, uint64_t d, uint32_t r, uint32_t g,
                      uint32_t m, uint32_t nch, const uint32_t* __restrict__ perm,
                      const uint32_t* __restrict__ cinfo, RegionLayout L) {
  const int64_t e = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (e >= k * r) return;
  const int64_t t = e / r;
  const uint32_t j = static_cast<uint32_t>(e - t * r);
  if (vals != nullptr && vals[t] == 0.f) return;
  const uint64_t i = static_cast<uint64_t>(idx[t]);
  if (i >= d) return;  // (top-k indices are always in range)
  const size_t cell = rh::cell_of(i, j, g, m, nch, perm, cinfo, L);
  if (cell == ~static_cast<size_t>(0)) return;  // another rank's group (sharded server)
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

// W = chunks per batch: one wave per chunk up to 16, two per wave at 32
bool region_geometry_supported(int64_t r, int64_t m, int64_t g, int64_t W) {
  return r >= 1 && r <= kMaxRows && m >= 1 && m <= 64 && g >= 1 && W >= 1 && (W <= 16 || W == 32) &&
         W <= g && r * g * m * 4 <= 160 * 1024;
}

void launch_cs_region_encode(float* table, const float* vec, const float* wvec, float scale,
                             float wscale, int64_t d, int r, int64_t c, int64_t m, int64_t g, int64_t G,
                             int64_t W, int64_t nch, const uint32_t* perm, const uint32_t* cinfo,
                             const int32_t* lists, const int32_t* goffs, bool overwrite, RegionLayout L,
                             hipStream_t stream, float* zero_vec) {
  const int lds = static_cast<int>(r * g * m * 4);
  const int nw = W > 16 ? 16 : static_cast<int>(W);
  const dim3 grid(static_cast<uint32_t>(G)), block(static_cast<uint32_t>(64 * nw));
#define COMMEFF_REGION_ENC(RR, SS, KK, HH)                                                               \
  do {                                                                                                   \
    static int done = 0;                                                                                 \
    set_lds_once(cs_region_encode_kernel<RR, SS, KK, HH>, lds, &done);                                   \
    COMMEFF_LAUNCH((cs_region_encode_kernel<RR, SS, KK, HH>), grid, block, lds, stream, table, vec, wvec, \
                       scale, wscale, static_cast<uint32_t>(d), static_cast<uint32_t>(c),                \
                       static_cast<uint32_t>(m), static_cast<uint32_t>(g), static_cast<uint32_t>(G),     \
                       static_cast<uint32_t>(nch), static_cast<uint32_t>(r), perm, cinfo, lists, goffs,  \
                       overwrite ? 1 : 0, zero_vec, L);                                                  \
  } while (0)
  const bool hw = wvec != nullptr && wscale != 0.f;
  if (W == 32) {  // two chunks per wave per batch
    if (r == 5 && hw) COMMEFF_REGION_ENC(5, 8, 2, true);
    else if (r == 5) COMMEFF_REGION_ENC(5, 8, 2, false);
    else if (hw) COMMEFF_REGION_ENC(0, 2, 2, true);
    else COMMEFF_REGION_ENC(0, 2, 2, false);
  } else {
    if (r == 5 && hw) COMMEFF_REGION_ENC(5, 8, 1, true);
    else if (r == 5) COMMEFF_REGION_ENC(5, 8, 1, false);
    else if (hw) COMMEFF_REGION_ENC(0, 2, 1, true);
    else COMMEFF_REGION_ENC(0, 2, 1, false);
  }
#undef COMMEFF_REGION_ENC
}

void launch_cs_region_query(float* table, float* est, int64_t d, int r, int64_t m, int64_t g,
                            int64_t W, int64_t nch, const uint32_t* perm, const uint32_t* cinfo,
                            const int32_t* lists, const int32_t* goffs, int64_t q0, int64_t q1,
                            RegionLayout L, hipStream_t stream, const uint32_t* hint, uint32_t* hist0,
                            float* momV, const float* momG, float rho, float gscale, int mom_mode,
                            uint64_t* ballots, uint32_t* segtot, const int32_t* cpos) {
  RegionMom mom{momV, momG, rho, gscale, mom_mode};
  if (m != 64 || hist0 == nullptr) ballots = nullptr;
  if (q1 <= q0 || L.g1 <= L.g0) return;
  const int lds = static_cast<int>(r * g * m * 4);
  const int vec4 = ((g * m) % 4 == 0 && L.gs % 4 == 0 && L.rs % 4 == 0) ? 1 : 0;
  // a group-major shard of few groups (the sharded server at N ranks: G / N
  // groups) would leave most CUs idle at one block per group while each
  // block's time stays that of a whole group: several blocks per group then,
  // the server momentum in its own elementwise pass first (the staging blocks
  // only read)
  static const int cus = [] {
    int dev = 0;
    hipDeviceProp_t prop;
    return (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
               ? prop.multiProcessorCount : 256;
  }();
  const uint32_t ng = L.g1 - L.g0;
  uint32_t bpg = 1;
  const bool shard = L.rs == static_cast<uint32_t>(g * m) && L.gs == static_cast<uint32_t>(r * g * m);
  if (shard && 2 * ng <= static_cast<uint32_t>(cus)) {
    bpg = static_cast<uint32_t>(cus) / ng;
    if (bpg > 16) bpg = 16;
  }
  if (bpg > 1 && mom.mode != 0) {
    const int64_t n = static_cast<int64_t>(ng) * r * g * m;  // the shard's cells, contiguous
    if (mom.mode == 1) launch_momentum_ef(momV, table, momG, n, rho, gscale, 1, stream);
    else launch_momentum_ef(table, nullptr, momG, n, rho, gscale, 0, stream);
    mom.mode = 0;
  }
  const dim3 grid(ng * bpg), block(static_cast<uint32_t>(64 * (W > 16 ? 16 : W)));
#define COMMEFF_REGION_QRY(RR, HH)                                                                       \
  do {                                                                                                   \
    static int done = 0;                                                                                 \
    set_lds_once(cs_region_query_kernel<RR, HH>, lds, &done);                                            \
    COMMEFF_LAUNCH((cs_region_query_kernel<RR, HH>), grid, block, lds, stream, table, est,           \
                       static_cast<uint32_t>(d), L, static_cast<uint32_t>(m),                            \
                       static_cast<uint32_t>(g), static_cast<uint32_t>(nch), static_cast<uint32_t>(r),   \
                       perm, cinfo, lists, goffs, static_cast<uint32_t>(q0), static_cast<uint32_t>(q1),  \
                       vec4, hint, hist0, mom, ballots, segtot, cpos, bpg);                              \
  } while (0)
  if (hist0 != nullptr) {
    if (r == 5) COMMEFF_REGION_QRY(5, true);
    else COMMEFF_REGION_QRY(0, true);
  } else {
    if (r == 5) COMMEFF_REGION_QRY(5, false);
    else COMMEFF_REGION_QRY(0, false);
  }
#undef COMMEFF_REGION_QRY
}

void launch_cs_region_zero(float* t1, float* t2, const int64_t* idx, const float* vals, int64_t k,
                           int64_t d, int r, int64_t g, int64_t m, int64_t nch, const uint32_t* perm,
                           const uint32_t* cinfo, RegionLayout L, hipStream_t stream) {
  const int64_t n = k * r;
  if (n <= 0) return;
  COMMEFF_LAUNCH(cs_region_zero_kernel, dim3(static_cast<uint32_t>((n + 255) / 256)), dim3(256), 0,
                 stream, t1, t2, idx, vals, k, static_cast<uint64_t>(d), static_cast<uint32_t>(r),
                 static_cast<uint32_t>(g), static_cast<uint32_t>(m), static_cast<uint32_t>(nch), perm, cinfo,
                 L);
}

}  // namespace commeff
