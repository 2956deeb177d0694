// Deterministic magnitude top-k (radix select) for gfx950.
//
// Replaces the reference's `_topk` (torch.topk(vec**2, k, sorted=False) +
// dense scatter, /root/reference/CommEfficient/utils.py:232-252) and the
// top-k inside CSVec.unSketch.
//
// Every rank must pick the SAME set (the server update is replicated on all
// ranks), so ties are broken by index (lower index wins) and the output is
// written in ascending index order -- the result is a pure function of x.
//
// Algorithm (no host sync, fixed launch sequence -> hipGraph capturable):
//   key(i) = bits(x[i]) & 0x7fffffff        (monotone in |x| for finite x)
//   three histogram passes over 11/11/9-bit digits of the key (one histogram
//   buffer each; pass 0 optionally bounded below by a hint, see hist_kernel), a count pass (per-block #>T, #==T) and an ordered
//   compaction pass.  The digit selections (walk a histogram from the top to
//   the bin holding the k-th largest key) and the scan of the per-block
//   counts are not kernels of their own: every block of the following pass
//   redoes them in its prologue from the (L2-resident) histograms / counts --
//   identical integer work in every block, so the result stays deterministic
//   -- which saves four one-workgroup launches per top-k.  Histograms are
//   privatised in LDS; only non-empty bins are flushed with atomics.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdlib>
#include <cstdint>
#include "kernels.h"

namespace commeff {
namespace {

constexpr int kBins = 2048;
constexpr int kNB = 4096;  // blocks for count/write passes (upper bound)
constexpr int kSegC = 1024;    // candidate lists: chunks per segment
constexpr int kSegMax = 2048;  // segments (n <= 2048 * 65536)

struct WS {
  uint32_t* hist[4];  // kBins each (pass 2 uses 512; [3]: pass-0 fill-in below the hint)
  uint32_t* cnt_gt;   // kNB
  uint32_t* cnt_eq;   // kNB
  uint32_t* wk;       // 16: the digit walk after pass p (prefix, remaining) at [2p - 2, 2p - 1]
};

WS carve(void* base) {
  char* p = reinterpret_cast<char*>(base);
  WS w;
  for (int i = 0; i < 4; ++i) {
    w.hist[i] = reinterpret_cast<uint32_t*>(p);
    p += kBins * 4;
  }
  w.cnt_gt = reinterpret_cast<uint32_t*>(p); p += kNB * 4;
  w.cnt_eq = reinterpret_cast<uint32_t*>(p); p += kNB * 4;
  w.wk = reinterpret_cast<uint32_t*>(p); p += 64;
  return w;
}

__device__ __forceinline__ uint32_t key_of(float x) {
  return __float_as_uint(x) & 0x7fffffffu;
}

// Block-wide (256 threads) digit selection: the bin of `hist` (nbins, walked
// from the top) that holds the `remaining`-th largest key and the count of
// keys in higher bins.  Every thread gets the result.
struct Sel {
  uint32_t bin, above;
};
template <int NBINS>
__device__ Sel select_bin(const uint32_t* __restrict__ hist, uint32_t remaining, uint32_t* tot,
                          uint32_t* res, const uint32_t* __restrict__ hist2 = nullptr) {
  constexpr int per = NBINS / 256;
  uint32_t c[per];
  uint32_t s = 0;
#pragma unroll
  for (int q = 0; q < per; ++q) {
    const int b = NBINS - 1 - (threadIdx.x * per + q);
    c[q] = hist[b] + (hist2 != nullptr ? hist2[b] : 0u);
    s += c[q];
  }
  // inclusive scan over threads: wave scans + 4 wave totals
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t inc = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(inc, o, 64);
    if (lane >= o) inc += t;
  }
  if (lane == 63) tot[wave] = inc;
  __syncthreads();
  uint32_t before = 0;
#pragma unroll
  for (int w = 0; w < 4; ++w) before += w < wave ? tot[w] : 0u;
  const uint32_t above = before + inc - s;
  if (threadIdx.x == 0) {
    res[0] = 0;
    res[1] = 0;
  }
  __syncthreads();
  if (above < remaining && above + s >= remaining) {
    uint32_t run = above;
#pragma unroll
    for (int q = 0; q < per; ++q) {
      if (run + c[q] >= remaining) {
        res[0] = NBINS - 1 - (threadIdx.x * per + q);
        res[1] = run;
        break;
      }
      run += c[q];
    }
  }
  __syncthreads();
  const Sel r = {res[0], res[1]};
  __syncthreads();  // tot / res reusable
  return r;
}

// the (prefix, remaining) after PASSES digit selections; thr/ties when 3
struct Walk {
  uint32_t prefix, remaining;
};
template <int PASSES>
__device__ Walk walk(const WS& w, uint32_t k, uint32_t* tot, uint32_t* res) {
  Walk s = {0u, k};
  if (PASSES >= 1) {
    const Sel a = select_bin<2048>(w.hist[0], s.remaining, tot, res, w.hist[3]);
    s.prefix = a.bin;
    s.remaining -= a.above;
  }
  if (PASSES >= 2) {
    const Sel a = select_bin<2048>(w.hist[1], s.remaining, tot, res);
    s.prefix = (s.prefix << 11) | a.bin;
    s.remaining -= a.above;
  }
  if (PASSES >= 3) {
    const Sel a = select_bin<512>(w.hist[2], s.remaining, tot, res);
    s.prefix = (s.prefix << 9) | a.bin;  // = the k-th largest key
    s.remaining -= a.above;              // = how many keys == thr to take
  }
  return s;
}

// The walk after PASSES selections with the earlier ones taken from ws.wk
// (written by block 0 of the previous pass -- every block computes the same
// integers, the stream orders the passes): one select_bin per pass instead
// of PASSES; block 0 stores this pass's result for the next
template <int PASSES>
__device__ Walk walk_cached(const WS& w, uint32_t k, uint32_t* tot, uint32_t* res) {
  Walk s = {0u, k};
  if constexpr (PASSES == 1) {
    const Sel a = select_bin<2048>(w.hist[0], s.remaining, tot, res, w.hist[3]);
    s.prefix = a.bin;
    s.remaining -= a.above;
  } else if constexpr (PASSES == 2) {
    s = Walk{w.wk[0], w.wk[1]};
    const Sel a = select_bin<2048>(w.hist[1], s.remaining, tot, res);
    s.prefix = (s.prefix << 11) | a.bin;
    s.remaining -= a.above;
  } else if constexpr (PASSES == 3) {
    s = Walk{w.wk[2], w.wk[3]};
    const Sel a = select_bin<512>(w.hist[2], s.remaining, tot, res);
    s.prefix = (s.prefix << 9) | a.bin;
    s.remaining -= a.above;
  }
  if (PASSES >= 1 && blockIdx.x == 0 && threadIdx.x == 0) {
    w.wk[2 * PASSES - 2] = s.prefix;
    w.wk[2 * PASSES - 1] = s.remaining;
  }
  return s;
}

// PASS 0: digit = key >> 20 (11 bits)
// PASS 1: digit = (key >> 9) & 0x7ff, needs (key >> 20) == prefix
// PASS 2: digit = key & 0x1ff,         needs (key >> 9)  == prefix
// With a lower-bound hint L (the previous call's threshold / 2, ``hint``):
// PASS 0 histograms only keys >= L -- for a tail selection almost every
// element is below L, so the pass streams instead of queueing on
// same-bin LDS atomics -- and PASS 3 (the fill-in) adds the keys < L only if
// fewer than k keys were >= L (the bound was too high).  Bins at and above
// L's bin then hold exact counts of every key >= L, which is all the top-down
// walk reads whenever >= k keys are >= L; otherwise the fill-in makes the
// histogram exact.  Deterministic either way (integer counts).
// Candidate mode (CAND): the passes read the compacted candidate list of
// cand_compact_kernel (ctl[0] = 1: values cval[0, ctl[1]), their indices
// cidx) instead of x[0, n) when the list is in use (see launch_topk_cand_rest)
struct Cand {
  const uint32_t* ctl;
  const float* val;
  const int32_t* idx;
};

template <int PASS, bool CAND = false>
__global__ void __launch_bounds__(256)
hist_kernel(const float* __restrict__ x, int64_t n, WS ws, uint32_t kk, const uint32_t* __restrict__ hint,
            Cand cd = Cand{}) {
  __shared__ uint32_t h[kBins];
  __shared__ uint32_t tot[4], res[2];
  if (CAND && cd.ctl[0] != 0u) {
    x = cd.val;
    n = cd.ctl[1];
  }
  for (int b = threadIdx.x; b < kBins; b += blockDim.x) h[b] = 0;
  const uint32_t lb = hint != nullptr ? hint[0] : 0u;
  if constexpr (PASS == 3) {
    // skip the fill-in when >= k keys were >= L (every block agrees)
    uint32_t c = 0;
    for (int b = threadIdx.x; b < kBins; b += blockDim.x) c += ws.hist[0][b];
    for (int o = 32; o > 0; o >>= 1) c += __shfl_down(c, o);
    if ((threadIdx.x & 63) == 0) tot[threadIdx.x >> 6] = c;
    __syncthreads();
    if (tot[0] + tot[1] + tot[2] + tot[3] >= kk) return;
    __syncthreads();
  }
  const uint32_t prefix = PASS == 3 ? 0u : walk_cached<PASS == 3 ? 0 : PASS>(ws, kk, tot, res).prefix;
  __syncthreads();  // h zeroed before any atomic
  // (LDS atomics retire ~0.4 lanes/clk/CU and bound pass 0; per-wave
  // sub-histograms measured no faster, wave-aggregated atomics 4x slower:
  // normal-ish data spreads a wave over too many distinct bins)
  auto add = [&](float v, bool in) __attribute__((always_inline)) {
    if (!in) return;
    const uint32_t k = key_of(v);
    if (PASS == 0) {
      if (k >= lb) atomicAdd(h + (k >> 20), 1u);
    } else if (PASS == 3) {
      if (k < lb) atomicAdd(h + (k >> 20), 1u);
    } else if (PASS == 1) {
      if ((k >> 20) == prefix) atomicAdd(h + ((k >> 9) & 0x7ff), 1u);
    } else {
      if ((k >> 9) == prefix) atomicAdd(h + (k & 0x1ff), 1u);
    }
  };
  // 16-byte loads, kU of them in flight per thread before the LDS atomics
  // (one load at a time left the pass latency-bound)
  constexpr int kU = 4;
  const int64_t n4 = (reinterpret_cast<uintptr_t>(x) & 15) == 0 ? n / 4 : 0;  // float4 count
  const float4* x4 = reinterpret_cast<const float4*>(x);
  const int64_t nt = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i0 = static_cast<int64_t>(blockIdx.x) * blockDim.x; i0 < n4; i0 += kU * nt) {
    const int64_t i = i0 + threadIdx.x;
    float4 v[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u)
      v[u] = i + u * nt < n4 ? x4[i + u * nt] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const bool in = i + u * nt < n4;
      add(v[u].x, in);
      add(v[u].y, in);
      add(v[u].z, in);
      add(v[u].w, in);
    }
  }
  // scalar tail
  const int64_t t0 = n4 * 4 + static_cast<int64_t>(blockIdx.x) * blockDim.x;
  for (int64_t i = t0; i < n; i += nt) {
    const int64_t j = i + threadIdx.x;
    add(j < n ? x[j] : 0.f, j < n);
  }
  __syncthreads();
  uint32_t* hist = ws.hist[PASS];
  for (int b = threadIdx.x; b < kBins; b += blockDim.x) {
    const uint32_t c = h[b];
    if (c) atomicAdd(hist + b, c);
  }
}

// candidate mode: a block's span from the device-side length
__device__ __forceinline__ int64_t cand_span(int64_t n) {
  const int64_t sp = (n + gridDim.x - 1) / gridDim.x;
  return ((sp + 1023) / 1024) * 1024;
}

template <bool CAND = false>
__global__ void __launch_bounds__(256)
count_kernel(const float* __restrict__ x, int64_t n, int64_t span, WS ws, uint32_t kk, Cand cd = Cand{}) {
  __shared__ uint32_t tot[4], res[2];
  if constexpr (CAND) {
    if (cd.ctl[0] != 0u) {
      x = cd.val;
      n = cd.ctl[1];
    }
    span = cand_span(n);
  }
  const uint32_t thr = walk_cached<3>(ws, kk, tot, res).prefix;
  const int64_t i0 = blockIdx.x * span;
  const int64_t i1 = min(n, i0 + span);
  uint32_t gt = 0, eq = 0;
  auto add = [&](float v, bool in) __attribute__((always_inline)) {
    const uint32_t k = key_of(v);
    gt += in && k > thr;
    eq += in && k == thr;
  };
  // 16-byte loads, 4 per thread in flight (4-byte loads left this pass
  // latency-bound at ~2 TB/s on GPT-2-size vectors); span is a multiple of
  // 1024, so every block's range starts 16-byte aligned
  const bool al = (reinterpret_cast<uintptr_t>(x) & 15) == 0;
  constexpr int kU = 4;
  for (int64_t base = i0 + 4 * threadIdx.x; base < i1; base += 1024 * kU) {
    float4 q[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t i = base + 1024 * u;
      if (al && i + 3 < i1) {
        q[u] = *reinterpret_cast<const float4*>(x + i);
      } else {
        q[u].x = i < i1 ? x[i] : 0.f;
        q[u].y = i + 1 < i1 ? x[i + 1] : 0.f;
        q[u].z = i + 2 < i1 ? x[i + 2] : 0.f;
        q[u].w = i + 3 < i1 ? x[i + 3] : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t i = base + 1024 * u;
      add(q[u].x, i < i1);
      add(q[u].y, i + 1 < i1);
      add(q[u].z, i + 2 < i1);
      add(q[u].w, i + 3 < i1);
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    gt += __shfl_down(gt, o);
    eq += __shfl_down(eq, o);
  }
  __shared__ uint32_t sg[4], se[4];
  if ((threadIdx.x & 63) == 0) {
    sg[threadIdx.x >> 6] = gt;
    se[threadIdx.x >> 6] = eq;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    ws.cnt_gt[blockIdx.x] = sg[0] + sg[1] + sg[2] + sg[3];
    ws.cnt_eq[blockIdx.x] = se[0] + se[1] + se[2] + se[3];
  }
}

// exclusive prefix sum over a 256-thread block (4 waves); `wt` is a 4-entry
// LDS array private to this call site; returns the block total in `total`
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* wt, uint32_t& total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(inc, o, 64);
    if (lane >= o) inc += t;
  }
  if (lane == 63) wt[wave] = inc;
  __syncthreads();
  uint32_t before = 0;
#pragma unroll
  for (int w = 0; w < 4; ++w) before += w < wave ? wt[w] : 0u;
  total = wt[0] + wt[1] + wt[2] + wt[3];
  return before + inc - v;
}

// ordered compaction: a block owns [i0, i1); its output offsets are the sums
// of the counts of the blocks before it (computed here, in a fixed order);
// per iteration each thread takes 4 consecutive elements (one 16-byte load),
// tie ranks and output slots come from two block-wide exclusive scans
// (elements stay in ascending order)
template <bool CAND = false>
__global__ void __launch_bounds__(256)
write_kernel(const float* __restrict__ x, int64_t n, int64_t span, WS ws, uint32_t kk,
             int64_t* __restrict__ idx, float* __restrict__ vals, uint32_t* __restrict__ hint, Cand cd = Cand{},
             float hint_frac = 0.5f, uint32_t* __restrict__ clean_seg = nullptr) {
  __shared__ uint32_t tot[4], res[2];
  __shared__ uint32_t wt_eq[4], wt_sel[4];
  const int32_t* cmap = nullptr;  // candidate -> index (ascending)
  if constexpr (CAND) {
    if (cd.ctl[0] != 0u) {
      x = cd.val;
      n = cd.ctl[1];
      cmap = cd.idx;
    }
    span = cand_span(n);
  }
  const Walk wk = {ws.wk[4], ws.wk[5]};  // count_kernel's walk
  if (clean_seg != nullptr) {
    // persistent workspace: leave the histograms and segment totals zeroed
    // for the next call (nothing after count_kernel reads them)
    const int nt = static_cast<int>(gridDim.x) * 256, t0 = static_cast<int>(blockIdx.x) * 256 + threadIdx.x;
    for (int e = t0; e < 4 * kBins; e += nt) ws.hist[0][e] = 0u;  // hist[0..3] are contiguous
    for (int e = t0; e < kSegMax; e += nt) clean_seg[e] = 0u;
  }
  const uint32_t thr = wk.prefix, ties = wk.remaining;
  // next call's lower bound: hint_frac x this threshold (finite thresholds only)
  if (hint != nullptr && blockIdx.x == 0 && threadIdx.x == 0)
    hint[0] = thr < 0x7f800000u ? __float_as_uint(__uint_as_float(thr) * hint_frac) : 0u;
  // counts of the blocks before this one
  uint32_t g = 0, e = 0;
  for (int b = threadIdx.x; b < static_cast<int>(blockIdx.x); b += 256) {
    g += ws.cnt_gt[b];
    e += ws.cnt_eq[b];
  }
  uint32_t gt_before, eq_before;
  (void)block_excl_scan(g, wt_sel, gt_before);
  __syncthreads();
  (void)block_excl_scan(e, wt_eq, eq_before);
  __syncthreads();
  uint32_t sel_base = gt_before + min(eq_before, ties);
  uint32_t eq_base = eq_before;
  const int64_t i0 = blockIdx.x * span;
  const int64_t i1 = min(n, i0 + span);
  const bool al = (reinterpret_cast<uintptr_t>(x) & 15) == 0;
  // 4 steps of 1024 elements loaded at once (the steps are processed in
  // order); a step without any element >= thr -- almost all of them for a
  // k << n selection -- costs one block-wide OR instead of two scans
  constexpr int kU = 4;
  for (int64_t outer = i0; outer < i1; outer += 1024 * kU) {
    float vv[kU][4];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t i = outer + 1024 * u + 4 * threadIdx.x;
      if (al && i + 3 < i1) {
        const float4 q = *reinterpret_cast<const float4*>(x + i);
        vv[u][0] = q.x; vv[u][1] = q.y; vv[u][2] = q.z; vv[u][3] = q.w;
      } else {
#pragma unroll
        for (int t = 0; t < 4; ++t) vv[u][t] = i + t < i1 ? x[i + t] : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t base = outer + 1024 * u;
      if (base >= i1) break;  // block-uniform
      const int64_t i = base + 4 * threadIdx.x;
      uint32_t gtm = 0, eqm = 0;  // bit t: element i+t is > thr / == thr
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const uint32_t k = key_of(vv[u][t]);
        const bool in = i + t < i1;
        gtm |= (in && k > thr ? 1u : 0u) << t;
        eqm |= (in && k == thr ? 1u : 0u) << t;
      }
      if (!__syncthreads_or(static_cast<int>(gtm | eqm))) continue;
      uint32_t eq_tot, sel_tot;
      uint32_t er = eq_base + block_excl_scan(__popc(eqm), wt_eq, eq_tot);
      uint32_t selm = gtm;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        if ((eqm >> t) & 1u) {
          if (er < ties) selm |= 1u << t;
          ++er;
        }
      }
      uint32_t pos = sel_base + block_excl_scan(__popc(selm), wt_sel, sel_tot);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        if ((selm >> t) & 1u) {
          idx[pos] = (CAND && cmap != nullptr) ? static_cast<int64_t>(cmap[i + t]) : i + t;
          vals[pos] = vv[u][t];
          ++pos;
        }
      }
      sel_base += sel_tot;
      eq_base += eq_tot;
      __syncthreads();  // wt_eq / wt_sel reuse
    }
  }
}

// ---- candidate lists (the region sketch query's top-k) ----
// The producer of hist[0] (keys >= hint) also writes one 64-bit mask per
// 64-element chunk of x (bit l: key(x[64 q + l]) >= hint) and the per-segment
// popcount totals (segments of kSegC chunks, LDS-aggregated integer atomics).
// cand_compact_kernel then copies the keys >= hint -- for a hint of half the
// previous threshold a few times k, not n -- into an ascending-index list,
// and the four radix passes run over that list on 256 blocks: each pass's
// cost had been its 1,024-block prologue and the n-element stream, not the
// selection.  Exact fallbacks decided on the device (same result bitwise):
// fewer than k keys >= hint -> the compaction blocks add the fill-in
// histogram of the keys < hint (hist[3]) and the passes read x; more than
// `cap` candidates -> the passes read x.

struct CandWS {
  uint32_t* seg;       // kSegMax popcount totals
  uint32_t* ctl;       // [0] list in use, [1] its length, [2] fill-in mode (cand_scan_kernel)
  uint32_t* segpre;    // kSegMax exclusive prefix of seg (cand_scan_kernel)
  uint64_t* ballots;   // one mask per chunk
  int32_t* cidx;       // cap
  float* cval;         // cap
};

int64_t cand_cap(int64_t n) {
  const int64_t c = n / 8;
  return c < 4096 ? (n < 4096 ? n : 4096) : c;
}

CandWS carve_cand(void* base, int64_t n) {
  char* p = reinterpret_cast<char*>(base) + 4 * kBins * 4 + 2 * kNB * 4 + 64;
  CandWS c;
  c.seg = reinterpret_cast<uint32_t*>(p); p += kSegMax * 4;
  c.ctl = reinterpret_cast<uint32_t*>(p); p += 16;
  c.segpre = reinterpret_cast<uint32_t*>(p); p += kSegMax * 4;
  const int64_t nch = (n + 63) / 64;
  c.ballots = reinterpret_cast<uint64_t*>(p); p += nch * 8;
  const int64_t cap = cand_cap(n);
  c.cidx = reinterpret_cast<int32_t*>(p); p += ((cap * 4 + 15) / 16) * 16;
  c.cval = reinterpret_cast<float*>(p);
  return c;
}

// Small vectors (< 2,048 x 4,096 elements: the ResNet-9 headline's 6.57M):
// one kernel, each block deriving the mode and its segment's prefix itself
// (13.4 us at 6.57M against 4.7 + 11.1 for the scan pass + the kernel below).
// block = kSub chunks (4,096 elements) of one segment, 256 threads of 16
// consecutive elements (four 16-byte loads, all in flight at once); a
// thread's output slot is the candidates before its segment (segment
// totals), before its sub-range inside the segment (ballot popcounts) and
// before it inside the block (one scan)
constexpr int kSub = 64;
__global__ void __launch_bounds__(256)
cand_compact_small_kernel(const float* __restrict__ x, int64_t n, WS ws, CandWS cw, uint32_t kk,
                    const uint32_t* __restrict__ hint, int64_t cap) {
  __shared__ uint32_t h[kBins];
  __shared__ uint32_t wt[4], wt2[4], wt3[4];
  const int tid = threadIdx.x;
  const uint32_t lb = hint != nullptr ? hint[0] : 0u;
  const int nseg = static_cast<int>((n + 64 * kSegC - 1) / (64 * kSegC));
  const int64_t nch = (n + 63) / 64;
  const int64_t cb0 = static_cast<int64_t>(blockIdx.x) * kSub;  // first chunk of the block
  const int seg = static_cast<int>(cb0 / kSegC);
  const int64_t sc0 = static_cast<int64_t>(seg) * kSegC;        // first chunk of its segment
  // every block decides the mode from the same integer totals
  uint32_t ht = 0, mt = 0, mb = 0;
#pragma unroll
  for (int q = 0; q < kBins / 256; ++q) ht += ws.hist[0][tid + 256 * q];
  for (int s2 = tid; s2 < nseg; s2 += 256) {
    const uint32_t v = cw.seg[s2];
    mt += v;
    mb += s2 < seg ? v : 0u;
  }
  // chunks of the segment before this block (< kSegC - kSub of them)
  for (int64_t ch = sc0 + tid; ch < cb0; ch += 256) mb += static_cast<uint32_t>(__popcll(cw.ballots[ch]));
  uint32_t hist_total, m_total, before;
  (void)block_excl_scan(ht, wt, hist_total);
  (void)block_excl_scan(mt, wt2, m_total);
  (void)block_excl_scan(mb, wt3, before);
  const bool fill = hist_total < kk;
  const bool use = !fill && static_cast<int64_t>(m_total) <= cap;
  if (blockIdx.x == 0 && tid == 0) {
    cw.ctl[0] = use ? 1u : 0u;
    cw.ctl[1] = m_total;
  }
  if (!fill && !use) return;
  // this thread's 16 elements
  const int64_t e0 = cb0 * 64 + 16 * tid;
  if (fill) {  // hist[3]: the keys < hint of this block's elements (clamped loads)
    const bool al = (reinterpret_cast<uintptr_t>(x) & 15) == 0 && (n & 3) == 0;
    float v[16];
    if (al) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t i = min(e0 + 4 * u, n - 4);
        const float4 q = *reinterpret_cast<const float4*>(x + i);
        v[4 * u] = q.x; v[4 * u + 1] = q.y; v[4 * u + 2] = q.z; v[4 * u + 3] = q.w;
      }
    } else {
#pragma unroll
      for (int t = 0; t < 16; ++t) v[t] = x[min(e0 + t, n - 1)];
    }
    for (int b = tid; b < kBins; b += 256) h[b] = 0u;
    __syncthreads();
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const uint32_t k = key_of(v[t]);
      if (e0 + t < n && k < lb) atomicAdd(h + (k >> 20), 1u);
    }
    __syncthreads();
    for (int b = tid; b < kBins; b += 256)
      if (h[b] != 0u) atomicAdd(ws.hist[3] + b, h[b]);
    return;
  }
  // the candidates only: the ballot bits say which elements are >= hint, so
  // x is read at those (a few times k of n) instead of streamed whole
  const int64_t ch = cb0 + (tid >> 2);
  const uint64_t bal = cw.ballots[ch < nch ? ch : nch - 1];
  const uint32_t bits = (ch < nch) ? static_cast<uint32_t>(bal >> (16 * (tid & 3))) & 0xffffu : 0u;
  uint32_t blk_tot;
  uint32_t pos = before + block_excl_scan(static_cast<uint32_t>(__popc(bits)), wt, blk_tot);
  for (uint32_t b = bits; b != 0u; b &= b - 1u) {
    const int t = __builtin_ctz(b);
    cw.cidx[pos] = static_cast<int32_t>(e0 + t);
    cw.cval[pos] = x[e0 + t];
    ++pos;
  }
}

// One block, before the compaction: the mode (fill-in / candidate list /
// full-vector fallback) from the integer totals, and the segments' exclusive
// prefix -- every compaction block used to re-derive both from the 2,048 bins
// and all segment totals (~20 KB of prologue reads per 4,096-element block:
// the GPT-2 compaction took 320 us for 124M elements).
__device__ __forceinline__ uint32_t block_excl_scan1024(uint32_t v, uint32_t* wt, uint32_t& total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(inc, o, 64);
    if (lane >= o) inc += t;
  }
  if (lane == 63) wt[wave] = inc;
  __syncthreads();
  uint32_t before = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < 16; ++w) {
    before += w < wave ? wt[w] : 0u;
    tot += wt[w];
  }
  total = tot;
  return before + inc - v;
}

__global__ void __launch_bounds__(1024) cand_scan_kernel(WS ws, CandWS cw, int nseg, uint32_t kk, int64_t cap) {
  __shared__ uint32_t wt[16];
  const int tid = threadIdx.x;
  uint32_t ht = 0;
  for (int b = tid; b < kBins; b += 1024) ht += ws.hist[0][b];
  uint32_t hist_total;
  (void)block_excl_scan1024(ht, wt, hist_total);
  __syncthreads();
  uint32_t run = 0;
  for (int base = 0; base < nseg; base += 1024) {
    const int sg = base + tid;
    const uint32_t v = sg < nseg ? cw.seg[sg] : 0u;
    uint32_t tot;
    const uint32_t ex = block_excl_scan1024(v, wt, tot);
    if (sg < nseg) cw.segpre[sg] = run + ex;
    run += tot;
    __syncthreads();  // (wt reuse)
  }
  if (tid == 0) {
    const bool fill = hist_total < kk;
    const bool use = !fill && static_cast<int64_t>(run) <= cap;
    cw.ctl[0] = use ? 1u : 0u;
    cw.ctl[1] = run;
    cw.ctl[2] = fill ? 1u : 0u;
  }
}

// block = IT x 64 chunks (IT x 4,096 elements) of one segment, 256 threads
// of 16 consecutive elements per step (four 16-byte loads, all in flight at
// once); a thread's output slot is the segment's prefix (cand_scan_kernel),
// the ballot popcounts of the segment's chunks before the block, and one
// block scan per step
template <int IT>
__global__ void __launch_bounds__(256)
cand_compact_kernel(const float* __restrict__ x, int64_t n, WS ws, CandWS cw, const uint32_t* __restrict__ hint) {
  __shared__ uint32_t h[kBins];
  __shared__ uint32_t wt[4];
  const int tid = threadIdx.x;
  const bool fill = cw.ctl[2] != 0u, use = cw.ctl[0] != 0u;
  if (!fill && !use) return;
  const uint32_t lb = hint != nullptr ? hint[0] : 0u;
  const int64_t nch = (n + 63) / 64;
  const int64_t cb0 = static_cast<int64_t>(blockIdx.x) * 64 * IT;  // first chunk of the block
  const bool al = (reinterpret_cast<uintptr_t>(x) & 15) == 0 && (n & 3) == 0;
  auto load16 = [&](int64_t e0, float (&v)[16]) __attribute__((always_inline)) {
    if (al) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t i = min(e0 + 4 * u, n - 4);
        const float4 q = *reinterpret_cast<const float4*>(x + i);
        v[4 * u] = q.x; v[4 * u + 1] = q.y; v[4 * u + 2] = q.z; v[4 * u + 3] = q.w;
      }
    } else {
#pragma unroll
      for (int t = 0; t < 16; ++t) v[t] = x[min(e0 + t, n - 1)];
    }
  };
  if (fill) {  // hist[3]: the keys < hint of this block's elements
    for (int b = tid; b < kBins; b += 256) h[b] = 0u;
    __syncthreads();
    for (int it = 0; it < IT; ++it) {
      const int64_t e0 = (cb0 + 64 * it) * 64 + 16 * tid;
      float v[16];
      load16(e0, v);
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        const uint32_t k = key_of(v[t]);
        if (e0 + t < n && k < lb) atomicAdd(h + (k >> 20), 1u);
      }
    }
    __syncthreads();
    for (int b = tid; b < kBins; b += 256)
      if (h[b] != 0u) atomicAdd(ws.hist[3] + b, h[b]);
    return;
  }
  // candidates of the segment's chunks before this block (< kSegC of them)
  const int seg = static_cast<int>(cb0 / kSegC);
  uint32_t mb = 0;
  for (int64_t ch = static_cast<int64_t>(seg) * kSegC + tid; ch < cb0; ch += 256)
    mb += static_cast<uint32_t>(__popcll(cw.ballots[ch]));
  uint32_t before;
  (void)block_excl_scan(mb, wt, before);
  __syncthreads();
  uint32_t base = cw.segpre[seg] + before;
  for (int it = 0; it < IT; ++it) {
    const int64_t c0 = cb0 + 64 * it;
    if (c0 >= nch) break;  // (block-uniform)
    const int64_t e0 = c0 * 64 + 16 * tid;
    const int64_t ch = c0 + (tid >> 2);
    const uint64_t bal = cw.ballots[ch < nch ? ch : nch - 1];
    const uint32_t bits = (ch < nch) ? static_cast<uint32_t>(bal >> (16 * (tid & 3))) & 0xffffu : 0u;
    uint32_t tot;
    uint32_t pos = base + block_excl_scan(static_cast<uint32_t>(__popc(bits)), wt, tot);
    // (x read at the candidates only)
    for (uint32_t b = bits; b != 0u; b &= b - 1u) {
      const int t = __builtin_ctz(b);
      cw.cidx[pos] = static_cast<int32_t>(e0 + t);
      cw.cval[pos] = x[e0 + t];
      ++pos;
    }
    base += tot;
    __syncthreads();  // (wt reuse)
  }
}

}  // namespace

int64_t topk_workspace_bytes(int64_t) {
  return 4 * kBins * 4 + 2 * kNB * 4 + 64;
}

bool topk_cand_supported(int64_t n) {
  return n >= 64 && n <= static_cast<int64_t>(kSegMax) * 64 * kSegC && n < (int64_t{1} << 31);
}

int64_t topk_cand_workspace_bytes(int64_t n) {
  const int64_t cap = cand_cap(n);
  return 4 * kBins * 4 + 2 * kNB * 4 + 64 + kSegMax * 4 + 16 + kSegMax * 4 + ((n + 63) / 64) * 8 +
         ((cap * 4 + 15) / 16) * 16 + cap * 4;
}

void topk_cand_prepare(void* workspace, hipStream_t stream) {
  // histograms, block counts and segment totals (contiguous)
  tape_memset(workspace, 0, 4 * kBins * 4 + 2 * kNB * 4 + 64 + kSegMax * 4, stream);
}

void topk_cand_ptrs(void* workspace, int64_t n, uint64_t** ballots, uint32_t** seg) {
  const CandWS c = carve_cand(workspace, n);
  *ballots = c.ballots;
  *seg = c.seg;
}

void launch_topk_cand_rest(const float* x, int64_t n, int64_t k, int64_t* idx, float* vals, void* workspace,
                           hipStream_t stream, uint32_t* hint, bool persistent) {
  if (k <= 0 || n <= 0) return;
  WS w = carve(workspace);
  const CandWS cw = carve_cand(workspace, n);
  const uint32_t kk = static_cast<uint32_t>(k < n ? k : n);
  const int64_t nch = (n + 63) / 64;
  const int nseg = static_cast<int>((nch + kSegC - 1) / kSegC);
  // chunks per compaction block: the most (<= 16 x 64, a divisor of a
  // segment) that still leaves >= 2,048 blocks
  int it = 16;
  while (it > 1 && (nch + 64 * it - 1) / (64 * it) < 2048) it >>= 1;
  if (it == 1) {
    const int nblk = static_cast<int>((nch + kSub - 1) / kSub);
    COMMEFF_LAUNCH(cand_compact_small_kernel, dim3(nblk), dim3(256), 0, stream, x, n, w, cw, kk, hint,
                   cand_cap(n));
  } else {
    COMMEFF_LAUNCH(cand_scan_kernel, dim3(1), dim3(1024), 0, stream, w, cw, nseg, kk, cand_cap(n));
  }
  const dim3 grid(static_cast<uint32_t>((nch + 64 * it - 1) / (64 * it)));
  switch (it) {
    case 16: COMMEFF_LAUNCH(cand_compact_kernel<16>, grid, dim3(256), 0, stream, x, n, w, cw, hint); break;
    case 8: COMMEFF_LAUNCH(cand_compact_kernel<8>, grid, dim3(256), 0, stream, x, n, w, cw, hint); break;
    case 4: COMMEFF_LAUNCH(cand_compact_kernel<4>, grid, dim3(256), 0, stream, x, n, w, cw, hint); break;
    case 2: COMMEFF_LAUNCH(cand_compact_kernel<2>, grid, dim3(256), 0, stream, x, n, w, cw, hint); break;
    default: break;  // (the small-vector kernel above)
  }
  const Cand cd{cw.ctl, cw.cval, cw.cidx};
  constexpr int nb = 256;  // candidate passes (the fallbacks stream x on these too)
  COMMEFF_LAUNCH((hist_kernel<1, true>), dim3(nb), dim3(256), 0, stream, x, n, w, kk, hint, cd);
  COMMEFF_LAUNCH((hist_kernel<2, true>), dim3(nb), dim3(256), 0, stream, x, n, w, kk, hint, cd);
  COMMEFF_LAUNCH(count_kernel<true>, dim3(nb), dim3(256), 0, stream, x, n, int64_t{0}, w, kk, cd);
  // the candidate list holds the keys >= hint: a tighter bound than the
  // full-vector passes' 0.5 (a threshold that drops below it between calls
  // takes the exact fill-in fallback).  ResNet-9 FetchSGD round (k = 50,000 of
  // 6.57M): 0.5 -> ~815k candidates, 0.75 -> ~340k, 0.85 -> ~200k, fallbacks
  // only in the first two rounds for all three
  constexpr float frac = 0.85f;
  COMMEFF_LAUNCH(write_kernel<true>, dim3(nb), dim3(256), 0, stream, x, n, int64_t{0}, w, kk, idx, vals,
                     hint, cd, frac, persistent ? cw.seg : nullptr);
}

void launch_topk_abs(const float* x, int64_t n, int64_t k, int64_t* idx, float* vals,
                     void* workspace, hipStream_t stream, uint32_t* hint) {
  if (k <= 0 || n <= 0) return;
  topk_prepare(workspace, stream);
  WS w = carve(workspace);
  int hb = static_cast<int>((n + 1023) / 1024);
  if (hb > 1024) hb = 1024;
  if (hb < 1) hb = 1;
  const uint32_t kk = static_cast<uint32_t>(k < n ? k : n);
  COMMEFF_LAUNCH((hist_kernel<0, false>), dim3(hb), dim3(256), 0, stream, x, n, w, kk, hint, Cand{});
  launch_topk_abs_rest(x, n, k, idx, vals, workspace, stream, hint);
}

void topk_prepare(void* workspace, hipStream_t stream) {
  WS w = carve(workspace);
  tape_memset(w.hist[0], 0, 4 * kBins * 4, stream);
}

// the passes after the first histogram (hist[0] at the workspace start: keys
// >= hint[0] counted by their top 11 bits -- hist_kernel<0> or a producer
// kernel that saw every element, e.g. the region sketch query)
void launch_topk_abs_rest(const float* x, int64_t n, int64_t k, int64_t* idx, float* vals,
                          void* workspace, hipStream_t stream, uint32_t* hint) {
  if (k <= 0 || n <= 0) return;
  WS w = carve(workspace);
  int hb = static_cast<int>((n + 1023) / 1024);
  if (hb > 1024) hb = 1024;
  if (hb < 1) hb = 1;
  const uint32_t kk = static_cast<uint32_t>(k < n ? k : n);
  if (hint != nullptr)
    COMMEFF_LAUNCH((hist_kernel<3, false>), dim3(hb), dim3(256), 0, stream, x, n, w, kk, hint, Cand{});
  COMMEFF_LAUNCH((hist_kernel<1, false>), dim3(hb), dim3(256), 0, stream, x, n, w, kk, hint, Cand{});
  COMMEFF_LAUNCH((hist_kernel<2, false>), dim3(hb), dim3(256), 0, stream, x, n, w, kk, hint, Cand{});
  // compaction blocks: 1,024 (every block's prologue sums the counts of the
  // blocks before it), up to kNB for very long vectors (>= 32 K elements a
  // block: GPT-2 size 151 -> 128 us for the ordered write pass)
  int nb = static_cast<int>((n + 255) / 256);
  const int cap = static_cast<int>(std::min<int64_t>(kNB, std::max<int64_t>(1024, n / 32768)));
  if (nb > cap) nb = cap;
  int64_t span = (n + nb - 1) / nb;
  span = ((span + 1023) / 1024) * 1024;  // write_kernel: 1024 elements per block step
  nb = static_cast<int>((n + span - 1) / span);
  COMMEFF_LAUNCH(count_kernel<false>, dim3(nb), dim3(256), 0, stream, x, n, span, w, kk, Cand{});
  COMMEFF_LAUNCH(write_kernel<false>, dim3(nb), dim3(256), 0, stream, x, n, span, w, kk, idx, vals, hint,
                 Cand{}, 0.5f, static_cast<uint32_t*>(nullptr));
}

}  // namespace commeff
