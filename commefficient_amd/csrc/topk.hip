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
//   three histogram passes over 11/11/9-bit digits of the key, each followed
//   by a one-workgroup "select" kernel that walks the histogram from the top
//   and fixes the next digit of the k-th largest key T (state in device
//   memory);  then a count pass (per-block #>T, #==T), a one-workgroup scan,
//   and an ordered compaction pass that uses wave ballots for intra-block
//   prefix sums.  Histograms are privatised in LDS; only non-empty bins are
//   flushed to global memory with atomics.
#include <hip/hip_runtime.h>
#include <cstdint>
#include "kernels.h"

namespace commeff {
namespace {

constexpr int kBins = 2048;
constexpr int kNB = 1024;  // blocks for count/write passes (upper bound)

struct State {
  uint32_t prefix;     // key bits fixed so far (right-aligned)
  uint32_t remaining;  // how many still needed among keys matching prefix
  uint32_t thr;        // final threshold key
  uint32_t ties;       // number of keys == thr to take
};

struct WS {
  uint32_t* hist;   // kBins
  State* st;
  uint32_t* cnt_gt; // kNB
  uint32_t* cnt_eq; // kNB
  uint32_t* off_sel;// kNB: selected before block
  uint32_t* off_eq; // kNB: ties before block
};

WS carve(void* base) {
  char* p = reinterpret_cast<char*>(base);
  WS w;
  w.hist = reinterpret_cast<uint32_t*>(p); p += kBins * 4;
  w.st = reinterpret_cast<State*>(p); p += 256;
  w.cnt_gt = reinterpret_cast<uint32_t*>(p); p += kNB * 4;
  w.cnt_eq = reinterpret_cast<uint32_t*>(p); p += kNB * 4;
  w.off_sel = reinterpret_cast<uint32_t*>(p); p += kNB * 4;
  w.off_eq = reinterpret_cast<uint32_t*>(p); p += kNB * 4;
  return w;
}

__device__ __forceinline__ uint32_t key_of(float x) {
  return __float_as_uint(x) & 0x7fffffffu;
}

// PASS 0: digit = key >> 20 (11 bits)
// PASS 1: digit = (key >> 9) & 0x7ff, needs (key >> 20) == prefix
// PASS 2: digit = key & 0x1ff,         needs (key >> 9)  == prefix
template <int PASS>
__global__ void __launch_bounds__(256)
hist_kernel(const float* __restrict__ x, int64_t n, uint32_t* __restrict__ hist,
            const State* __restrict__ st) {
  __shared__ uint32_t h[kBins];
  for (int b = threadIdx.x; b < kBins; b += blockDim.x) h[b] = 0;
  __syncthreads();
  const uint32_t prefix = PASS == 0 ? 0u : st->prefix;
  // (LDS atomics retire ~0.4 lanes/clk/CU and bound pass 0; per-wave
  // sub-histograms measured no faster, wave-aggregated atomics 4x slower:
  // normal-ish data spreads a wave over too many distinct bins)
  auto add = [&](float v, bool in) __attribute__((always_inline)) {
    if (!in) return;
    const uint32_t k = key_of(v);
    if (PASS == 0) {
      atomicAdd(h + (k >> 20), 1u);
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
  for (int b = threadIdx.x; b < kBins; b += blockDim.x) {
    const uint32_t c = h[b];
    if (c) atomicAdd(hist + b, c);
  }
}

// One workgroup of 256 threads.  Finds the bin holding the `remaining`-th
// largest key among the histogrammed ones, updates prefix/remaining and
// zeroes the histogram for the next pass.
template <int PASS>
__global__ void __launch_bounds__(256)
select_kernel(uint32_t* __restrict__ hist, State* __restrict__ st, uint32_t k_init) {
  constexpr int nbins = PASS == 2 ? 512 : 2048;
  constexpr int per = nbins / 256;  // bins per thread (8 or 2)
  __shared__ uint32_t tot[256];
  __shared__ uint32_t found_bin, found_above;
  const uint32_t remaining = PASS == 0 ? k_init : st->remaining;
  // thread t owns bins [nbins-1 - t*per - (per-1), nbins-1 - t*per]: scanning
  // from the top means thread 0 has the largest bins.
  uint32_t c[per];
  uint32_t s = 0;
#pragma unroll
  for (int q = 0; q < per; ++q) {
    int b = nbins - 1 - (threadIdx.x * per + q);
    c[q] = hist[b];
    s += c[q];
  }
  tot[threadIdx.x] = s;
  __syncthreads();
  // exclusive prefix over threads (Hillis-Steele in LDS, 8 steps)
  for (int o = 1; o < 256; o <<= 1) {
    uint32_t v = threadIdx.x >= o ? tot[threadIdx.x - o] : 0u;
    __syncthreads();
    tot[threadIdx.x] += v;
    __syncthreads();
  }
  uint32_t above = threadIdx.x ? tot[threadIdx.x - 1] : 0u;  // keys in higher bins
  if (threadIdx.x == 0) {
    found_bin = 0;
    found_above = 0;
  }
  __syncthreads();
  if (above < remaining && above + s >= remaining) {
    uint32_t run = above;
#pragma unroll
    for (int q = 0; q < per; ++q) {
      if (run + c[q] >= remaining) {
        found_bin = nbins - 1 - (threadIdx.x * per + q);
        found_above = run;
        break;
      }
      run += c[q];
    }
  }
  __syncthreads();
  // zero the histogram for the next pass / next call
  for (int b = threadIdx.x; b < kBins; b += 256) hist[b] = 0;
  if (threadIdx.x == 0) {
    uint32_t prefix = PASS == 0 ? 0u : st->prefix;
    const int bits = PASS == 2 ? 9 : 11;
    prefix = (prefix << bits) | found_bin;
    st->prefix = prefix;
    st->remaining = remaining - found_above;
    if (PASS == 2) {
      st->thr = prefix;
      st->ties = remaining - found_above;
    }
  }
}

__global__ void __launch_bounds__(256)
count_kernel(const float* __restrict__ x, int64_t n, int64_t span,
             const State* __restrict__ st, uint32_t* __restrict__ cnt_gt,
             uint32_t* __restrict__ cnt_eq) {
  const uint32_t thr = st->thr;
  const int64_t i0 = blockIdx.x * span;
  const int64_t i1 = min(n, i0 + span);
  uint32_t gt = 0, eq = 0;
  for (int64_t i = i0 + threadIdx.x; i < i1; i += 4 * blockDim.x) {
    float v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = i + u * blockDim.x < i1 ? x[i + u * blockDim.x] : 0.f;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint32_t k = key_of(v[u]);
      const bool in = i + u * blockDim.x < i1;
      gt += in && k > thr;
      eq += in && k == thr;
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
    cnt_gt[blockIdx.x] = sg[0] + sg[1] + sg[2] + sg[3];
    cnt_eq[blockIdx.x] = se[0] + se[1] + se[2] + se[3];
  }
}

__global__ void __launch_bounds__(1024)
scan_kernel(int nb, const State* __restrict__ st, const uint32_t* __restrict__ cnt_gt,
            const uint32_t* __restrict__ cnt_eq, uint32_t* __restrict__ off_sel,
            uint32_t* __restrict__ off_eq) {
  __shared__ uint32_t a[kNB], b[kNB];
  const int t = threadIdx.x;
  a[t] = t < nb ? cnt_gt[t] : 0u;
  b[t] = t < nb ? cnt_eq[t] : 0u;
  __syncthreads();
  for (int o = 1; o < kNB; o <<= 1) {
    uint32_t va = t >= o ? a[t - o] : 0u;
    uint32_t vb = t >= o ? b[t - o] : 0u;
    __syncthreads();
    a[t] += va;
    b[t] += vb;
    __syncthreads();
  }
  if (t < nb) {
    uint32_t gt_before = t ? a[t - 1] : 0u;
    uint32_t eq_before = t ? b[t - 1] : 0u;
    uint32_t ties = st->ties;
    off_sel[t] = gt_before + min(eq_before, ties);
    off_eq[t] = eq_before;
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

// ordered compaction: a block owns [i0, i1); per iteration each thread takes
// 4 consecutive elements (one 16-byte load), tie ranks and output slots come
// from two block-wide exclusive scans (elements stay in ascending order)
__global__ void __launch_bounds__(256)
write_kernel(const float* __restrict__ x, int64_t n, int64_t span,
             const State* __restrict__ st, const uint32_t* __restrict__ off_sel,
             const uint32_t* __restrict__ off_eq, int64_t* __restrict__ idx,
             float* __restrict__ vals) {
  const uint32_t thr = st->thr;
  const uint32_t ties = st->ties;
  const int64_t i0 = blockIdx.x * span;
  const int64_t i1 = min(n, i0 + span);
  uint32_t sel_base = off_sel[blockIdx.x];
  uint32_t eq_base = off_eq[blockIdx.x];
  __shared__ uint32_t wt_eq[4], wt_sel[4];
  const bool al = (reinterpret_cast<uintptr_t>(x) & 15) == 0;
  for (int64_t base = i0; base < i1; base += 1024) {
    const int64_t i = base + 4 * threadIdx.x;
    float v[4];
    if (al && i + 3 < i1) {
      const float4 q = *reinterpret_cast<const float4*>(x + i);
      v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = i + u < i1 ? x[i + u] : 0.f;
    }
    uint32_t gtm = 0, eqm = 0;  // bit u: element i+u is > thr / == thr
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint32_t k = key_of(v[u]);
      const bool in = i + u < i1;
      gtm |= (in && k > thr ? 1u : 0u) << u;
      eqm |= (in && k == thr ? 1u : 0u) << u;
    }
    uint32_t eq_tot, sel_tot;
    uint32_t er = eq_base + block_excl_scan(__popc(eqm), wt_eq, eq_tot);
    uint32_t selm = gtm;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if ((eqm >> u) & 1u) {
        if (er < ties) selm |= 1u << u;
        ++er;
      }
    }
    uint32_t pos = sel_base + block_excl_scan(__popc(selm), wt_sel, sel_tot);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if ((selm >> u) & 1u) {
        idx[pos] = i + u;
        vals[pos] = v[u];
        ++pos;
      }
    }
    sel_base += sel_tot;
    eq_base += eq_tot;
    __syncthreads();  // wt_eq / wt_sel reuse
  }
}

}  // namespace

int64_t topk_workspace_bytes(int64_t) {
  return kBins * 4 + 256 + 4 * kNB * 4;
}

void launch_topk_abs(const float* x, int64_t n, int64_t k, int64_t* idx, float* vals,
                     void* workspace, hipStream_t stream) {
  if (k <= 0 || n <= 0) return;
  WS w = carve(workspace);
  (void)hipMemsetAsync(w.hist, 0, kBins * 4, stream);
  int hb = static_cast<int>((n + 1023) / 1024);
  if (hb > 1024) hb = 1024;
  if (hb < 1) hb = 1;
  uint32_t kk = static_cast<uint32_t>(k < n ? k : n);
  hipLaunchKernelGGL(hist_kernel<0>, dim3(hb), dim3(256), 0, stream, x, n, w.hist, w.st);
  hipLaunchKernelGGL(select_kernel<0>, dim3(1), dim3(256), 0, stream, w.hist, w.st, kk);
  hipLaunchKernelGGL(hist_kernel<1>, dim3(hb), dim3(256), 0, stream, x, n, w.hist, w.st);
  hipLaunchKernelGGL(select_kernel<1>, dim3(1), dim3(256), 0, stream, w.hist, w.st, kk);
  hipLaunchKernelGGL(hist_kernel<2>, dim3(hb), dim3(256), 0, stream, x, n, w.hist, w.st);
  hipLaunchKernelGGL(select_kernel<2>, dim3(1), dim3(256), 0, stream, w.hist, w.st, kk);
  int nb = static_cast<int>((n + 255) / 256);
  if (nb > kNB) nb = kNB;
  int64_t span = (n + nb - 1) / nb;
  span = ((span + 1023) / 1024) * 1024;  // write_kernel: 1024 elements per block step
  nb = static_cast<int>((n + span - 1) / span);
  hipLaunchKernelGGL(count_kernel, dim3(nb), dim3(256), 0, stream, x, n, span, w.st, w.cnt_gt,
                     w.cnt_eq);
  hipLaunchKernelGGL(scan_kernel, dim3(1), dim3(kNB), 0, stream, nb, w.st, w.cnt_gt, w.cnt_eq,
                     w.off_sel, w.off_eq);
  hipLaunchKernelGGL(write_kernel, dim3(nb), dim3(256), 0, stream, x, n, span, w.st, w.off_sel,
                     w.off_eq, idx, vals);
}

}  // namespace commeff
