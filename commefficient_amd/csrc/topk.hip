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
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x * 4;
  // 16-byte loads where possible
  const int64_t n4 = (reinterpret_cast<uintptr_t>(x) & 15) == 0 ? (n / 4) * 4 : 0;
  for (int64_t i = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) * 4; i < n4;
       i += stride) {
    float4 v = *reinterpret_cast<const float4*>(x + i);
    float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      uint32_t k = key_of(vv[q]);
      if (PASS == 0) {
        atomicAdd(h + (k >> 20), 1u);
      } else if (PASS == 1) {
        if ((k >> 20) == prefix) atomicAdd(h + ((k >> 9) & 0x7ff), 1u);
      } else {
        if ((k >> 9) == prefix) atomicAdd(h + (k & 0x1ff), 1u);
      }
    }
  }
  for (int64_t i = n4 + static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    uint32_t k = key_of(x[i]);
    if (PASS == 0) {
      atomicAdd(h + (k >> 20), 1u);
    } else if (PASS == 1) {
      if ((k >> 20) == prefix) atomicAdd(h + ((k >> 9) & 0x7ff), 1u);
    } else {
      if ((k >> 9) == prefix) atomicAdd(h + (k & 0x1ff), 1u);
    }
  }
  __syncthreads();
  for (int b = threadIdx.x; b < kBins; b += blockDim.x) {
    uint32_t c = h[b];
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
  for (int64_t i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
    uint32_t k = key_of(x[i]);
    gt += k > thr;
    eq += k == thr;
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
  __shared__ uint32_t wsel[4], weq[4];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const uint64_t lt_mask = lane ? (~0ull >> (64 - lane)) : 0ull;
  for (int64_t base = i0; base < i1; base += blockDim.x) {
    int64_t i = base + threadIdx.x;
    float v = 0.f;
    uint32_t k = 0;
    bool in = i < i1;
    if (in) {
      v = x[i];
      k = key_of(v);
    }
    bool gt = in && k > thr;
    bool eq = in && k == thr;
    uint64_t bal_eq = __ballot(eq);
    // tie rank needs the eq-prefix first
    uint32_t eq_lane = __popcll(bal_eq & lt_mask);
    if (lane == 0) weq[wave] = __popcll(bal_eq);
    __syncthreads();
    uint32_t eq_wave = 0;
    for (int w = 0; w < wave; ++w) eq_wave += weq[w];
    uint32_t eq_tot = weq[0] + weq[1] + weq[2] + weq[3];
    uint32_t tie_rank = eq_base + eq_wave + eq_lane;
    bool sel = gt || (eq && tie_rank < ties);
    uint64_t bal_sel = __ballot(sel);
    uint32_t sel_lane = __popcll(bal_sel & lt_mask);
    if (lane == 0) wsel[wave] = __popcll(bal_sel);
    __syncthreads();
    uint32_t sel_wave = 0;
    for (int w = 0; w < wave; ++w) sel_wave += wsel[w];
    uint32_t sel_tot = wsel[0] + wsel[1] + wsel[2] + wsel[3];
    if (sel) {
      uint32_t pos = sel_base + sel_wave + sel_lane;
      idx[pos] = i;
      vals[pos] = v;
    }
    sel_base += sel_tot;
    eq_base += eq_tot;
    __syncthreads();  // wsel/weq reuse
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
  span = ((span + 255) / 256) * 256;
  nb = static_cast<int>((n + span - 1) / span);
  hipLaunchKernelGGL(count_kernel, dim3(nb), dim3(256), 0, stream, x, n, span, w.st, w.cnt_gt,
                     w.cnt_eq);
  hipLaunchKernelGGL(scan_kernel, dim3(1), dim3(kNB), 0, stream, nb, w.st, w.cnt_gt, w.cnt_eq,
                     w.off_sel, w.off_eq);
  hipLaunchKernelGGL(write_kernel, dim3(nb), dim3(256), 0, stream, x, n, span, w.st, w.off_sel,
                     w.off_eq, idx, vals);
}

}  // namespace commeff
