// Fused streaming kernels of the federated round (gfx950).
//
//  momentum_ef   server V/E update           fed_aggregator.py:489-503,517-521,578-582 (K6)
//  sparse_apply  w[idx] -= lr*delta + track  fed_aggregator.py:455,613 (K12, K13)
//  dense_apply   w -= lr*delta + track       fed_aggregator.py:455,509,566 (K12, K13)
//  count_ge      download accounting         fed_aggregator.py:239-289 (K13)
//  l2norm        deterministic L2 norm       utils.py:305-313 (K14/K15)
//  clip_noise    DP clip + Gaussian noise    fed_worker.py:304-309 (K14)
//  client_state  local momentum / error      fed_worker.py:193-202 (K9)
//  zero_at       error/momentum masking      fed_worker.py:209-216, fed_aggregator.py:531-540 (K9, K11)
//  axpby         FedAvg local step / deltas  fed_worker.py:98-108 (K17)
//
// All streaming kernels use 16-byte vector accesses on aligned, length%4==0
// inputs (the flat parameter/gradient buffers always are) and a scalar tail.
#include <hip/hip_runtime.h>
#include <cstdint>
#include "kernels.h"
#include "region_hash.h"

namespace commeff {
namespace {

constexpr int kBlock = 256;

inline int grid_for(int64_t n, int max_blocks = 4096) {
  int64_t b = (n + kBlock - 1) / kBlock;
  if (b < 1) b = 1;
  return static_cast<int>(b < max_blocks ? b : max_blocks);
}

inline bool aligned16(const void* p) { return p == nullptr || (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// ----------------------------------------------------------- momentum / EF
__global__ void __launch_bounds__(kBlock)
momentum_ef_kernel(float4* __restrict__ V, float4* __restrict__ E, const float4* __restrict__ G,
                   int64_t n4, float rho, float gscale, int mode) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n4; i += stride) {
    float4 v = V[i], g = G[i];
    // explicit fmaf: the region query's fused momentum (sketch_region.hip)
    // must round identically
    v.x = fmaf(rho, v.x, gscale * g.x);
    v.y = fmaf(rho, v.y, gscale * g.y);
    v.z = fmaf(rho, v.z, gscale * g.z);
    v.w = fmaf(rho, v.w, gscale * g.w);
    V[i] = v;
    if (mode == 1) {
      float4 e = E[i];
      e.x += v.x; e.y += v.y; e.z += v.z; e.w += v.w;
      E[i] = e;
    } else if (mode == 2) {
      E[i] = v;
    }
  }
}

__global__ void momentum_ef_tail(float* V, float* E, const float* G, int64_t start, int64_t n,
                                 float rho, float gscale, int mode) {
  int64_t i = start + blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
  if (i >= n) return;
  float v = fmaf(rho, V[i], gscale * G[i]);
  V[i] = v;
  if (mode == 1) E[i] += v;
  else if (mode == 2) E[i] = v;
}

// ----------------------------------------------------------------- apply
// Change histogram for download accounting: hist[r + 1] = #{i : last_mod[i]
// == r} (bin 0: never changed).  A coordinate whose stamp moves from `from`
// to `round` leaves bin from+1 and enters bin round+1.  The moves of a block
// are first counted in an LDS window -- bin 0 and the kHistWin most recent
// rounds, where nearly all stamps live -- and flushed with one global atomic
// per nonzero bin; only stamps older than the window go to global memory
// directly.  A round's accounting is then a suffix sum over the bins
// (account_hist) instead of a pass over d stamps.
constexpr int kHistWin = 4095;  // LDS bins: [0] = never changed, [1..kHistWin] = recent rounds

struct HistWin {
  int32_t* lh;  // LDS, kHistWin + 1 bins
  int32_t round;
  // LDS slot of global bin b (b = from + 1), or -1 outside the window
  __device__ __forceinline__ int slot(int32_t b) const {
    if (b == 0) return 0;
    const int32_t off = b - (round + 1 - (kHistWin - 1));  // recent bins [round+2-kHistWin, round+1]
    return (off >= 0 && off < kHistWin) ? off + 1 : -1;
  }
  __device__ __forceinline__ int32_t bin(int s) const {
    return s == 0 ? 0 : round + 1 - (kHistWin - 1) + (s - 1);
  }
};

__device__ __forceinline__ void hist_init(int32_t* lh) {
  for (int b = threadIdx.x; b <= kHistWin; b += blockDim.x) lh[b] = 0;
  __syncthreads();
}

__device__ __forceinline__ void hist_move(const HistWin& hw, int32_t* hist, bool moved, int32_t from) {
  const int lane = threadIdx.x & 63;
  const uint64_t act = __ballot(moved);
  if (act == 0) return;
  const int leader = __ffsll(static_cast<long long>(act)) - 1;
  // every mover enters bin round+1; the leader's source bin (usually the
  // previous round) is aggregated over the wave, the rest one LDS atomic each
  const int32_t b0 = __shfl(from, leader) + 1;
  const uint64_t same = __ballot(moved && from + 1 == b0);
  if (lane == leader) {
    atomicAdd(hw.lh + hw.slot(hw.round + 1), static_cast<int32_t>(__popcll(act)));
    const int s0 = hw.slot(b0);
    if (s0 >= 0) atomicSub(hw.lh + s0, static_cast<int32_t>(__popcll(same)));
    else atomicSub(hist + b0, static_cast<int32_t>(__popcll(same)));
  }
  if (moved && from + 1 != b0) {
    const int s = hw.slot(from + 1);
    if (s >= 0) atomicSub(hw.lh + s, 1);
    else atomicSub(hist + from + 1, 1);
  }
}

__device__ __forceinline__ void hist_flush(const HistWin& hw, int32_t* hist) {
  __syncthreads();
  for (int s = threadIdx.x; s <= kHistWin; s += blockDim.x) {
    const int32_t v = hw.lh[s];
    const int32_t b = hw.bin(s);
    if (v != 0 && b >= 0) atomicAdd(hist + b, v);
  }
}

constexpr int kApplyBlock = 1024;

// ZERO: also the region sketch's heavy-hitter zeroing of the same list
// (cs_region_zero_kernel semantics: the r cells of every coordinate with a
// nonzero value, in t1 and t2) -- one launch fewer per server step
template <bool ZERO = false>
__global__ void __launch_bounds__(kApplyBlock)
sparse_apply_kernel(float* __restrict__ w, const int64_t* __restrict__ idx,
                    const float* __restrict__ vals, int64_t k, float lr,
                    const float* __restrict__ lr_vec, int32_t* __restrict__ last_mod,
                    int32_t round, const int32_t* __restrict__ step, int32_t* __restrict__ hist,
                    rh::RegionZero rz = rh::RegionZero{}) {
  __shared__ int32_t lh[kHistWin + 1];
  const int64_t q = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
  if (step != nullptr) {  // graph replay: [lr bits, round] from device memory
    lr = __int_as_float(step[0]);
    round = step[1];
  }
  const HistWin hw{lh, round};
  if (hist != nullptr) hist_init(lh);
  bool moved = false;
  int32_t from = 0;
  if (q < k) {
    const int64_t i = idx[q];
    const float l = lr_vec != nullptr ? lr_vec[i] : lr;
    const float old = w[i];
    const float vq = vals[q];
    const float nw = old - l * vq;
    w[i] = nw;
    if constexpr (ZERO) {
      // the rows' hash words loaded together (unconditional, clamped row):
      // one dependent-load latency per coordinate, not one per row
      const uint64_t ic = static_cast<uint64_t>(i) < rz.d ? static_cast<uint64_t>(i) : 0u;
      const uint32_t qc = static_cast<uint32_t>(ic / rz.m), o = static_cast<uint32_t>(ic - static_cast<uint64_t>(qc) * rz.m);
      uint32_t cw[rh::kZeroRows], pw[rh::kZeroRows];
#pragma unroll
      for (int j = 0; j < rh::kZeroRows; ++j) {
        const uint32_t jj = static_cast<uint32_t>(j) < rz.r ? static_cast<uint32_t>(j) : rz.r - 1;
        cw[j] = rz.cinfo[static_cast<size_t>(jj) * rz.nch + qc];
        pw[j] = rz.perm[jj * rz.m + o];
      }
      if (vq != 0.f && static_cast<uint64_t>(i) < rz.d) {
#pragma unroll
        for (int j = 0; j < rh::kZeroRows; ++j) {
          if (static_cast<uint32_t>(j) < rz.r) {
            const uint32_t region = rh::ci_region(cw[j]), grp = region / rz.g;
            if (grp >= rz.L.g0 && grp < rz.L.g1) {  // (sharded server: this rank's groups only)
              const size_t cell = rh::cell_at(region, rh::in_region(pw[j], cw[j], rz.m), j, rz.g, rz.m, rz.L);
              rz.t1[cell] = 0.f;
              if (rz.t2 != nullptr) rz.t2[cell] = 0.f;
            }
          }
        }
      }
    }
    if (last_mod != nullptr && nw != old) {
      from = last_mod[i];
      last_mod[i] = round;
      moved = from != round;
    }
  }
  if (hist != nullptr) {
    hist_move(hw, hist, moved, from);
    hist_flush(hw, hist);
  }
}

__global__ void __launch_bounds__(kApplyBlock)
dense_apply_kernel(float* __restrict__ w, const float* __restrict__ delta, int64_t n, float lr,
                   const float* __restrict__ lr_vec, int32_t* __restrict__ last_mod,
                   int32_t round, const int32_t* __restrict__ step, int32_t* __restrict__ hist) {
  __shared__ int32_t lh[kHistWin + 1];
  if (step != nullptr) {
    lr = __int_as_float(step[0]);
    round = step[1];
  }
  const HistWin hw{lh, round};
  if (hist != nullptr) hist_init(lh);
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  // wave-uniform trip count (hist_move uses wave ballots)
  for (int64_t base = blockIdx.x * static_cast<int64_t>(blockDim.x); base < n; base += stride) {
    const int64_t i = base + threadIdx.x;
    bool moved = false;
    int32_t from = 0;
    if (i < n) {
      const float l = lr_vec != nullptr ? lr_vec[i] : lr;
      const float old = w[i];
      const float nw = old - l * delta[i];
      w[i] = nw;
      if (last_mod != nullptr && nw != old) {
        from = last_mod[i];
        last_mod[i] = round;
        moved = from != round;
      }
    }
    if (hist != nullptr) hist_move(hw, hist, moved, from);
  }
  if (hist != nullptr) hist_flush(hw, hist);
}

// Round accounting from the change histogram (one block): per participating
// client j, dl[j] = 4 * #{i : last_mod[i] >= last_seen_j} = 4 * sum of bins
// >= last_seen_j + 1; running per-client totals updated.  meta = int64
// [last_seen (W) | clients (W)].
__global__ void __launch_bounds__(1024)
account_hist_kernel(const int32_t* __restrict__ hist, int nbins, const int64_t* __restrict__ meta,
                    int W, double* __restrict__ client_dl, double* __restrict__ client_ul,
                    double upc, double* __restrict__ dl) {
  __shared__ long long seg_suffix[1025];
  const int seg = (nbins + 1023) / 1024;
  const int t = threadIdx.x;
  long long s = 0;
  for (int b = t * seg; b < min(nbins, (t + 1) * seg); ++b) s += hist[b];
  seg_suffix[t] = s;
  if (t == 0) seg_suffix[1024] = 0;
  __syncthreads();
  // suffix scan over the 1024 segment sums (Hillis-Steele, in place)
  for (int off = 1; off < 1024; off <<= 1) {
    const long long v = t + off < 1024 ? seg_suffix[t + off] : 0;
    __syncthreads();
    seg_suffix[t] += v;
    __syncthreads();
  }
  const int64_t* clients = meta + W;
  for (int j = t; j < W; j += 1024) {
    int64_t b0 = meta[j] + 1;  // first counted bin
    if (b0 < 0) b0 = 0;
    long long cnt = 0;
    if (b0 < nbins) {
      const int sg = static_cast<int>(b0 / seg);
      cnt = seg_suffix[sg + 1];
      for (int64_t b = b0; b < min<int64_t>(nbins, static_cast<int64_t>(sg + 1) * seg); ++b) cnt += hist[b];
    }
    const double v = 4.0 * static_cast<double>(cnt);
    const int64_t c = clients[j];
    dl[j] = v;
    client_dl[c] += v;  // clients are unique within a round
    client_ul[c] += upc;
  }
}

// -------------------------------------------------------------- count_ge
__global__ void __launch_bounds__(kBlock)
count_ge_kernel(const int32_t* __restrict__ last_mod, int64_t n, const int32_t* __restrict__ thr,
                int T, unsigned long long* __restrict__ counts) {
  // counts[t] = #{i : last_mod[i] >= thr[t]}, thr ascending.  Histogram each
  // element into the number of thresholds it passes (upper-bound search), then
  // suffix-sum at the end (host side of the binding).
  __shared__ unsigned int h[1025];
  __shared__ int th[1024];
  for (int t = threadIdx.x; t <= T; t += blockDim.x) h[t] = 0;
  for (int t = threadIdx.x; t < T; t += blockDim.x) th[t] = thr[t];
  __syncthreads();
  // wave-aggregated histogram: most elements of a wave land in a few hot
  // bins, so one LDS atomic per distinct bin per wave (per-lane atomics on a
  // hot bin serialise)
  const int lane = threadIdx.x & 63;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t base = blockIdx.x * static_cast<int64_t>(blockDim.x); base < n; base += stride) {
    const int64_t i = base + threadIdx.x;
    int bin = 0;
    if (i < n) {
      const int v = last_mod[i];
      // number of thresholds <= v
      int lo = 0, hi = T;
      while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if (th[mid] <= v) lo = mid + 1; else hi = mid;
      }
      bin = lo;
    }
    unsigned long long pending = __ballot(bin > 0);
    while (pending) {  // wave-uniform
      const int leader = __ffsll(static_cast<long long>(pending)) - 1;
      const int b = __shfl(bin, leader);
      const unsigned long long same = __ballot(bin == b) & pending;
      if (lane == leader) atomicAdd(h + b, static_cast<unsigned>(__popcll(same)));
      pending &= ~same;
    }
  }
  __syncthreads();
  for (int t = threadIdx.x + 1; t <= T; t += blockDim.x)
    if (h[t]) atomicAdd(counts + t, static_cast<unsigned long long>(h[t]));
}

__global__ void count_ge_finish(unsigned long long* counts, int T, int64_t* out) {
  // element histogrammed into bin b passes thresholds 0..b-1 ->
  // out[t] = sum_{b > t} counts[b]
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    unsigned long long run = 0;
    for (int b = T; b >= 1; --b) {
      run += counts[b];
      out[b - 1] = static_cast<int64_t>(run);
    }
  }
}

// ------------------------------------------------------ round accounting
// Fused download/upload accounting of one round (ByteAccountant.round):
// per-block threshold histograms of last_mod (no global atomics: every block
// writes its whole histogram row), then one block sums the rows in a fixed
// order, suffix-sums them into counts[t] = #{i : last_mod[i] >= thr[t]} and
// charges each participating client.
__global__ void __launch_bounds__(kBlock)
count_partial_kernel(const int32_t* __restrict__ last_mod, int64_t n, const int64_t* __restrict__ thr,
                     int T, uint32_t* __restrict__ partial) {
  __shared__ unsigned int h[1025];
  __shared__ int th[1024];
  for (int t = threadIdx.x; t <= T; t += blockDim.x) h[t] = 0;
  for (int t = threadIdx.x; t < T; t += blockDim.x) th[t] = static_cast<int>(thr[t]);
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t base = blockIdx.x * static_cast<int64_t>(blockDim.x); base < n; base += stride) {
    const int64_t i = base + threadIdx.x;
    int bin = 0;
    if (i < n) {
      const int v = last_mod[i];
      int lo = 0, hi = T;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (th[mid] <= v) lo = mid + 1; else hi = mid;
      }
      bin = lo;
    }
    unsigned long long pending = __ballot(bin > 0);
    while (pending) {
      const int leader = __ffsll(static_cast<long long>(pending)) - 1;
      const int b = __shfl(bin, leader);
      const unsigned long long same = __ballot(bin == b) & pending;
      if (lane == leader) atomicAdd(h + b, static_cast<unsigned>(__popcll(same)));
      pending &= ~same;
    }
  }
  __syncthreads();
  uint32_t* row = partial + static_cast<size_t>(blockIdx.x) * (T + 1);
  for (int t = threadIdx.x; t <= T; t += blockDim.x) row[t] = h[t];
}

__global__ void __launch_bounds__(1024)
account_finish_kernel(const uint32_t* __restrict__ partial, int nb, int T, const int64_t* __restrict__ meta,
                      int W, double* __restrict__ client_dl, double* __restrict__ client_ul, double upc,
                      double* __restrict__ dl) {
  __shared__ uint32_t red[2048];
  __shared__ uint32_t cnt[1025];
  const int nbins = T + 1;
  const int parts = nbins >= 1024 ? 1 : 1024 / nbins;
  for (int e = threadIdx.x; e < parts * nbins; e += 1024) {
    const int part = e / nbins, bin = e - part * nbins;
    uint32_t s = 0;
#pragma unroll 4
    for (int b = part; b < nb; b += parts) s += partial[static_cast<size_t>(b) * nbins + bin];
    red[e] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    // bin b holds elements passing thresholds 0..b-1: cnt[t] = sum_{b > t} bins[b]
    uint32_t run = 0;
    for (int b = T; b >= 1; --b) {
      uint32_t v = 0;
      for (int q = 0; q < parts; ++q) v += red[q * nbins + b];
      run += v;
      cnt[b - 1] = run;
    }
  }
  __syncthreads();
  const int64_t* inv = meta + T;
  const int64_t* clients = meta + T + W;
  for (int j = threadIdx.x; j < W; j += 1024) {
    const double v = 4.0 * static_cast<double>(cnt[inv[j]]);
    const int64_t c = clients[j];
    dl[j] = v;
    client_dl[c] += v;  // clients are unique within a round
    client_ul[c] += upc;
  }
}

// ----------------------------------------------------------------- axpby
__global__ void __launch_bounds__(kBlock)
axpby_kernel(float* __restrict__ out, const float* __restrict__ a, float alpha,
             const float* __restrict__ b, float beta, int64_t n) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n; i += stride) {
    float v = alpha * a[i];
    if (b != nullptr) v += beta * b[i];
    out[i] = v;
  }
}

// ---------------------------------------------------------------- l2norm
__global__ void __launch_bounds__(kBlock)
sqsum_kernel(const float* __restrict__ x, int64_t n, float* __restrict__ partial) {
  float acc = 0.f;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n; i += stride) {
    float v = x[i];
    acc += v * v;
  }
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o);
  __shared__ float ws[kBlock / 64];
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int w = 0; w < kBlock / 64; ++w) s += ws[w];
    partial[blockIdx.x] = s;
  }
}

__global__ void __launch_bounds__(1024)
sqrt_sum_kernel(const float* __restrict__ partial, int nb, float* __restrict__ out) {
  __shared__ float s[1024];
  s[threadIdx.x] = threadIdx.x < nb ? partial[threadIdx.x] : 0.f;
  __syncthreads();
  for (int o = 512; o > 0; o >>= 1) {
    if (threadIdx.x < o) s[threadIdx.x] += s[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = sqrtf(s[0]);
}

// ------------------------------------------------------ Philox + clip_noise
struct U4 { uint32_t x, y, z, w; };

__device__ __forceinline__ U4 philox(uint64_t seed, uint64_t ctr) {
  uint32_t k0 = static_cast<uint32_t>(seed), k1 = static_cast<uint32_t>(seed >> 32);
  U4 c{static_cast<uint32_t>(ctr), static_cast<uint32_t>(ctr >> 32), 0u, 0u};
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0 = __umulhi(0xD2511F53u, c.x), lo0 = 0xD2511F53u * c.x;
    uint32_t hi1 = __umulhi(0xCD9E8D57u, c.z), lo1 = 0xCD9E8D57u * c.z;
    c = U4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

__device__ __forceinline__ float u01(uint32_t x) {
  return (static_cast<float>(x >> 8) + 0.5f) * (1.0f / 16777216.0f);
}

__global__ void __launch_bounds__(kBlock)
clip_noise_kernel(float* __restrict__ x, int64_t n, const float* __restrict__ norm, float clip,
                  float noise_std, uint64_t seed, uint64_t offset) {
  float scale = 1.f;
  if (clip > 0.f && norm != nullptr) {
    float nr = norm[0];
    if (nr > clip) scale = clip / nr;  // utils.py:clip_grad: record / (norm/clip)
  }
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n; i += stride) {
    float v = x[i] * scale;
    if (noise_std != 0.f) {
      U4 r = philox(seed, offset + static_cast<uint64_t>(i));
      float u1 = u01(r.x), u2 = u01(r.y);
      float z = sqrtf(-2.f * __logf(u1)) * __cosf(6.28318530718f * u2);
      v += noise_std * z;
    }
    x[i] = v;
  }
}

// ---------------------------------------------------------- client state
__global__ void __launch_bounds__(kBlock)
client_state_kernel(const float* __restrict__ g, float* __restrict__ u, float* __restrict__ e,
                    int64_t n, float rho) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n; i += stride) {
    float t = g[i];
    if (u != nullptr) {
      t = rho * u[i] + t;
      u[i] = t;
    }
    if (e != nullptr) e[i] += t;
  }
}

// The client's whole transmit tail in one pass (fed_worker.py:184-230 after
// utils.py:257-258 get_grad): t = scale (g + wd w); local momentum u = rho u +
// t (t = u); local error e += t; g = t only when there is neither (the
// transmit is then g itself).  Replaces axpby (weight decay) + a scale + the
// state update: 3 passes over g -> 1.  16-byte accesses (n % 4 == 0, aligned).
template <bool HAS_W, bool HAS_U, bool HAS_E>
__global__ void __launch_bounds__(kBlock)
client_tail_kernel(float4* __restrict__ g, const float4* __restrict__ w, float wd, float scale,
                   float4* __restrict__ u, float4* __restrict__ e, float rho, int64_t n4) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n4; i += stride) {
    float4 t = g[i];
    if constexpr (HAS_W) {
      const float4 x = w[i];
      t.x += wd * x.x; t.y += wd * x.y; t.z += wd * x.z; t.w += wd * x.w;
    }
    t.x *= scale; t.y *= scale; t.z *= scale; t.w *= scale;
    if constexpr (HAS_U) {
      const float4 m = u[i];
      t.x = rho * m.x + t.x; t.y = rho * m.y + t.y; t.z = rho * m.z + t.z; t.w = rho * m.w + t.w;
      u[i] = t;
    }
    if constexpr (HAS_E) {
      float4 r = e[i];
      r.x += t.x; r.y += t.y; r.z += t.z; r.w += t.w;
      e[i] = r;
    }
    if constexpr (!HAS_U && !HAS_E) g[i] = t;
  }
}

__global__ void __launch_bounds__(kBlock)
zero_at_kernel(float* a, float* b, float* c, const int64_t* __restrict__ idx, int64_t k) {
  int64_t q = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
  if (q >= k) return;
  int64_t i = idx[q];
  if (a) a[i] = 0.f;
  if (b) b[i] = 0.f;
  if (c) c[i] = 0.f;
}

__global__ void __launch_bounds__(kBlock)
scatter_kernel(float* __restrict__ out, const int64_t* __restrict__ idx,
               const float* __restrict__ vals, int64_t k) {
  int64_t q = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
  if (q < k) out[idx[q]] = vals[q];
}

}  // namespace

void launch_momentum_ef(float* V, float* E, const float* G, int64_t n, float rho, float gscale,
                        int mode, hipStream_t stream) {
  if (n <= 0) return;
  int64_t n4 = (aligned16(V) && aligned16(E) && aligned16(G)) ? n / 4 : 0;
  if (n4 > 0)
    COMMEFF_LAUNCH(momentum_ef_kernel, dim3(grid_for(n4)), dim3(kBlock), 0, stream,
                       reinterpret_cast<float4*>(V), reinterpret_cast<float4*>(E),
                       reinterpret_cast<const float4*>(G), n4, rho, gscale, mode);
  int64_t start = n4 * 4;
  if (start < n)
    COMMEFF_LAUNCH(momentum_ef_tail, dim3((n - start + kBlock - 1) / kBlock), dim3(kBlock), 0,
                       stream, V, E, G, start, n, rho, gscale, mode);
}

void launch_sparse_apply(float* w, const int64_t* idx, const float* vals, int64_t k, float lr,
                         const float* lr_vec, int32_t* last_mod, int32_t round,
                         const int32_t* step, int32_t* hist, hipStream_t stream) {
  if (k <= 0) return;
  COMMEFF_LAUNCH(sparse_apply_kernel<false>, dim3((k + kApplyBlock - 1) / kApplyBlock), dim3(kApplyBlock),
                     0, stream, w, idx, vals, k, lr, lr_vec, last_mod, round, step, hist, rh::RegionZero{});
}

void launch_sparse_apply_region_zero(float* w, const int64_t* idx, const float* vals, int64_t k, float lr,
                                     const float* lr_vec, int32_t* last_mod, int32_t round, const int32_t* step,
                                     int32_t* hist, float* t1, float* t2, const uint32_t* perm,
                                     const uint32_t* cinfo, int r, int64_t g, int64_t m, int64_t nch, int64_t d,
                                     RegionLayout L, hipStream_t stream) {
  if (k <= 0) return;
  const rh::RegionZero rz{t1, t2, perm, cinfo, static_cast<uint32_t>(r), static_cast<uint32_t>(g),
                          static_cast<uint32_t>(m), static_cast<uint32_t>(nch), static_cast<uint64_t>(d), L};
  // 256-thread blocks: 4x the blocks of the plain apply for the scattered zeroing
  COMMEFF_LAUNCH(sparse_apply_kernel<true>, dim3((k + 255) / 256), dim3(256), 0, stream, w, idx, vals, k, lr,
                 lr_vec, last_mod, round, step, hist, rz);
}

void launch_dense_apply(float* w, const float* delta, int64_t n, float lr, const float* lr_vec,
                        int32_t* last_mod, int32_t round, const int32_t* step, int32_t* hist,
                        hipStream_t stream) {
  if (n <= 0) return;
  int64_t nb = (n + kApplyBlock - 1) / kApplyBlock;
  if (nb > 512) nb = 512;  // each block flushes its LDS histogram window once
  COMMEFF_LAUNCH(dense_apply_kernel, dim3(static_cast<int>(nb)), dim3(kApplyBlock), 0, stream, w,
                     delta, n, lr, lr_vec, last_mod, round, step, hist);
}

void launch_account_hist(const int32_t* hist, int nbins, const int64_t* meta, int W,
                         double* client_dl, double* client_ul, double upc, double* dl,
                         hipStream_t stream) {
  if (W <= 0) return;
  COMMEFF_LAUNCH(account_hist_kernel, dim3(1), dim3(1024), 0, stream, hist, nbins, meta, W,
                     client_dl, client_ul, upc, dl);
}

void launch_count_ge(const int32_t* last_mod, int64_t n, const int32_t* thr, int T, int64_t* counts,
                     hipStream_t stream) {
  // counts must hold 2*(T+1) int64: [0, T+1) scratch bins, [T+1, 2T+1) output
  if (T <= 0) return;
  unsigned long long* bins = reinterpret_cast<unsigned long long*>(counts);
  tape_memset(bins, 0, (T + 1) * sizeof(unsigned long long), stream);
  COMMEFF_LAUNCH(count_ge_kernel, dim3(grid_for(n, 1024)), dim3(kBlock), 0, stream, last_mod,
                     n, thr, T, bins);
  COMMEFF_LAUNCH(count_ge_finish, dim3(1), dim3(64), 0, stream, bins, T, counts + T + 1);
}

int account_round_blocks(int64_t n) { return grid_for(n, 256); }

void launch_account_round(const int32_t* last_mod, int64_t n, const int64_t* meta, int T, int W,
                          uint32_t* partial, double* client_dl, double* client_ul, double upc,
                          double* dl, hipStream_t stream) {
  const int nb = account_round_blocks(n);
  if (T > 0)
    COMMEFF_LAUNCH(count_partial_kernel, dim3(nb), dim3(kBlock), 0, stream, last_mod, n, meta, T,
                       partial);
  COMMEFF_LAUNCH(account_finish_kernel, dim3(1), dim3(1024), 0, stream, partial, T > 0 ? nb : 0, T,
                     meta, W, client_dl, client_ul, upc, dl);
}

void launch_axpby(float* out, const float* a, float alpha, const float* b, float beta, int64_t n,
                  hipStream_t stream) {
  if (n <= 0) return;
  COMMEFF_LAUNCH(axpby_kernel, dim3(grid_for(n)), dim3(kBlock), 0, stream, out, a, alpha, b,
                     beta, n);
}

void launch_l2norm(const float* x, int64_t n, float* partial, float* out, hipStream_t stream) {
  int nb = grid_for(n, 1024);
  COMMEFF_LAUNCH(sqsum_kernel, dim3(nb), dim3(kBlock), 0, stream, x, n, partial);
  COMMEFF_LAUNCH(sqrt_sum_kernel, dim3(1), dim3(1024), 0, stream, partial, nb, out);
}

void launch_clip_noise(float* x, int64_t n, const float* norm, float clip, float noise_std,
                       uint64_t seed, uint64_t offset, hipStream_t stream) {
  if (n <= 0) return;
  COMMEFF_LAUNCH(clip_noise_kernel, dim3(grid_for(n)), dim3(kBlock), 0, stream, x, n, norm,
                     clip, noise_std, seed, offset);
}

void launch_client_state(const float* g, float* u, float* e, int64_t n, float rho,
                         hipStream_t stream) {
  if (n <= 0) return;
  COMMEFF_LAUNCH(client_state_kernel, dim3(grid_for(n)), dim3(kBlock), 0, stream, g, u, e, n,
                     rho);
}

void launch_client_tail(float* g, const float* w, float wd, float scale, float* u, float* e, float rho,
                        int64_t n, hipStream_t stream) {
  if (n <= 0) return;
  const int64_t n4 = n / 4;
  auto g4 = reinterpret_cast<float4*>(g);
  auto w4 = reinterpret_cast<const float4*>(w);
  auto u4 = reinterpret_cast<float4*>(u), e4 = reinterpret_cast<float4*>(e);
  const dim3 grid(grid_for(n4)), block(kBlock);
  const int key = (w != nullptr ? 4 : 0) | (u != nullptr ? 2 : 0) | (e != nullptr ? 1 : 0);
  switch (key) {
#define CT_CASE(K, HW, HU, HE) \
    case K: COMMEFF_LAUNCH((client_tail_kernel<HW, HU, HE>), grid, block, 0, stream, g4, w4, wd, scale, u4, e4, rho, n4); break;
    CT_CASE(0, false, false, false) CT_CASE(1, false, false, true) CT_CASE(2, false, true, false)
    CT_CASE(3, false, true, true) CT_CASE(4, true, false, false) CT_CASE(5, true, false, true)
    CT_CASE(6, true, true, false) CT_CASE(7, true, true, true)
#undef CT_CASE
  }
}

void launch_zero_at(float* a, float* b, float* c, const int64_t* idx, int64_t k,
                    hipStream_t stream) {
  if (k <= 0) return;
  COMMEFF_LAUNCH(zero_at_kernel, dim3((k + kBlock - 1) / kBlock), dim3(kBlock), 0, stream, a,
                     b, c, idx, k);
}

void launch_scatter_dense(float* out, int64_t n, const int64_t* idx, const float* vals, int64_t k,
                          hipStream_t stream) {
  tape_memset(out, 0, n * sizeof(float), stream);
  if (k <= 0) return;
  COMMEFF_LAUNCH(scatter_kernel, dim3((k + kBlock - 1) / kBlock), dim3(kBlock), 0, stream, out,
                     idx, vals, k);
}

}  // namespace commeff
