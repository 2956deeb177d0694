// Fused per-example cross-entropy for the CV loss (reference cv_train.py:31-84
// compute_loss_ce / Correct): one wave per example computes, in one pass over
// its logits row, the per-example loss lse(x) - x[t], top-1 correctness
// (argmax with ties to the lower index, like torch.argmax) and the unit
// gradient softmax(x) - onehot(t) (scaled by dL/dloss in backward).  Replaces
// log_softmax / nll / argmax / eq / cast kernels forward and backward.  Rows
// whose target is outside [0, C) (the LM's ignore label -100) get zero loss and
// gradient: the GPT-2 LM loss at the labelled positions (train/losses.py).
#include <hip/hip_runtime.h>
#include <cstdint>
#include "kernels.h"

namespace commeff {
namespace {

template <typename T>
__device__ __forceinline__ float ld(const T* p, int64_t i);
template <>
__device__ __forceinline__ float ld<float>(const float* p, int64_t i) { return p[i]; }
template <>
__device__ __forceinline__ float ld<uint16_t>(const uint16_t* p, int64_t i) {
  return __uint_as_float(static_cast<uint32_t>(p[i]) << 16);
}
template <typename T>
__device__ __forceinline__ void st(T* p, int64_t i, float v);
template <>
__device__ __forceinline__ void st<float>(float* p, int64_t i, float v) { p[i] = v; }
template <>
__device__ __forceinline__ void st<uint16_t>(uint16_t* p, int64_t i, float v) {
  const __bf16 b = static_cast<__bf16>(v);
  p[i] = __builtin_bit_cast(uint16_t, b);
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <typename T>
__global__ void __launch_bounds__(256) ce_fwd_kernel(const T* __restrict__ x,
                                                     const int64_t* __restrict__ tgt, int64_t B,
                                                     int C, float* __restrict__ loss,
                                                     float* __restrict__ correct,
                                                     T* __restrict__ grad) {
  const int lane = threadIdx.x & 63;
  const int64_t row = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (row >= B) return;
  const T* xr = x + row * C;
  const int64_t t = tgt[row];
  if (t < 0 || t >= C) {  // ignored row (label -100): zero loss and gradient
    if (lane == 0) {
      loss[row] = 0.f;
      correct[row] = 0.f;
    }
    for (int j = lane; j < C; j += 64) st<T>(grad, row * C + j, 0.f);
    return;
  }
  // max and its first index
  float m = -__builtin_huge_valf();
  int mi = C;
  for (int j = lane; j < C; j += 64) {
    const float v = ld<T>(xr, j);
    if (v > m) { m = v; mi = j; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(m, o, 64);
    const int oi = __shfl_xor(mi, o, 64);
    if (om > m || (om == m && oi < mi)) { m = om; mi = oi; }
  }
  float s = 0.f;
  for (int j = lane; j < C; j += 64) s += __expf(ld<T>(xr, j) - m);
  s = wave_sum(s);
  const float lse = m + __logf(s);
  if (lane == 0) {
    loss[row] = lse - ld<T>(xr, t);
    correct[row] = mi == t ? 1.f : 0.f;
  }
  const float inv = 1.f / s;
  for (int j = lane; j < C; j += 64) {
    const float p = __expf(ld<T>(xr, j) - m) * inv;
    st<T>(grad, row * C + j, p - (j == t ? 1.f : 0.f));
  }
}

// Large vocabularies (the GPT-2 LM head, C = 50,257): one 256-thread block per
// row, an online max / sum pass (running max with rescaled sum, first argmax)
// reduced over the block in a fixed tree, then the gradient pass -- two passes
// over the row instead of three, 4x the lanes of the one-wave kernel.
template <typename T>
__global__ void __launch_bounds__(256) ce_fwd_row_kernel(const T* __restrict__ x,
                                                         const int64_t* __restrict__ tgt, int C,
                                                         float* __restrict__ loss,
                                                         float* __restrict__ correct,
                                                         T* __restrict__ grad) {
  __shared__ float sm[256], ss[256];
  __shared__ int si[256];
  const int64_t row = blockIdx.x;
  const int tid = threadIdx.x;
  const T* xr = x + row * C;
  T* gr = grad + row * C;
  const int64_t t = tgt[row];
  if (t < 0 || t >= C) {  // ignored row (label -100): zero loss and gradient
    if (tid == 0) {
      loss[row] = 0.f;
      correct[row] = 0.f;
    }
    for (int j = tid; j < C; j += 256) st<T>(gr, j, 0.f);
    return;
  }
  float m = -__builtin_huge_valf(), sum = 0.f;
  int mi = C;
  for (int j = tid; j < C; j += 256) {
    const float v = ld<T>(xr, j);
    if (v > m) {
      sum = sum * __expf(m - v) + 1.f;
      m = v;
      mi = j;
    } else {
      sum += __expf(v - m);
    }
  }
  sm[tid] = m;
  ss[tid] = sum;
  si[tid] = mi;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) {
      const float m1 = sm[tid], m2 = sm[tid + o];
      const float mm = fmaxf(m1, m2);
      const float s1 = m1 == -__builtin_huge_valf() ? 0.f : ss[tid] * __expf(m1 - mm);
      const float s2 = m2 == -__builtin_huge_valf() ? 0.f : ss[tid + o] * __expf(m2 - mm);
      const int i1 = si[tid], i2 = si[tid + o];
      si[tid] = (m2 > m1 || (m2 == m1 && i2 < i1)) ? i2 : i1;
      sm[tid] = mm;
      ss[tid] = s1 + s2;
    }
    __syncthreads();
  }
  const float mx = sm[0], tot = ss[0];
  if (tid == 0) {
    loss[row] = mx + __logf(tot) - ld<T>(xr, t);
    correct[row] = si[0] == t ? 1.f : 0.f;
  }
  const float inv = 1.f / tot;
  for (int j = tid; j < C; j += 256) st<T>(gr, j, __expf(ld<T>(xr, j) - mx) * inv - (j == t ? 1.f : 0.f));
}

// g[r][j] *= s[r] (the CE backward: the unit gradient scaled by dL/dloss), one
// wave per row
template <typename T>
__global__ void __launch_bounds__(256) scale_rows_kernel(T* __restrict__ g, const float* __restrict__ s,
                                                         int64_t B, int C) {
  const int lane = threadIdx.x & 63;
  const int64_t row = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (row >= B) return;
  const float f = s[row];
  T* gr = g + row * C;
  for (int j = lane; j < C; j += 64) st<T>(gr, j, ld<T>(gr, j) * f);
}

template <typename T>
__global__ void __launch_bounds__(256) scale_row_block_kernel(T* __restrict__ g, const float* __restrict__ s, int C) {
  const int64_t row = blockIdx.x;
  const float f = s[row];
  T* gr = g + row * C;
  for (int j = threadIdx.x; j < C; j += 256) st<T>(gr, j, ld<T>(gr, j) * f);
}

}  // namespace

void launch_scale_rows(void* g, bool bf16, const float* s, int64_t B, int C, hipStream_t stream) {
  if (B == 0) return;
  if (C > 4096) {  // a block per (long) row
    if (bf16)
      COMMEFF_LAUNCH(scale_row_block_kernel<uint16_t>, dim3(static_cast<uint32_t>(B)), dim3(256), 0, stream,
                     static_cast<uint16_t*>(g), s, C);
    else
      COMMEFF_LAUNCH(scale_row_block_kernel<float>, dim3(static_cast<uint32_t>(B)), dim3(256), 0, stream,
                     static_cast<float*>(g), s, C);
    return;
  }
  const dim3 grid(static_cast<uint32_t>((B + 3) / 4));
  if (bf16)
    COMMEFF_LAUNCH(scale_rows_kernel<uint16_t>, grid, dim3(256), 0, stream, static_cast<uint16_t*>(g), s, B, C);
  else
    COMMEFF_LAUNCH(scale_rows_kernel<float>, grid, dim3(256), 0, stream, static_cast<float*>(g), s, B, C);
}

void launch_ce_fwd(const void* x, bool bf16, const int64_t* tgt, int64_t B, int C, float* loss,
                   float* correct, void* grad, hipStream_t stream) {
  if (B == 0) return;
  if (C > 4096) {
    if (bf16)
      COMMEFF_LAUNCH(ce_fwd_row_kernel<uint16_t>, dim3(static_cast<uint32_t>(B)), dim3(256), 0, stream,
                     static_cast<const uint16_t*>(x), tgt, C, loss, correct, static_cast<uint16_t*>(grad));
    else
      COMMEFF_LAUNCH(ce_fwd_row_kernel<float>, dim3(static_cast<uint32_t>(B)), dim3(256), 0, stream,
                     static_cast<const float*>(x), tgt, C, loss, correct, static_cast<float*>(grad));
    return;
  }
  const dim3 grid(static_cast<uint32_t>((B + 3) / 4));
  if (bf16)
    COMMEFF_LAUNCH(ce_fwd_kernel<uint16_t>, grid, dim3(256), 0, stream,
                       static_cast<const uint16_t*>(x), tgt, B, C, loss, correct,
                       static_cast<uint16_t*>(grad));
  else
    COMMEFF_LAUNCH(ce_fwd_kernel<float>, grid, dim3(256), 0, stream,
                       static_cast<const float*>(x), tgt, B, C, loss, correct,
                       static_cast<float*>(grad));
}

// Per-client mean metrics (fed_model.py _metric_sums): out[i, w] = mean of
// rows[i][e] over the examples e with slot[e] == w (slot sorted ascending:
// each client's examples are contiguous), 0 for clients without examples on
// this rank.  Thread per (metric, client), sequential sum in example order
// (deterministic); replaces zeros + index_add per metric + divide + copy.
namespace {
__global__ void __launch_bounds__(256)
client_means_kernel(ClientMeanRows rows, const int64_t* __restrict__ slot, int n,
                    const void* __restrict__ counts, bool counts_f32, int W, float* __restrict__ out) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= rows.m * W) return;
  const int i = t / W, w = t - i * W;
  int lo = 0, hi = n;  // first e with slot[e] >= w
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (slot[mid] < w) lo = mid + 1; else hi = mid;
  }
  const float* r = rows.p[0];
#pragma unroll
  for (int q = 1; q < kClientMeanRows; ++q)
    if (q == i) r = rows.p[q];
  float s = 0.f;
  for (int e = lo; e < n && slot[e] == w; ++e) s += r[e];
  const float c = counts_f32 ? static_cast<const float*>(counts)[w]
                             : static_cast<float>(static_cast<const int64_t*>(counts)[w]);
  out[t] = s / c;
}
}  // namespace

void launch_client_means(const ClientMeanRows& rows, const int64_t* slot, int n, const void* counts,
                         bool counts_f32, int W, float* out, hipStream_t stream) {
  const int total = rows.m * W;
  if (total <= 0) return;
  COMMEFF_LAUNCH(client_means_kernel, dim3((total + 255) / 256), dim3(256), 0, stream, rows, slot,
                     n, counts, counts_f32, W, out);
}

}  // namespace commeff
