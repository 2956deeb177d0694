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
                                                     int C, int64_t ldx, float* __restrict__ loss,
                                                     float* __restrict__ correct,
                                                     T* __restrict__ grad) {
  const int lane = threadIdx.x & 63;
  const int64_t row = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (row >= B) return;
  const T* xr = x + row * ldx;
  const int64_t t = tgt[row];
  if (t < 0 || t >= C) {  // ignored row (label -100): zero loss and gradient
    if (lane == 0) {
      loss[row] = 0.f;
      correct[row] = 0.f;
    }
    for (int j = lane; j < C; j += 64) st<T>(grad, row * ldx + j, 0.f);
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
    st<T>(grad, row * ldx + j, p - (j == t ? 1.f : 0.f));
  }
}

typedef uint32_t cev4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t ce_pack2(float lo, float hi) {
  const __bf16 a = static_cast<__bf16>(lo), b = static_cast<__bf16>(hi);
  return static_cast<uint32_t>(__builtin_bit_cast(uint16_t, a)) |
         (static_cast<uint32_t>(__builtin_bit_cast(uint16_t, b)) << 16);
}

// (max, first argmax) of a 512-lane block: waves by shuffles, then the 8 wave
// results in order through LDS (ties to the lower index, as torch.argmax)
__device__ __forceinline__ void block_max_arg(float& m, int& mi, float* sm, int* si) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(m, o, 64);
    const int oi = __shfl_xor(mi, o, 64);
    if (om > m || (om == m && oi < mi)) { m = om; mi = oi; }
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { sm[w] = m; si[w] = mi; }
  __syncthreads();
  m = sm[0];
  mi = si[0];
  for (int q = 1; q < 8; ++q)
    if (sm[q] > m || (sm[q] == m && si[q] < mi)) { m = sm[q]; mi = si[q]; }
}

// Large vocabularies in a padded bf16 buffer (the tied GPT-2 LM head's logits,
// C = 50,257 in rows of a multiple of 8, 16-byte aligned): one 512-lane block
// per row holds the row in registers (NV 16-byte chunks a lane) -- ONE read of
// the logits and one write of the gradient (the pad columns get 0), against
// the two-pass scalar kernel below (145 us per GPT-2 round at 640 rows).
template <int NV>
__global__ void __launch_bounds__(512) ce_fwd_rowv_kernel(const uint16_t* __restrict__ x,
                                                          const int64_t* __restrict__ tgt, int C, int64_t ldx,
                                                          float* __restrict__ loss, float* __restrict__ correct,
                                                          uint16_t* __restrict__ grad) {
  __shared__ float sm[8], ss[8];
  __shared__ int si[8];
  const int64_t row = blockIdx.x;
  const int tid = threadIdx.x;
  const cev4* xr = reinterpret_cast<const cev4*>(x + row * ldx);
  cev4* gr = reinterpret_cast<cev4*>(grad + row * ldx);
  const int nvec = (C + 7) >> 3;
  const int64_t t = tgt[row];
  if (t < 0 || t >= C) {  // ignored row (label -100): zero loss and gradient
    if (tid == 0) {
      loss[row] = 0.f;
      correct[row] = 0.f;
    }
    for (int i = tid; i < nvec; i += 512) gr[i] = cev4{0u, 0u, 0u, 0u};
    return;
  }
  cev4 v[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int idx = tid + i * 512;
    v[i] = idx < nvec ? xr[idx] : cev4{0u, 0u, 0u, 0u};
  }
  float m = -__builtin_huge_valf();
  int mi = C;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c0 = (tid + i * 512) * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t wv = v[i][j >> 1];
      const float f = __uint_as_float((j & 1) ? (wv & 0xffff0000u) : (wv << 16));
      if (c0 + j < C && f > m) { m = f; mi = c0 + j; }
    }
  }
  block_max_arg(m, mi, sm, si);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c0 = (tid + i * 512) * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t wv = v[i][j >> 1];
      const float f = __uint_as_float((j & 1) ? (wv & 0xffff0000u) : (wv << 16));
      if (c0 + j < C) s += __expf(f - m);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((tid & 63) == 0) ss[tid >> 6] = s;
  __syncthreads();
  s = 0.f;
  for (int q = 0; q < 8; ++q) s += ss[q];
  if (tid == (t >> 3) % 512) {  // the lane holding the target
    const int i = static_cast<int>((t >> 3) / 512), j = static_cast<int>(t & 7);
    uint32_t wv = 0u;
#pragma unroll
    for (int q = 0; q < NV; ++q)
      if (q == i) wv = v[q][j >> 1];
    const float xt = __uint_as_float((j & 1) ? (wv & 0xffff0000u) : (wv << 16));
    loss[row] = m + __logf(s) - xt;
    correct[row] = mi == t ? 1.f : 0.f;
  }
  const float inv = 1.f / s;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int idx = tid + i * 512;
    if (idx >= nvec) continue;
    const int c0 = idx * 8;
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t wv = v[i][j >> 1];
      const float f = __uint_as_float((j & 1) ? (wv & 0xffff0000u) : (wv << 16));
      o[j] = c0 + j < C ? __expf(f - m) * inv - (c0 + j == t ? 1.f : 0.f) : 0.f;
    }
    gr[idx] = cev4{ce_pack2(o[0], o[1]), ce_pack2(o[2], o[3]), ce_pack2(o[4], o[5]), ce_pack2(o[6], o[7])};
  }
}

// Large vocabularies (the GPT-2 LM head, C = 50,257): one 256-thread block per
// row, an online max / sum pass (running max with rescaled sum, first argmax)
// reduced over the block in a fixed tree, then the gradient pass -- two passes
// over the row instead of three, 4x the lanes of the one-wave kernel.
template <typename T>
__global__ void __launch_bounds__(256) ce_fwd_row_kernel(const T* __restrict__ x,
                                                         const int64_t* __restrict__ tgt, int C,
                                                         int64_t ldx, float* __restrict__ loss,
                                                         float* __restrict__ correct,
                                                         T* __restrict__ grad) {
  __shared__ float sm[256], ss[256];
  __shared__ int si[256];
  const int64_t row = blockIdx.x;
  const int tid = threadIdx.x;
  const T* xr = x + row * ldx;
  T* gr = grad + row * ldx;
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
                                                         int64_t B, int C, int64_t ldg) {
  const int lane = threadIdx.x & 63;
  const int64_t row = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (row >= B) return;
  const float f = s[row];
  T* gr = g + row * ldg;
  for (int j = lane; j < C; j += 64) st<T>(gr, j, ld<T>(gr, j) * f);
}

template <typename T>
__global__ void __launch_bounds__(256) scale_row_block_kernel(T* __restrict__ g, const float* __restrict__ s, int C,
                                                              int64_t ldg) {
  const int64_t row = blockIdx.x;
  const float f = s[row];
  T* gr = g + row * ldg;
  for (int j = threadIdx.x; j < C; j += 256) st<T>(gr, j, ld<T>(gr, j) * f);
}

// bf16 rows of a padded buffer (row stride % 8 == 0, 16-byte aligned): 16-byte
// chunks, the pad columns past C (zero) scaled too
__global__ void __launch_bounds__(256) scale_row_vec_kernel(uint16_t* __restrict__ g, const float* __restrict__ s,
                                                            int C, int64_t ldg) {
  const int64_t row = blockIdx.x;
  const float f = s[row];
  cev4* gr = reinterpret_cast<cev4*>(g + row * ldg);
  const int nvec = (C + 7) >> 3;
  for (int i = threadIdx.x; i < nvec; i += 256) {
    const cev4 v = gr[i];
    cev4 o;
#pragma unroll
    for (int h = 0; h < 4; ++h)
      o[h] = ce_pack2(__uint_as_float(v[h] << 16) * f, __uint_as_float(v[h] & 0xffff0000u) * f);
    gr[i] = o;
  }
}

}  // namespace

void launch_scale_rows(void* g, bool bf16, const float* s, int64_t B, int C, int64_t ldg, hipStream_t stream) {
  if (B == 0) return;
  if (C > 4096) {  // a block per (long) row
    if (bf16 && ldg % 8 == 0 && reinterpret_cast<uintptr_t>(g) % 16 == 0)
      COMMEFF_LAUNCH(scale_row_vec_kernel, dim3(static_cast<uint32_t>(B)), dim3(256), 0, stream,
                     static_cast<uint16_t*>(g), s, C, ldg);
    else if (bf16)
      COMMEFF_LAUNCH(scale_row_block_kernel<uint16_t>, dim3(static_cast<uint32_t>(B)), dim3(256), 0, stream,
                     static_cast<uint16_t*>(g), s, C, ldg);
    else
      COMMEFF_LAUNCH(scale_row_block_kernel<float>, dim3(static_cast<uint32_t>(B)), dim3(256), 0, stream,
                     static_cast<float*>(g), s, C, ldg);
    return;
  }
  const dim3 grid(static_cast<uint32_t>((B + 3) / 4));
  if (bf16)
    COMMEFF_LAUNCH(scale_rows_kernel<uint16_t>, grid, dim3(256), 0, stream, static_cast<uint16_t*>(g), s, B, C, ldg);
  else
    COMMEFF_LAUNCH(scale_rows_kernel<float>, grid, dim3(256), 0, stream, static_cast<float*>(g), s, B, C, ldg);
}

void launch_ce_fwd(const void* x, bool bf16, const int64_t* tgt, int64_t B, int C, int64_t ldx, float* loss,
                   float* correct, void* grad, hipStream_t stream) {
  if (B == 0) return;
  if (C > 4096) {
    constexpr int kNV = 13;  // 512 lanes x 13 chunks x 8 = 53,248 columns
    if (bf16 && ldx % 8 == 0 && (C + 7) / 8 <= 512 * kNV && reinterpret_cast<uintptr_t>(x) % 16 == 0 &&
        reinterpret_cast<uintptr_t>(grad) % 16 == 0) {
      COMMEFF_LAUNCH(ce_fwd_rowv_kernel<kNV>, dim3(static_cast<uint32_t>(B)), dim3(512), 0, stream,
                     static_cast<const uint16_t*>(x), tgt, C, ldx, loss, correct, static_cast<uint16_t*>(grad));
      return;
    }
    if (bf16)
      COMMEFF_LAUNCH(ce_fwd_row_kernel<uint16_t>, dim3(static_cast<uint32_t>(B)), dim3(256), 0, stream,
                     static_cast<const uint16_t*>(x), tgt, C, ldx, loss, correct, static_cast<uint16_t*>(grad));
    else
      COMMEFF_LAUNCH(ce_fwd_row_kernel<float>, dim3(static_cast<uint32_t>(B)), dim3(256), 0, stream,
                     static_cast<const float*>(x), tgt, C, ldx, loss, correct, static_cast<float*>(grad));
    return;
  }
  const dim3 grid(static_cast<uint32_t>((B + 3) / 4));
  if (bf16)
    COMMEFF_LAUNCH(ce_fwd_kernel<uint16_t>, grid, dim3(256), 0, stream,
                       static_cast<const uint16_t*>(x), tgt, B, C, ldx, loss, correct,
                       static_cast<uint16_t*>(grad));
  else
    COMMEFF_LAUNCH(ce_fwd_kernel<float>, grid, dim3(256), 0, stream,
                       static_cast<const float*>(x), tgt, B, C, ldx, loss, correct,
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
