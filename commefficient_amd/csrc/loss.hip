// Fused per-example cross-entropy for the CV loss (reference cv_train.py:31-84
// compute_loss_ce / Correct): one wave per example computes, in one pass over
// its logits row, the per-example loss lse(x) - x[t], top-1 correctness
// (argmax with ties to the lower index, like torch.argmax) and the unit
// gradient softmax(x) - onehot(t) (scaled by dL/dloss in backward).  Replaces
// log_softmax / nll / argmax / eq / cast kernels forward and backward.
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
  const int64_t t = tgt[row];
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

}  // namespace

void launch_ce_fwd(const void* x, bool bf16, const int64_t* tgt, int64_t B, int C, float* loss,
                   float* correct, void* grad, hipStream_t stream) {
  if (B == 0) return;
  const dim3 grid(static_cast<uint32_t>((B + 3) / 4));
  if (bf16)
    hipLaunchKernelGGL(ce_fwd_kernel<uint16_t>, grid, dim3(256), 0, stream,
                       static_cast<const uint16_t*>(x), tgt, B, C, loss, correct,
                       static_cast<uint16_t*>(grad));
  else
    hipLaunchKernelGGL(ce_fwd_kernel<float>, grid, dim3(256), 0, stream,
                       static_cast<const float*>(x), tgt, B, C, loss, correct,
                       static_cast<float*>(grad));
}

}  // namespace commeff
