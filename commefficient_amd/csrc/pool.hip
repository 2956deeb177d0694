// Fused ReLU + k x k max-pool (stride k) on channels_last (NHWC) bf16
// activations, forward and backward (gfx950).
//
// ResNet-9's ConvBN blocks end in relu -> maxpool2 (reference
// /root/reference/CommEfficient/models/resnet9.py:44-52); relu and max commute,
// so one pass reads the conv output once, writes the pooled output and a
// 1-byte argmax code per output element (window position, or 255 when the
// max is <= 0 and ReLU zeroes the gradient).  The backward pass writes the
// full input gradient (zeros + routed values) in one coalesced sweep.
// PyTorch's separate NHWC max_pool2d backward + two ReLU passes measured
// ~110 us per pool layer for a 500-image batch (profiles/r1_v1_*).
//
// Vectorisation: each thread owns 8 consecutive channels (16-byte loads and
// stores of bf16x8); C must be a multiple of 8 (all ResNet-9 widths are).
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <cstdint>
#include "kernels.h"

namespace commeff {
namespace {

typedef uint16_t bf16raw;

__device__ __forceinline__ float bf2f(bf16raw v) {
  return __uint_as_float(static_cast<uint32_t>(v) << 16);
}

struct alignas(16) V8 {
  bf16raw h[8];
};

// index math: 32-bit with precomputed reciprocals (64-bit div/mod is a long
// software sequence per thread and made these kernels VALU-bound)
struct PoolGeom {
  int H, W, C, OH, OW, C8;
  uint32_t total;
  FastDivU32 d_c8, d_ow, d_oh;
};

__device__ __forceinline__ void pool_coords(uint32_t g, const PoolGeom& q, uint32_t& c8, uint32_t& ow,
                                            uint32_t& oh, uint32_t& n) {
  uint32_t p = fdiv(g, q.d_c8);
  c8 = g - p * q.C8;
  uint32_t p2 = fdiv(p, q.d_ow);
  ow = p - p2 * q.OW;
  n = fdiv(p2, q.d_oh);
  oh = p2 - n * q.OH;
}

template <int K>
__global__ void __launch_bounds__(256)
relu_maxpool_fwd_kernel(const bf16raw* __restrict__ x, bf16raw* __restrict__ y,
                        uint8_t* __restrict__ idx, PoolGeom q) {
  const int H = q.H, W = q.W, C = q.C;
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < q.total; g += stride) {
    uint32_t c8, ow, oh, n;
    pool_coords(g, q, c8, ow, oh, n);
    float best[8];
    uint8_t arg[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      best[q] = -__builtin_huge_valf();
      arg[q] = 0;
    }
#pragma unroll
    for (int dy = 0; dy < K; ++dy) {
#pragma unroll
      for (int dx = 0; dx < K; ++dx) {
        const size_t off = static_cast<size_t>((n * H + oh * K + dy) * W + ow * K + dx) * C + c8 * 8;
        V8 v = *reinterpret_cast<const V8*>(x + off);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          float f = bf2f(v.h[q]);
          if (f > best[q]) {
            best[q] = f;
            arg[q] = static_cast<uint8_t>(dy * K + dx);
          }
        }
      }
    }
    V8 o;
    uint64_t codes = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const bool pos = best[q] > 0.f;
      // the max is one of the inputs, so its bf16 bits are exact
      o.h[q] = pos ? static_cast<bf16raw>(__float_as_uint(best[q]) >> 16) : static_cast<bf16raw>(0);
      codes |= static_cast<uint64_t>(pos ? arg[q] : 255u) << (8 * q);
    }
    const size_t oo = static_cast<size_t>(g) * 8;  // == ((n*OH+oh)*OW+ow)*C + c8*8
    *reinterpret_cast<V8*>(y + oo) = o;
    *reinterpret_cast<uint64_t*>(idx + oo) = codes;
  }
}

template <int K>
__global__ void __launch_bounds__(256)
relu_maxpool_bwd_kernel(const bf16raw* __restrict__ gy, const uint8_t* __restrict__ idx,
                        bf16raw* __restrict__ gx, PoolGeom q) {
  const int H = q.H, W = q.W, C = q.C;
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < q.total; g += stride) {
    uint32_t c8, ow, oh, n;
    pool_coords(g, q, c8, ow, oh, n);
    const V8 gv = *reinterpret_cast<const V8*>(gy + static_cast<size_t>(g) * 8);
    const uint64_t codes = *reinterpret_cast<const uint64_t*>(idx + static_cast<size_t>(g) * 8);
#pragma unroll
    for (int dy = 0; dy < K; ++dy) {
#pragma unroll
      for (int dx = 0; dx < K; ++dx) {
        V8 o;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const uint32_t code = static_cast<uint32_t>(codes >> (8 * q)) & 0xffu;
          o.h[q] = code == static_cast<uint32_t>(dy * K + dx) ? gv.h[q] : static_cast<bf16raw>(0);
        }
        const size_t off = static_cast<size_t>((n * H + oh * K + dy) * W + ow * K + dx) * C + c8 * 8;
        *reinterpret_cast<V8*>(gx + off) = o;
      }
    }
  }
}

PoolGeom make_pool_geom(int N, int H, int W, int C, int k) {
  PoolGeom q;
  q.H = H; q.W = W; q.C = C;
  q.OH = H / k; q.OW = W / k; q.C8 = C / 8;
  q.total = static_cast<uint32_t>(static_cast<int64_t>(N) * q.OH * q.OW * q.C8);
  q.d_c8 = make_fastdiv(q.C8);
  q.d_ow = make_fastdiv(q.OW);
  q.d_oh = make_fastdiv(q.OH);
  return q;
}

int grid_for(int64_t n) {
  int64_t b = (n + 255) / 256;
  if (b < 1) b = 1;
  return static_cast<int>(b < 16384 ? b : 16384);
}

}  // namespace

void launch_relu_maxpool_fwd(const uint16_t* x, uint16_t* y, uint8_t* idx, int N, int H, int W,
                             int C, int k, hipStream_t stream) {
  const int64_t total = static_cast<int64_t>(N) * (H / k) * (W / k) * (C / 8);
  if (total == 0) return;
  const PoolGeom q = make_pool_geom(N, H, W, C, k);
  if (k == 2)
    COMMEFF_LAUNCH(relu_maxpool_fwd_kernel<2>, dim3(grid_for(total)), dim3(256), 0, stream, x,
                       y, idx, q);
  else
    COMMEFF_LAUNCH(relu_maxpool_fwd_kernel<4>, dim3(grid_for(total)), dim3(256), 0, stream, x,
                       y, idx, q);
}

void launch_relu_maxpool_bwd(const uint16_t* gy, const uint8_t* idx, uint16_t* gx, int N, int H,
                             int W, int C, int k, hipStream_t stream) {
  const int64_t total = static_cast<int64_t>(N) * (H / k) * (W / k) * (C / 8);
  if (total == 0) return;
  const PoolGeom q = make_pool_geom(N, H, W, C, k);
  if (k == 2)
    COMMEFF_LAUNCH(relu_maxpool_bwd_kernel<2>, dim3(grid_for(total)), dim3(256), 0, stream,
                       gy, idx, gx, q);
  else
    COMMEFF_LAUNCH(relu_maxpool_bwd_kernel<4>, dim3(grid_for(total)), dim3(256), 0, stream,
                       gy, idx, gx, q);
}

}  // namespace commeff
