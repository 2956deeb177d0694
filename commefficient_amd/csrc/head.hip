// ResNet-9 classifier head as two kernels (gfx950): the reference head
// (/root/reference/CommEfficient/models/resnet9.py:118-130: MaxPool2d(4) ->
// flatten -> Linear(512, classes, bias=False) -> Mul(0.125)) followed by the
// per-example cross-entropy and top-1 (cv_train.py:31-84).
//
// Forward (one wave per example): max-pool of the res3 output over its HxW
// pixels (relu is the identity there: res3's output is >= 0) with a 1-byte
// window code, logits = scale * pooled . W^T in fp32 (W read in place from the
// fp32 master weights), then loss = lse - logit[t], correct, and the unit
// gradient softmax - onehot.  Saved for backward: pooled (bf16, exact),
// codes, unit gradient.
// Backward (one launch): blocks [0, nrow) route dx = scale * (g . W) to the
// argmax pixel of every (example, channel) window (zeros elsewhere, full
// NHWC input gradient written once); blocks [nrow, ...) compute dW[c, j] =
// scale * sum_b g[b, c] pooled[b, j] with one thread per weight in a fixed
// order (deterministic) and accumulate it into the existing fp32 gradient.
// Replaces relu_maxpool(4) fwd/bwd, three hipBLASLt GEMMs, the scale
// multiplies, casts and the CE kernel of the unfused head (~10 launches).
#include <hip/hip_runtime.h>
#include <cstdint>
#include "kernels.h"

namespace commeff {
namespace {

constexpr int kMaxCls = 128;

__device__ __forceinline__ float bfv(uint16_t h) { return __uint_as_float(static_cast<uint32_t>(h) << 16); }

__device__ __forceinline__ float wsum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

struct alignas(16) H8 {
  uint16_t h[8];
};

// x: [B, NPIX, C] bf16 (NHWC of a [B, C, h, w] channels_last tensor)
__global__ void __launch_bounds__(256)
head_fwd_kernel(const uint16_t* __restrict__ x, const float* __restrict__ w, const int64_t* __restrict__ tgt,
                int B, int C, int NPIX, int NCLS, float scale, float* __restrict__ loss,
                float* __restrict__ correct, float* __restrict__ gunit, uint16_t* __restrict__ pooled,
                uint8_t* __restrict__ codes) {
  __shared__ float logit_s[4][kMaxCls];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int b = blockIdx.x * (blockDim.x >> 6) + wv;
  if (b >= B) return;
  const uint16_t* xb = x + static_cast<size_t>(b) * NPIX * C;
  // each lane owns 8 consecutive channels per 512-channel chunk
  for (int c0 = 0; c0 < NCLS; c0 += 64) {
    if (lane + c0 < NCLS) logit_s[wv][lane + c0] = 0.f;
  }
  __builtin_amdgcn_wave_barrier();  // (one wave's LDS ops complete in program order)
  for (int ch = lane * 8; ch < C; ch += 512) {
    float best[8];
    uint32_t arg[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      best[j] = -__builtin_huge_valf();
      arg[j] = 0;
    }
    // 8 pixels' loads in flight at a time (a load-compare chain per pixel
    // left the kernel latency-bound)
    for (int p0 = 0; p0 < NPIX; p0 += 8) {
      H8 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (p0 + u < NPIX) v[u] = *reinterpret_cast<const H8*>(xb + static_cast<size_t>(p0 + u) * C + ch);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (p0 + u >= NPIX) break;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float f = bfv(v[u].h[j]);
          if (f > best[j]) {
            best[j] = f;
            arg[j] = static_cast<uint32_t>(p0 + u);
          }
        }
      }
    }
    H8 pv;
    uint64_t cd = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bool pos = best[j] > 0.f;  // relu(max) == max(relu)
      if (!pos) best[j] = 0.f;
      pv.h[j] = static_cast<uint16_t>(__float_as_uint(best[j]) >> 16);
      cd |= static_cast<uint64_t>(pos ? arg[j] : 255u) << (8 * j);
    }
    *reinterpret_cast<H8*>(pooled + static_cast<size_t>(b) * C + ch) = pv;
    *reinterpret_cast<uint64_t*>(codes + static_cast<size_t>(b) * C + ch) = cd;
    // partial logits of this lane's 8 channels, 4 classes at a time (loads
    // first, then 4 independent wave sums)
    for (int k0 = 0; k0 < NCLS; k0 += 4) {
      float4 w0[4], w1[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int k = k0 + u < NCLS ? k0 + u : NCLS - 1;
        w0[u] = *reinterpret_cast<const float4*>(w + static_cast<size_t>(k) * C + ch);
        w1[u] = *reinterpret_cast<const float4*>(w + static_cast<size_t>(k) * C + ch + 4);
      }
      float sv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        sv[u] = best[0] * w0[u].x + best[1] * w0[u].y + best[2] * w0[u].z + best[3] * w0[u].w +
                best[4] * w1[u].x + best[5] * w1[u].y + best[6] * w1[u].z + best[7] * w1[u].w;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1)
#pragma unroll
        for (int u = 0; u < 4; ++u) sv[u] += __shfl_xor(sv[u], o, 64);
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (lane == 0 && k0 + u < NCLS) logit_s[wv][k0 + u] += sv[u];
    }
  }
  __builtin_amdgcn_wave_barrier();
  // softmax / CE over the classes (lane per class, NCLS <= 128)
  float m = -__builtin_huge_valf();
  int mi = NCLS;
  float lg[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int k = lane + 64 * q;
    lg[q] = k < NCLS ? scale * logit_s[wv][k] : -__builtin_huge_valf();
    if (k < NCLS && lg[q] > m) {
      m = lg[q];
      mi = k;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(m, o, 64);
    const int oi = __shfl_xor(mi, o, 64);
    if (om > m || (om == m && oi < mi)) {
      m = om;
      mi = oi;
    }
  }
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < 2; ++q)
    if (lane + 64 * q < NCLS) s += __expf(lg[q] - m);
  s = wsum(s);
  const float lse = m + __logf(s);
  const int64_t t = tgt[b];
  const float inv = 1.f / s;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int k = lane + 64 * q;
    if (k < NCLS) {
      gunit[static_cast<size_t>(b) * NCLS + k] = __expf(lg[q] - m) * inv - (k == t ? 1.f : 0.f);
      if (k == t) loss[b] = lse - lg[q];
    }
  }
  if (lane == 0) correct[b] = mi == t ? 1.f : 0.f;
}

// g[b, k] = gl[b] * gunit[b, k]  (dL/dlogit); dx and dW as described above
__global__ void __launch_bounds__(256)
head_bwd_kernel(const float* __restrict__ gl, const float* __restrict__ gunit, const float* __restrict__ w,
                const uint16_t* __restrict__ pooled, const uint8_t* __restrict__ codes, int B, int C,
                int NPIX, int NCLS, float scale, int nrow_blocks, uint16_t* __restrict__ dx,
                float* __restrict__ dw, float beta, const uint16_t* __restrict__ ymask,
                uint16_t* __restrict__ dxm) {
  // ymask / dxm (optional): also dx masked by ymask > 0 -- the producing
  // residual unit's ReLU backward (nn.py _MaskLink), one pass fewer
  const int lane = threadIdx.x & 63;
  if (static_cast<int>(blockIdx.x) < nrow_blocks) {
    const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b >= B) return;
    const float glb = gl[b] * scale;
    for (int ch = lane * 8; ch < C; ch += 512) {
      float d[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int k = 0; k < NCLS; ++k) {
        const float gk = glb * gunit[static_cast<size_t>(b) * NCLS + k];
        const float4 w0 = *reinterpret_cast<const float4*>(w + static_cast<size_t>(k) * C + ch);
        const float4 w1 = *reinterpret_cast<const float4*>(w + static_cast<size_t>(k) * C + ch + 4);
        d[0] += gk * w0.x; d[1] += gk * w0.y; d[2] += gk * w0.z; d[3] += gk * w0.w;
        d[4] += gk * w1.x; d[5] += gk * w1.y; d[6] += gk * w1.z; d[7] += gk * w1.w;
      }
      const uint64_t cd = *reinterpret_cast<const uint64_t*>(codes + static_cast<size_t>(b) * C + ch);
      uint16_t hv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const __bf16 h = static_cast<__bf16>(d[j]);
        hv[j] = __builtin_bit_cast(uint16_t, h);
      }
      for (int p = 0; p < NPIX; ++p) {
        H8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j)
          o.h[j] = ((cd >> (8 * j)) & 0xffu) == static_cast<uint64_t>(p) ? hv[j] : static_cast<uint16_t>(0);
        const size_t off = (static_cast<size_t>(b) * NPIX + p) * C + ch;
        *reinterpret_cast<H8*>(dx + off) = o;
        if (ymask != nullptr) {
          const H8 y = *reinterpret_cast<const H8*>(ymask + off);
          H8 om;
#pragma unroll
          for (int j = 0; j < 8; ++j)
            om.h[j] = (!(y.h[j] & 0x8000u) && y.h[j] != 0u) ? o.h[j] : static_cast<uint16_t>(0);
          *reinterpret_cast<H8*>(dxm + off) = om;
        }
      }
    }
    return;
  }
  // dW: block per (class k, 64-channel chunk); wave w sums the rows
  // b = w, w + 4, ... for its lane's channel (8 independent loads in flight),
  // then the 4 wave partials are added in fixed order (deterministic)
  __shared__ float part[4][64];
  const int e = blockIdx.x - nrow_blocks;
  const int nchunk = (C + 63) / 64;
  const int k = e / nchunk, j = (e - k * nchunk) * 64 + lane, wv = threadIdx.x >> 6;
  float s = 0.f;
  if (j < C) {
    int b = wv;
    for (; b + 28 < B; b += 32) {
      float pv[8], gv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        pv[u] = bfv(pooled[static_cast<size_t>(b + 4 * u) * C + j]);
        gv[u] = gl[b + 4 * u] * gunit[static_cast<size_t>(b + 4 * u) * NCLS + k];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) s += gv[u] * pv[u];
    }
    for (; b < B; b += 4) s += gl[b] * gunit[static_cast<size_t>(b) * NCLS + k] * bfv(pooled[static_cast<size_t>(b) * C + j]);
  }
  part[wv][lane] = s;
  __syncthreads();
  if (wv == 0 && j < C) {
    const float t = ((part[0][lane] + part[1][lane]) + part[2][lane]) + part[3][lane];
    const size_t o = static_cast<size_t>(k) * C + j;
    dw[o] = beta != 0.f ? beta * dw[o] + scale * t : scale * t;
  }
}

}  // namespace

bool head_supported(int C, int NCLS) { return C % 8 == 0 && NCLS >= 1 && NCLS <= kMaxCls; }

void launch_head_fwd(const uint16_t* x, const float* w, const int64_t* tgt, int B, int C, int NPIX, int NCLS,
                     float scale, float* loss, float* correct, float* gunit, uint16_t* pooled, uint8_t* codes,
                     hipStream_t stream) {
  if (B <= 0) return;
  // two waves (examples) per block: 250 blocks for B = 500 fill the 256 CUs
  COMMEFF_LAUNCH(head_fwd_kernel, dim3((B + 1) / 2), dim3(128), 0, stream, x, w, tgt, B, C, NPIX, NCLS,
                     scale, loss, correct, gunit, pooled, codes);
}

void launch_head_bwd(const float* gl, const float* gunit, const float* w, const uint16_t* pooled,
                     const uint8_t* codes, int B, int C, int NPIX, int NCLS, float scale, uint16_t* dx,
                     float* dw, float beta, hipStream_t stream, const uint16_t* ymask, uint16_t* dxm) {
  const int nrow = (B + 3) / 4;
  const int nw = NCLS * ((C + 63) / 64);
  if (nrow + nw <= 0) return;
  COMMEFF_LAUNCH(head_bwd_kernel, dim3(nrow + nw), dim3(256), 0, stream, gl, gunit, w, pooled, codes, B, C,
                     NPIX, NCLS, scale, nrow, dx, dw, beta, ymask, dxm);
}

}  // namespace commeff
