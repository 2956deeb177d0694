// Explicit-GEMM convolutions and the overlapping max-pool of the ImageNet
// ResNets (gfx950): the 7x7/s2 stem, the strided 3x3 of each stage's first
// bottleneck, the strided 1x1 downsample and the 3x3/s2 max-pool.
//
// Reference model: torchvision-style ResNet-101 of
// /root/reference/CommEfficient/models/resnets.py:140-230 (stem conv1 + maxpool,
// Bottleneck conv2 with stride, downsample conv1x1 with stride).  These shapes
// fall outside the stride-1 3x3 MFMA kernels of conv.hip; MIOpen served them
// (igemm_fwd / igemm_bwd / igemm_wrw) and at::native the NHWC max-pool
// (655 us per backward, profiles/r2_pmc_imagenet.txt).  Here every such conv
// is an explicit GEMM over a bf16 column image:
//   * im2col_kernel writes col[p][(r*S + s)*C + c] (zero outside the image
//     and in the padding columns up to Kc); with C % 8 == 0 every thread moves
//     one 16-byte chunk (8 channels of one tap), otherwise (the 3-channel
//     stem input, any pixel stride) 8 single gathers;
//   * the forward / dgrad GEMMs are plain hipBLASLt GEMMs on col and the
//     [K][Kc] weight image (ops/nn.py);
//   * col2im_kernel is the dgrad's gather: every input pixel sums the <=
//     ceil(R/stride) x ceil(S/stride) column entries that read it, in fp32, in
//     a fixed tap order (deterministic, no atomics, zeros written where no
//     tap lands -- the strided 1x1 scatter in the same pass);
//   * wgrad_rsc_add_kernel folds the split-K partial products of the weight
//     gradient (fixed order), permutes (r, s, c) -> (c, r, s) and adds into
//     the flat fp32 gradient (or the per-group rows of ops/grouped.py);
//     wgrad_split_add4_kernel is its 1x1 case (no permutation: float4 moves,
//     8 split loads in flight), also used by the 1x1 GEMM convs' split-K;
//   * maxpool_fwd_kernel / maxpool_bwd_kernel: k x k max-pool with stride s and
//     padding p, 1-byte window codes, and a gather backward (each input pixel
//     collects the outputs whose code points at it).
#include <hip/hip_runtime.h>
#include <cstdint>
#include "kernels.h"
#include "sketch_hash.h"

namespace commeff {
namespace {

typedef uint16_t bf16raw;

struct alignas(16) V8 {
  bf16raw h[8];
};

__device__ __forceinline__ float bf2f(bf16raw v) { return __uint_as_float(static_cast<uint32_t>(v) << 16); }

__device__ __forceinline__ bf16raw f2bf(float f) {  // round to nearest even (NaN kept quiet)
  const uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return static_cast<bf16raw>((u >> 16) | 0x40u);
  return static_cast<bf16raw>((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

int blocks_for(int64_t n) {
  int64_t b = (n + 255) / 256;
  if (b < 1) b = 1;
  return static_cast<int>(b < 32768 ? b : 32768);
}

// ---------------------------------------------------------------- im2col
struct ColGeom {
  int H, W, C, OH, OW, R, S, stride, pad, Kc, KC8;
  int64_t sN, sH, sW;  // input strides in elements (channel stride 1)
  int64_t sG;          // grouped: input offset of group g's channels / images
  uint32_t total;      // P * G * Kc / 8
  FastDivU32 d_kc8, d_ow, d_oh, d_c8, d_s, d_c, d_g;
};

__device__ __forceinline__ void col_row(uint32_t p, const ColGeom& q, int& n, int& oh, int& ow) {
  const uint32_t p2 = fdiv(p, q.d_ow);
  ow = static_cast<int>(p - p2 * q.OW);
  const uint32_t nn = fdiv(p2, q.d_oh);
  oh = static_cast<int>(p2 - nn * q.OH);
  n = static_cast<int>(nn);
}

// C % 8 == 0: one 16-byte tap chunk per thread
__global__ void __launch_bounds__(256) im2col_vec_kernel(const bf16raw* __restrict__ x,
                                                         bf16raw* __restrict__ col, ColGeom q) {
  const uint32_t step = gridDim.x * blockDim.x;
  const int taps = q.R * q.S;
  for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < q.total; g += step) {
    const uint32_t pg = fdiv(g, q.d_kc8);  // (pixel, group) row of the [P][G][Kc] image
    const uint32_t j8 = g - pg * q.KC8;
    const uint32_t p = fdiv(pg, q.d_g);
    const bf16raw* xg = x + static_cast<int64_t>(pg - p * static_cast<uint32_t>(q.d_g.d)) * q.sG;
    const uint32_t tap = fdiv(j8, q.d_c8);
    const uint32_t c8 = j8 - tap * (q.C / 8);
    V8 v;
#pragma unroll
    for (int e = 0; e < 8; ++e) v.h[e] = 0;
    if (static_cast<int>(tap) < taps) {
      int n, oh, ow;
      col_row(p, q, n, oh, ow);
      const uint32_t r = fdiv(tap, q.d_s);
      const int s = static_cast<int>(tap - r * q.S);
      const int ih = oh * q.stride - q.pad + static_cast<int>(r);
      const int iw = ow * q.stride - q.pad + s;
      if (ih >= 0 && ih < q.H && iw >= 0 && iw < q.W)
        v = *reinterpret_cast<const V8*>(xg + n * q.sN + ih * q.sH + iw * q.sW + c8 * 8);
    }
    *reinterpret_cast<V8*>(col + static_cast<size_t>(g) * 8) = v;
  }
}

// any C / pixel stride (the 3-channel network input): 8 single gathers
__global__ void __launch_bounds__(256) im2col_any_kernel(const bf16raw* __restrict__ x,
                                                         bf16raw* __restrict__ col, ColGeom q) {
  const uint32_t step = gridDim.x * blockDim.x;
  const int rsc = q.R * q.S * q.C;
  for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < q.total; g += step) {
    const uint32_t pg = fdiv(g, q.d_kc8);
    const int j0 = static_cast<int>(g - pg * q.KC8) * 8;
    const uint32_t p = fdiv(pg, q.d_g);
    int n, oh, ow;
    col_row(p, q, n, oh, ow);
    const bf16raw* xn = x + static_cast<int64_t>(pg - p * static_cast<uint32_t>(q.d_g.d)) * q.sG + n * q.sN;
    // (r, s, c) of the chunk's first column by two divisions, then stepped
    // (three divisions per element had made the 7x7 ImageNet stem's 1 GB
    // column image compute-bound: 614 us)
    const uint32_t tap0 = fdiv(static_cast<uint32_t>(j0 < rsc ? j0 : 0), q.d_c);
    int c = (j0 < rsc ? j0 : 0) - static_cast<int>(tap0) * q.C;
    const uint32_t r0 = fdiv(tap0, q.d_s);
    int r = static_cast<int>(r0), s = static_cast<int>(tap0 - r0 * q.S);
    const int ih0 = oh * q.stride - q.pad, iw0 = ow * q.stride - q.pad;
    bf16raw vals[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int ih = ih0 + r, iw = iw0 + s;
      const bool in = j0 + e < rsc && ih >= 0 && ih < q.H && iw >= 0 && iw < q.W;
      vals[e] = in ? xn[ih * q.sH + iw * q.sW + c] : bf16raw{0};
      if (++c == q.C) {
        c = 0;
        if (++s == q.S) {
          s = 0;
          ++r;
        }
      }
    }
    V8 v;
#pragma unroll
    for (int e = 0; e < 8; ++e) v.h[e] = vals[e];
    *reinterpret_cast<V8*>(col + static_cast<size_t>(g) * 8) = v;
  }
}

// ---------------------------------------------------------------- col2im
struct GatherGeom {
  int H, W, C, OH, OW, R, S, stride, pad, Kc, G;  // C per group; gcol [P][G][Kc]
  uint32_t total;  // N * H * W * G * C / 8
  FastDivU32 d_c8, d_w, d_h, d_gc8;  // d_c8: G*C/8 per pixel, d_gc8: C/8 per group
};

// gx[n][h][w][c] = sum over taps (r, s) hitting (h, w) of gcol[p(oh, ow)][(r*S+s)*C + c]
__global__ void __launch_bounds__(256) col2im_kernel(const bf16raw* __restrict__ gcol,
                                                     bf16raw* __restrict__ gx, GatherGeom q) {
  const uint32_t step = gridDim.x * blockDim.x;
  const int C8 = q.G * q.C / 8;
  for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < q.total; g += step) {
    const uint32_t pix = fdiv(g, q.d_c8);
    const int gc8 = static_cast<int>(g - pix * C8);
    const int grp = static_cast<int>(fdiv(static_cast<uint32_t>(gc8), q.d_gc8));
    const int c8 = gc8 - grp * (q.C / 8);
    const bf16raw* gsrc = gcol + static_cast<size_t>(grp) * q.Kc;
    const uint32_t p2 = fdiv(pix, q.d_w);
    const int w = static_cast<int>(pix - p2 * q.W);
    const uint32_t n = fdiv(p2, q.d_h);
    const int h = static_cast<int>(p2 - n * q.H);
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
    for (int r = 0; r < q.R; ++r) {
      const int th = h + q.pad - r;  // = oh * stride
      if (th < 0 || th % q.stride) continue;
      const int oh = th / q.stride;
      if (oh >= q.OH) continue;
      for (int s = 0; s < q.S; ++s) {
        const int tw = w + q.pad - s;
        if (tw < 0 || tw % q.stride) continue;
        const int ow = tw / q.stride;
        if (ow >= q.OW) continue;
        const size_t p = (static_cast<size_t>(n) * q.OH + oh) * q.OW + ow;
        const V8 v = *reinterpret_cast<const V8*>(gsrc + p * q.G * q.Kc + (r * q.S + s) * q.C + c8 * 8);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += bf2f(v.h[e]);
      }
    }
    V8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o.h[e] = f2bf(acc[e]);
    *reinterpret_cast<V8*>(gx + static_cast<size_t>(g) * 8) = o;
  }
}

// ---------------------------------------------------------------- weights
// w fp32 [K][C][R][S] -> bf16 [K][Kc], column (r*S + s)*C + c, zero padding
__global__ void __launch_bounds__(256) weight_rsc_kernel(const float* __restrict__ w,
                                                         bf16raw* __restrict__ out, int K, int C,
                                                         int RS, int Kc) {
  const int64_t total = static_cast<int64_t>(K) * Kc;
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int k = static_cast<int>(i / Kc), j = static_cast<int>(i - static_cast<int64_t>(k) * Kc);
    bf16raw v = 0;
    if (j < RS * C) {
      const int tap = j / C, c = j - tap * C;
      v = f2bf(w[(static_cast<int64_t>(k) * C + c) * RS + tap]);
    }
    out[i] = v;
  }
}

// dst[g][k][c][t] (+)= sum_{u < splits} src[g*splits + u][k][t*C + c]   (u in order)
__global__ void __launch_bounds__(256) wgrad_rsc_add_kernel(float* __restrict__ dst, int64_t dst_ld,
                                                            const float* __restrict__ src, int G,
                                                            int splits, int K, int C, int RS, int Kc,
                                                            int accumulate) {
  const int per = K * C * RS;
  const int64_t total = static_cast<int64_t>(G) * per;
  const int64_t plane = static_cast<int64_t>(K) * Kc;
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int g = static_cast<int>(i / per);
    const int rem = static_cast<int>(i - static_cast<int64_t>(g) * per);
    const int k = rem / (C * RS);
    const int ct = rem - k * (C * RS);
    const int c = ct / RS, t = ct - c * RS;
    const float* s0 = src + static_cast<int64_t>(g) * splits * plane + static_cast<int64_t>(k) * Kc + t * C + c;
    float acc = 0.f;
    for (int u = 0; u < splits; ++u) acc += s0[u * plane];
    float* d = dst + g * dst_ld + rem;
    *d = accumulate ? *d + acc : acc;
  }
}

// RS == 1 (1x1 convs): dst[g][k][c..c+3] (+)= sum_u src[g*splits + u][k][c..c+3],
// float4 per thread, 8 split loads in flight, summed in split order
__global__ void __launch_bounds__(256) wgrad_split_add4_kernel(float* __restrict__ dst, int64_t dst_ld,
                                                              const float* __restrict__ src, int G,
                                                              int splits, int KC, int accumulate) {
  const int per4 = KC / 4;
  const int64_t total = static_cast<int64_t>(G) * per4;
  const int64_t plane = KC;
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int g = static_cast<int>(i / per4);
    const int e = static_cast<int>(i - static_cast<int64_t>(g) * per4) * 4;
    const float* s0 = src + static_cast<int64_t>(g) * splits * plane + e;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    constexpr int kU = 8;
    for (int u0 = 0; u0 < splits; u0 += kU) {
      float4 v[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u)
        v[u] = u0 + u < splits ? *reinterpret_cast<const float4*>(s0 + (u0 + u) * plane)
                               : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        acc.x += v[u].x;
        acc.y += v[u].y;
        acc.z += v[u].z;
        acc.w += v[u].w;
      }
    }
    float4* d = reinterpret_cast<float4*>(dst + g * dst_ld + e);
    if (accumulate) {
      const float4 o = *d;
      acc.x += o.x;
      acc.y += o.y;
      acc.z += o.z;
      acc.w += o.w;
    }
    *d = acc;
  }
}

// ---------------------------------------------------------------- max-pool
struct MaxPoolGeom {
  int H, W, C, OH, OW, k, s, p;
  uint32_t total;
  FastDivU32 d_c8, d_w, d_h;  // output (fwd) or input (bwd) grid
};

// KK > 0: a compile-time k x k window whose KK*KK loads are all issued before
// the first comparison (clamped addresses, validity applied at use; the
// runtime-k loop waited for each load inside its bounds branch)
template <int KK>
__global__ void __launch_bounds__(256) maxpool_fwd_kernel(const bf16raw* __restrict__ x,
                                                          bf16raw* __restrict__ y,
                                                          uint8_t* __restrict__ codes, MaxPoolGeom q) {
  const uint32_t step = gridDim.x * blockDim.x;
  const int C8 = q.C / 8;
  const int k = KK > 0 ? KK : q.k;
  for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < q.total; g += step) {
    const uint32_t pix = fdiv(g, q.d_c8);
    const int c8 = static_cast<int>(g - pix * C8);
    const uint32_t p2 = fdiv(pix, q.d_w);
    const int ow = static_cast<int>(pix - p2 * q.OW);
    const uint32_t n = fdiv(p2, q.d_h);
    const int oh = static_cast<int>(p2 - n * q.OH);
    float best[8];
    uint32_t arg[8];
    bool first = true;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      best[e] = 0.f;
      arg[e] = 0;
    }
    const int h0 = oh * q.s - q.p, w0 = ow * q.s - q.p;
    const bf16raw* xn = x + static_cast<size_t>(n) * q.H * q.W * q.C + c8 * 8;
    auto take = [&](const V8& v, uint32_t code) __attribute__((always_inline)) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float f = bf2f(v.h[e]);
        // first maximum in window order; a NaN wins and stays (PyTorch's rule)
        if (first || f > best[e] || (f != f && best[e] == best[e])) {
          best[e] = f;
          arg[e] = code;
        }
      }
      first = false;
    };
    if constexpr (KK > 0) {
      V8 v[KK * KK];
      bool ok[KK * KK];
#pragma unroll
      for (int t = 0; t < KK * KK; ++t) {
        const int ih = h0 + t / KK, iw = w0 + t % KK;
        ok[t] = ih >= 0 && ih < q.H && iw >= 0 && iw < q.W;
        const int ihc = min(max(ih, 0), q.H - 1), iwc = min(max(iw, 0), q.W - 1);
        v[t] = *reinterpret_cast<const V8*>(xn + (static_cast<size_t>(ihc) * q.W + iwc) * q.C);
      }
#pragma unroll
      for (int t = 0; t < KK * KK; ++t)
        if (ok[t]) take(v[t], static_cast<uint32_t>(t));
    } else {
      for (int dy = 0; dy < k; ++dy) {
        const int ih = h0 + dy;
        if (ih < 0 || ih >= q.H) continue;
        for (int dx = 0; dx < k; ++dx) {
          const int iw = w0 + dx;
          if (iw < 0 || iw >= q.W) continue;
          take(*reinterpret_cast<const V8*>(xn + (static_cast<size_t>(ih) * q.W + iw) * q.C),
               static_cast<uint32_t>(dy * k + dx));
        }
      }
    }
    V8 o;
    uint64_t cw = 0;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      o.h[e] = static_cast<bf16raw>(__float_as_uint(best[e]) >> 16);  // an input value: exact
      cw |= static_cast<uint64_t>(arg[e]) << (8 * e);
    }
    *reinterpret_cast<V8*>(y + static_cast<size_t>(g) * 8) = o;
    *reinterpret_cast<uint64_t*>(codes + static_cast<size_t>(g) * 8) = cw;
  }
}

// NW > 0: at most NW x NW windows contain an input pixel (k = 3, s = 2: 2 x 2);
// their code and gradient loads are all issued before the first use
template <int NW>
__global__ void __launch_bounds__(256) maxpool_bwd_kernel(const bf16raw* __restrict__ gy,
                                                          const uint8_t* __restrict__ codes,
                                                          bf16raw* __restrict__ gx, MaxPoolGeom q) {
  const uint32_t step = gridDim.x * blockDim.x;
  const int C8 = q.C / 8;
  for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < q.total; g += step) {
    const uint32_t pix = fdiv(g, q.d_c8);
    const int c8 = static_cast<int>(g - pix * C8);
    const uint32_t p2 = fdiv(pix, q.d_w);
    const int w = static_cast<int>(pix - p2 * q.W);
    const uint32_t n = fdiv(p2, q.d_h);
    const int h = static_cast<int>(p2 - n * q.H);
    // outputs whose window [o*s - p, o*s - p + k) contains h
    const int th = h + q.p, tw = w + q.p;
    const int oh_lo = th - q.k + 1 > 0 ? (th - q.k + 1 + q.s - 1) / q.s : 0;
    const int oh_hi = min(th / q.s, q.OH - 1);
    const int ow_lo = tw - q.k + 1 > 0 ? (tw - q.k + 1 + q.s - 1) / q.s : 0;
    const int ow_hi = min(tw / q.s, q.OW - 1);
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
    const size_t nb = static_cast<size_t>(n) * q.OH * q.OW;
    if constexpr (NW > 0) {
      uint64_t cw[NW * NW];
      V8 v[NW * NW];
      bool ok[NW * NW];
      uint32_t want[NW * NW];
#pragma unroll
      for (int t = 0; t < NW * NW; ++t) {
        const int oh = oh_lo + t / NW, ow = ow_lo + t % NW;
        ok[t] = oh <= oh_hi && ow <= ow_hi;
        const int ohc = min(oh, q.OH - 1), owc = min(ow, q.OW - 1);
        want[t] = static_cast<uint32_t>((th - oh * q.s) * q.k + (tw - ow * q.s));
        const size_t o = (nb + static_cast<size_t>(ohc) * q.OW + owc) * q.C + c8 * 8;
        cw[t] = *reinterpret_cast<const uint64_t*>(codes + o);
        v[t] = *reinterpret_cast<const V8*>(gy + o);
      }
      // (window order, as the runtime loop: row-major over (oh, ow))
#pragma unroll
      for (int t = 0; t < NW * NW; ++t) {
        if (!ok[t]) continue;
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (((cw[t] >> (8 * e)) & 0xffu) == want[t]) acc[e] += bf2f(v[t].h[e]);
      }
    } else {
      for (int oh = oh_lo; oh <= oh_hi; ++oh) {
        for (int ow = ow_lo; ow <= ow_hi; ++ow) {
          const uint32_t want = static_cast<uint32_t>((th - oh * q.s) * q.k + (tw - ow * q.s));
          const size_t o = (nb + static_cast<size_t>(oh) * q.OW + ow) * q.C + c8 * 8;
          const uint64_t cw = *reinterpret_cast<const uint64_t*>(codes + o);
          const V8 v = *reinterpret_cast<const V8*>(gy + o);
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (((cw >> (8 * e)) & 0xffu) == want) acc[e] += bf2f(v.h[e]);
        }
      }
    }
    V8 out;
#pragma unroll
    for (int e = 0; e < 8; ++e) out.h[e] = f2bf(acc[e]);
    *reinterpret_cast<V8*>(gx + static_cast<size_t>(g) * 8) = out;
  }
}

}  // namespace

void launch_im2col(const Im2colArgs& a, hipStream_t stream) {
  const int G = a.G > 1 ? a.G : 1;
  const int64_t P = static_cast<int64_t>(a.N) * a.OH * a.OW;
  const int64_t total = P * G * (a.Kc / 8);
  if (total == 0) return;
  ColGeom q;
  q.H = a.H; q.W = a.W; q.C = a.C; q.OH = a.OH; q.OW = a.OW; q.R = a.R; q.S = a.S;
  q.stride = a.stride; q.pad = a.pad; q.Kc = a.Kc; q.KC8 = a.Kc / 8;
  q.sN = a.sN; q.sH = a.sH; q.sW = a.sW;
  q.sG = a.sG;
  q.total = static_cast<uint32_t>(total);
  q.d_g = make_fastdiv(G);
  q.d_kc8 = make_fastdiv(q.KC8);
  q.d_ow = make_fastdiv(a.OW);
  q.d_oh = make_fastdiv(a.OH);
  q.d_c8 = make_fastdiv(a.C % 8 == 0 ? a.C / 8 : 1);
  q.d_s = make_fastdiv(a.S);
  q.d_c = make_fastdiv(a.C);
  if (a.vec)
    COMMEFF_LAUNCH(im2col_vec_kernel, dim3(blocks_for(total)), dim3(256), 0, stream, a.x, a.col, q);
  else
    COMMEFF_LAUNCH(im2col_any_kernel, dim3(blocks_for(total)), dim3(256), 0, stream, a.x, a.col, q);
}

void launch_col2im(const Im2colArgs& a, const uint16_t* gcol, uint16_t* gx, hipStream_t stream) {
  const int G = a.G > 1 ? a.G : 1;
  const int64_t total = static_cast<int64_t>(a.N) * a.H * a.W * G * (a.C / 8);
  if (total == 0) return;
  GatherGeom q;
  q.H = a.H; q.W = a.W; q.C = a.C; q.OH = a.OH; q.OW = a.OW; q.R = a.R; q.S = a.S;
  q.stride = a.stride; q.pad = a.pad; q.Kc = a.Kc; q.G = G;
  q.total = static_cast<uint32_t>(total);
  q.d_c8 = make_fastdiv(G * a.C / 8);
  q.d_gc8 = make_fastdiv(a.C / 8);
  q.d_w = make_fastdiv(a.W);
  q.d_h = make_fastdiv(a.H);
  COMMEFF_LAUNCH(col2im_kernel, dim3(blocks_for(total)), dim3(256), 0, stream, gcol, gx, q);
}

void launch_weight_rsc(const float* w, uint16_t* out, int K, int C, int RS, int Kc, hipStream_t stream) {
  const int64_t total = static_cast<int64_t>(K) * Kc;
  if (total == 0) return;
  COMMEFF_LAUNCH(weight_rsc_kernel, dim3(blocks_for(total)), dim3(256), 0, stream, w, out, K, C, RS,
                     Kc);
}

void launch_wgrad_rsc_add(float* dst, int64_t dst_ld, const float* src, int G, int splits, int K, int C,
                          int RS, int Kc, bool accumulate, hipStream_t stream) {
  const int64_t total = static_cast<int64_t>(G) * K * C * RS;
  if (total == 0) return;
  const bool al16 = reinterpret_cast<uintptr_t>(dst) % 16 == 0 && reinterpret_cast<uintptr_t>(src) % 16 == 0 &&
                    (G == 1 || dst_ld % 4 == 0);
  if (RS == 1 && Kc == C && (K * C) % 4 == 0 && al16) {
    COMMEFF_LAUNCH(wgrad_split_add4_kernel, dim3(blocks_for(total / 4)), dim3(256), 0, stream, dst, dst_ld,
                       src, G, splits, K * C, accumulate ? 1 : 0);
    return;
  }
  COMMEFF_LAUNCH(wgrad_rsc_add_kernel, dim3(blocks_for(total)), dim3(256), 0, stream, dst, dst_ld, src,
                     G, splits, K, C, RS, Kc, accumulate ? 1 : 0);
}

void launch_maxpool_fwd(const uint16_t* x, uint16_t* y, uint8_t* codes, int N, int H, int W, int C, int k,
                        int s, int p, hipStream_t stream) {
  MaxPoolGeom q;
  q.H = H; q.W = W; q.C = C; q.k = k; q.s = s; q.p = p;
  q.OH = (H + 2 * p - k) / s + 1;
  q.OW = (W + 2 * p - k) / s + 1;
  const int64_t total = static_cast<int64_t>(N) * q.OH * q.OW * (C / 8);
  if (total == 0) return;
  q.total = static_cast<uint32_t>(total);
  q.d_c8 = make_fastdiv(C / 8);
  q.d_w = make_fastdiv(q.OW);
  q.d_h = make_fastdiv(q.OH);
  if (k == 3)
    COMMEFF_LAUNCH(maxpool_fwd_kernel<3>, dim3(blocks_for(total)), dim3(256), 0, stream, x, y, codes, q);
  else
    COMMEFF_LAUNCH(maxpool_fwd_kernel<0>, dim3(blocks_for(total)), dim3(256), 0, stream, x, y, codes, q);
}

void launch_maxpool_bwd(const uint16_t* gy, const uint8_t* codes, uint16_t* gx, int N, int H, int W, int C,
                        int k, int s, int p, hipStream_t stream) {
  MaxPoolGeom q;
  q.H = H; q.W = W; q.C = C; q.k = k; q.s = s; q.p = p;
  q.OH = (H + 2 * p - k) / s + 1;
  q.OW = (W + 2 * p - k) / s + 1;
  const int64_t total = static_cast<int64_t>(N) * H * W * (C / 8);
  if (total == 0) return;
  q.total = static_cast<uint32_t>(total);
  q.d_c8 = make_fastdiv(C / 8);
  q.d_w = make_fastdiv(W);
  q.d_h = make_fastdiv(H);
  if (k == 3 && s == 2)  // every input pixel in at most 2 x 2 windows
    COMMEFF_LAUNCH(maxpool_bwd_kernel<2>, dim3(blocks_for(total)), dim3(256), 0, stream, gy, codes, gx, q);
  else
    COMMEFF_LAUNCH(maxpool_bwd_kernel<0>, dim3(blocks_for(total)), dim3(256), 0, stream, gy, codes, gx, q);
}

}  // namespace commeff
