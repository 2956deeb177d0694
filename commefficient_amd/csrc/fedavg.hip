// Batched FedAvg local SGD (parallel/fedavg_native.py) for gfx950: the
// elementwise / layout kernels around the convolutions of G clients trained
// side by side.
//
// Reference: /root/reference/CommEfficient/fed_worker.py:61-113 (local SGD of
// one client at a time: every client copies the server weights, takes its
// local steps -- clip, weight decay, SGD -- and uploads n (w0 - w)).  Here the
// G clients of a round are one program: their weights are the rows of one fp32
// [G, ld] matrix, their activations are channel-stacked ([pixels][G*C]: each
// client's channels side by side, the grouped halo convolutions of conv.hip),
// and the per-client tails below run over all rows in one launch each:
//   * weight_image_kernel: per-step bf16 images of every client's conv weight
//     (halo forward [G K][3][3][C], flipped halo dgrad [G C][3][3][K], column
//     GEMM [G][K][Kc]) straight from the fp32 rows;
//   * row_sumsq_kernel + row_sgd_kernel: per-client gradient norm (fixed-order
//     partials), then clip + weight decay + SGD of every row in one pass;
//   * upload_kernel: out += n sum_g (w0 - w_g), clients in order;
//   * avgmax_head_*: the ResNet-18 head's avg || max pool of the channel-stacked
//     4x4 maps into per-client [n][2C] features, and its gather backward;
//   * ew_bf16_kernel: residual adds / the stem ReLU (16-byte moves).
#include <hip/hip_runtime.h>
#include <cstdint>
#include "kernels.h"

namespace commeff {
namespace {

typedef uint16_t bf16raw;
typedef uint32_t u4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float bf2f(bf16raw v) { return __uint_as_float(static_cast<uint32_t>(v) << 16); }

__device__ __forceinline__ bf16raw f2bf(float f) {  // round to nearest even (NaN kept quiet)
  const uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return static_cast<bf16raw>((u >> 16) | 0x40u);
  return static_cast<bf16raw>((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

int grid_for(int64_t n, int64_t cap = 16384) {
  int64_t b = (n + 255) / 256;
  if (b < 1) b = 1;
  return static_cast<int>(b < cap ? b : cap);
}

// ------------------------------------------------------------ weight images
// source element of (client g, out k, in c, tap t): W[g*ld + (k*C + c)*RS + t]
// kind 0: dst[((g*K + k)*RS + t)*C + c]                (halo forward)
// kind 1: dst[((g*C + c)*RS + t)*K + k] = tap RS-1-t   (halo dgrad: flipped, transposed)
// kind 2: dst[(g*K + k)*Kc + t*C + c], zero past RS*C  (column-GEMM image)
__global__ void __launch_bounds__(256) weight_image_kernel(const float* __restrict__ W, int64_t ld, int G,
                                                           int K, int C, int RS, int Kc, int kind,
                                                           bf16raw* __restrict__ dst) {
  const int64_t per = kind == 2 ? static_cast<int64_t>(K) * Kc : static_cast<int64_t>(K) * C * RS;
  const int64_t total = per * G;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += static_cast<int64_t>(gridDim.x) * 256) {
    const int g = static_cast<int>(i / per);
    const int64_t r = i - g * per;
    int k, c, t;
    bool pad = false;
    if (kind == 0) {
      c = static_cast<int>(r % C);
      const int64_t kt = r / C;
      t = static_cast<int>(kt % RS);
      k = static_cast<int>(kt / RS);
    } else if (kind == 1) {
      k = static_cast<int>(r % K);
      const int64_t ct = r / K;
      t = RS - 1 - static_cast<int>(ct % RS);
      c = static_cast<int>(ct / RS);
    } else {
      const int j = static_cast<int>(r % Kc);
      k = static_cast<int>(r / Kc);
      pad = j >= RS * C;
      t = pad ? 0 : j / C;
      c = pad ? 0 : j - t * C;
    }
    dst[i] = pad ? bf16raw(0) : f2bf(W[g * ld + (static_cast<int64_t>(k) * C + c) * RS + t]);
  }
}

// ------------------------------------------------------------- per-row SGD
constexpr int kRowParts = 64;  // partial sums per row (fixed order)

// part[g*kRowParts + b] = sum of squares of block b's share of row g
__global__ void __launch_bounds__(256) row_sumsq_kernel(const float* __restrict__ Gr, int64_t ld, int64_t d4,
                                                        float* __restrict__ part) {
  __shared__ float red[256];
  const int g = blockIdx.y, b = blockIdx.x;
  const float4* row = reinterpret_cast<const float4*>(Gr + g * ld);
  float acc = 0.f;
  for (int64_t i = b * 256ll + threadIdx.x; i < d4; i += kRowParts * 256ll) {
    const float4 v = row[i];
    acc += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[g * kRowParts + b] = red[0];
}

// W[g] = S[g] - lr * (scale_g * G[g] + wd * S[g]),  scale_g = clip / |G[g]| when
// that is < 1 (clip > 0), else 1.  S = W (in place) or the broadcast w0 (sld 0)
__global__ void __launch_bounds__(256) row_sgd_kernel(float* __restrict__ W, int64_t ld,
                                                      const float* __restrict__ Src, int64_t sld,
                                                      const float* __restrict__ Gr, int64_t gld, int64_t d4,
                                                      const float* __restrict__ part, float clip, float lr,
                                                      float wd, bf16raw* __restrict__ Wb) {
  const int g = blockIdx.y;
  float scale = 1.f;
  if (clip > 0.f) {
    float s = 0.f;
    for (int b = 0; b < kRowParts; ++b) s += part[g * kRowParts + b];
    const float nrm = sqrtf(s);
    if (nrm > clip) scale = clip / nrm;
  }
  const float a = -lr * scale, c = 1.f - lr * wd;
  float4* w = reinterpret_cast<float4*>(W + g * ld);
  const float4* src = reinterpret_cast<const float4*>(Src + g * sld);
  const float4* gr = reinterpret_cast<const float4*>(Gr + g * gld);
  uint2* wb = Wb != nullptr ? reinterpret_cast<uint2*>(Wb + g * ld) : nullptr;
  // 4 float4 of W and of G in flight per thread (one per pass: ~5.4 TB/s)
  constexpr int U = 4;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * 256;
  for (int64_t i0 = blockIdx.x * 256ll + threadIdx.x; i0 < d4; i0 += U * stride) {
    float4 sv[U], qv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + u * stride;
      if (i < d4) {
        sv[u] = src[i];
        qv[u] = gr[i];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + u * stride;
      if (i >= d4) break;
      const float4 s = sv[u], q = qv[u];
      const float4 o = make_float4(c * s.x + a * q.x, c * s.y + a * q.y, c * s.z + a * q.z, c * s.w + a * q.w);
      w[i] = o;
      // the bf16 mirror the next step's convolutions read (same row layout)
      if (wb != nullptr)
        wb[i] = make_uint2(static_cast<uint32_t>(f2bf(o.x)) | (static_cast<uint32_t>(f2bf(o.y)) << 16),
                           static_cast<uint32_t>(f2bf(o.z)) | (static_cast<uint32_t>(f2bf(o.w)) << 16));
    }
  }
}

// out[j] += n * sum_g (w0[j] - W[g][j]), clients in order (exact zeros where no
// client moved a coordinate)
// (perm: the rows hold the engine's layout, element j of a row is coordinate
// perm[j] of the flat vector; a bijection, so the scattered adds never collide)
// 4 columns a thread (16-byte loads; ld % 4 == 0), 8 client rows' loads in
// flight before they are added in client order (one row at a time: 3.5 TB/s)
// (perm: internal position -> coordinate of out; < 0 or >= dout: layout padding, skipped)
__global__ void __launch_bounds__(256) upload_kernel(float* __restrict__ out, const float* __restrict__ w0,
                                                     const float* __restrict__ W, int64_t ld, int G, int64_t d,
                                                     float n, const int32_t* __restrict__ perm, int64_t dout) {
  const int64_t d4 = d / 4;
  for (int64_t j4 = blockIdx.x * 256ll + threadIdx.x; j4 < d4; j4 += static_cast<int64_t>(gridDim.x) * 256) {
    const float4 w = reinterpret_cast<const float4*>(w0)[j4];
    const float4* col = reinterpret_cast<const float4*>(W) + j4;
    const int64_t ld4 = ld / 4;
    float4 acc = {0.f, 0.f, 0.f, 0.f};
    int g = 0;
    for (; g + 8 <= G; g += 8) {
      float4 v[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = col[(g + q) * ld4];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        acc.x += w.x - v[q].x;
        acc.y += w.y - v[q].y;
        acc.z += w.z - v[q].z;
        acc.w += w.w - v[q].w;
      }
    }
    for (; g < G; ++g) {
      const float4 v = col[g * ld4];
      acc.x += w.x - v.x;
      acc.y += w.y - v.y;
      acc.z += w.z - v.z;
      acc.w += w.w - v.w;
    }
    const int64_t j = j4 * 4;
    const float a4[4] = {acc.x, acc.y, acc.z, acc.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t o = perm != nullptr ? perm[j + q] : j + q;
      if (o >= 0 && o < dout) out[o] += n * a4[q];
    }
  }
  // the last d % 4 columns
  for (int64_t j = d4 * 4 + blockIdx.x * 256ll + threadIdx.x; j < d; j += static_cast<int64_t>(gridDim.x) * 256) {
    const float w = w0[j];
    float acc = 0.f;
    for (int g = 0; g < G; ++g) acc += w - W[g * ld + j];
    const int64_t o = perm != nullptr ? perm[j] : j;
    if (o >= 0 && o < dout) out[o] += n * acc;
  }
}

// W[g][j] = src[j] (every client row = the server row), float4
__global__ void __launch_bounds__(256) bcast_rows_kernel(float* __restrict__ W, int64_t ld,
                                                         const float* __restrict__ src, int64_t d4) {
  float4* w = reinterpret_cast<float4*>(W + blockIdx.y * ld);
  const float4* s = reinterpret_cast<const float4*>(src);
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < d4; i += static_cast<int64_t>(gridDim.x) * 256) w[i] = s[i];
}

// Wb[g*ld + off + j] = bf16(W[g*ld + off + j]), j < n (a segment's bf16 mirror)
__global__ void __launch_bounds__(256) cast_rows_kernel(uint16_t* __restrict__ Wb, const float* __restrict__ W,
                                                        int64_t ld, int64_t off, int64_t n) {
  const float* w = W + blockIdx.y * ld + off;
  uint16_t* b = Wb + blockIdx.y * ld + off;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += static_cast<int64_t>(gridDim.x) * 256)
    b[i] = f2bf(w[i]);
}

// dst[j] = src[perm[j]] (the server weights in the engine's layout) and its bf16 copy
__global__ void __launch_bounds__(256) gather_rows_kernel(float* __restrict__ dst, bf16raw* __restrict__ dstb,
                                                          const float* __restrict__ src,
                                                          const int32_t* __restrict__ perm, int64_t d,
                                                          int64_t dsrc) {
  for (int64_t j = blockIdx.x * 256ll + threadIdx.x; j < d; j += static_cast<int64_t>(gridDim.x) * 256) {
    const int32_t pj = perm[j];
    const float v = pj >= 0 && pj < dsrc ? src[pj] : 0.f;  // (layout padding: 0)
    dst[j] = v;
    dstb[j] = f2bf(v);
  }
}

// flipped, transposed dgrad image of 3x3 weights held as bf16 (r, s, c) rows:
// src[g*ld + (k*9 + t)*C + c] -> dst[((g*C + c)*9 + 8 - t)*K + k].  Per client
// a [K][9C] -> [9C][K] transpose in 64 x 64 tiles through LDS (reads along c,
// writes along k: both coalesced).  grid (9C/64, K/64, G)
__global__ void __launch_bounds__(256) dgrad_image_kernel(const bf16raw* __restrict__ src, int64_t ld, int K,
                                                          int C, bf16raw* __restrict__ dst) {
  __shared__ bf16raw t[64][66];
  const int g = blockIdx.z, j0 = blockIdx.x * 64, k0 = blockIdx.y * 64;
  const bf16raw* s = src + g * ld;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int r = ty; r < 64; r += 4) t[r][tx] = s[static_cast<int64_t>(k0 + r) * 9 * C + j0 + tx];
  __syncthreads();
  const int tap = j0 / C, c0 = j0 - tap * C;  // 64 | C: one tap per tile
  bf16raw* d = dst + static_cast<int64_t>(g) * C * 9 * K;
  for (int r = ty; r < 64; r += 4)  // tile column r = channel c0 + r
    d[(static_cast<int64_t>(c0 + r) * 9 + 8 - tap) * K + k0 + tx] = t[tx][r];
}

// ------------------------------------------------------------------ head
// x [n][HW][G*C] bf16 -> feat [G][n][2C] fp32 (mean | max over HW), codes
// [n][G*C] (first argmax)
__global__ void __launch_bounds__(256) avgmax_head_fwd_kernel(const bf16raw* __restrict__ x, int n, int HW,
                                                              int G, int C, float* __restrict__ feat,
                                                              uint8_t* __restrict__ codes) {
  const int GC = G * C;
  const int64_t total = static_cast<int64_t>(n) * GC;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += static_cast<int64_t>(gridDim.x) * 256) {
    const int e = static_cast<int>(i / GC), gc = static_cast<int>(i - static_cast<int64_t>(e) * GC);
    const bf16raw* p = x + static_cast<int64_t>(e) * HW * GC + gc;
    float s = 0.f, m = bf2f(p[0]);
    int am = 0;
    for (int h = 0; h < HW; ++h) {
      const float v = bf2f(p[static_cast<int64_t>(h) * GC]);
      s += v;
      if (v > m) {
        m = v;
        am = h;
      }
    }
    const int g = gc / C, c = gc - g * C;
    float* f = feat + (static_cast<int64_t>(g) * n + e) * 2 * C;
    f[c] = s / HW;
    f[C + c] = m;
    codes[i] = static_cast<uint8_t>(am);
  }
}

// dx[e][h][g*C + c] = df[g][e][c] / HW + (h == code ? df[g][e][C + c] : 0)
// (df: S partial slabs [S][G][n][2C] summed in slab order -- the class-chunk
// partials of fa_linear_kernel)
__global__ void __launch_bounds__(256) avgmax_head_bwd_kernel(const float* __restrict__ df,
                                                              const uint8_t* __restrict__ codes, int n, int HW,
                                                              int G, int C, bf16raw* __restrict__ dx, int S) {
  const int GC = G * C;
  const int64_t total = static_cast<int64_t>(n) * HW * GC, slab = static_cast<int64_t>(G) * n * 2 * C;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += static_cast<int64_t>(gridDim.x) * 256) {
    const int gc = static_cast<int>(i % GC);
    const int64_t eh = i / GC;
    const int h = static_cast<int>(eh % HW), e = static_cast<int>(eh / HW);
    const int g = gc / C, c = gc - g * C;
    const float* f = df + (static_cast<int64_t>(g) * n + e) * 2 * C;
    float fa = f[c], fm = f[C + c];
    for (int q = 1; q < S; ++q) {
      fa += f[q * slab + c];
      fm += f[q * slab + C + c];
    }
    float v = fa / HW;
    if (codes[static_cast<int64_t>(e) * GC + gc] == h) v += fm;
    dx[i] = f2bf(v);
  }
}

// ------------------------------------------------------------ elementwise
// mode 0: y = a + b;  mode 1: y = relu(a)   (n8 chunks of 8 bf16)
__global__ void __launch_bounds__(256) ew_bf16_kernel(const bf16raw* __restrict__ a, const bf16raw* __restrict__ b,
                                                      bf16raw* __restrict__ y, int64_t n8, int mode) {
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n8; i += static_cast<int64_t>(gridDim.x) * 256) {
    const u4 va = reinterpret_cast<const u4*>(a)[i];
    u4 o;
    if (mode == 0) {
      const u4 vb = reinterpret_cast<const u4*>(b)[i];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float lo = bf2f(static_cast<bf16raw>(va[q] & 0xffffu)) + bf2f(static_cast<bf16raw>(vb[q] & 0xffffu));
        const float hi = bf2f(static_cast<bf16raw>(va[q] >> 16)) + bf2f(static_cast<bf16raw>(vb[q] >> 16));
        o[q] = static_cast<uint32_t>(f2bf(lo)) | (static_cast<uint32_t>(f2bf(hi)) << 16);
      }
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t lo = va[q] & 0xffffu, hi = va[q] >> 16;
        o[q] = ((lo & 0x8000u) ? 0u : lo) | (((hi & 0x8000u) ? 0u : hi) << 16);
      }
    }
    reinterpret_cast<u4*>(y)[i] = o;
  }
}

// ------------------------------------------------------------ classifier
// The per-client classifier of a local step in two kernels (replacing three
// batched hipBLASLt GEMMs, the loss kernel and the bias GEMM of the step in
// fedavg_native.py's heads):
//   fa_logits_kernel   grid (G, class blocks): logits = scale feat W^T (+ b),
//                      a wave per class, lanes over the features (coalesced
//                      row reads, 4 rows in flight a wave);
//   fa_linear_kernel   grid (G, feature blocks of 256): every block redoes its
//                      client's softmax from the logits (n x C values), then
//                      streams the client's rows once -- for each class the
//                      lanes' features accumulate the feature gradient
//                      (scale / n) sum_c gl[i][c] W[c][f] with the step's
//                      weights and write the SGD-updated weight beta src +
//                      alpha (scale / n) sum_i gl[i][c] feat[i][f] (bias:
//                      alpha / n); block 0 writes the loss and top-1.
// Each block owns distinct columns of its client's rows: every row element is
// read before it is rewritten by the same thread.
template <typename TI>
__device__ __forceinline__ float fa_ld(const TI* p, int64_t i) {
  if constexpr (sizeof(TI) == 2) return bf2f(p[i]);
  else return p[i];
}

template <typename TI, int NM>  // NM: the examples' register budget (>= n)
__global__ void __launch_bounds__(256) fa_logits_kernel(FaLinearArgs a, float* __restrict__ logits) {
  extern __shared__ float sf[];  // [n][F]
  const int g = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int n = a.n, C = a.C, F = a.F;
  const TI* feat = static_cast<const TI*>(a.feat) + g * a.fsg;
  for (int e = tid; e < n * F; e += 256) {
    const int i = e / F, f = e - i * F;
    sf[e] = fa_ld(feat, i * a.fsn + f);
  }
  __syncthreads();
  const float* Wg = a.W + g * a.wld + a.woff;
  const int c_end = min(C, static_cast<int>(blockIdx.y + 1) * kFaCls);
  for (int c0 = blockIdx.y * kFaCls + wv * 4; c0 < c_end; c0 += 16) {
    float acc[4][NM];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int i = 0; i < NM; ++i) acc[q][i] = 0.f;
    for (int f = lane; f < F; f += 64) {
      float w[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) w[q] = c0 + q < c_end ? Wg[static_cast<int64_t>(c0 + q) * F + f] : 0.f;
#pragma unroll
      for (int i = 0; i < NM; ++i) {
        if (i < n) {
          const float x = sf[i * F + f];
#pragma unroll
          for (int q = 0; q < 4; ++q) acc[q][i] = fmaf(w[q], x, acc[q][i]);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = c0 + q;
      const float b = (a.boff >= 0 && c < c_end) ? a.W[g * a.wld + a.boff + c] : 0.f;
#pragma unroll
      for (int i = 0; i < NM; ++i) {
        if (i < n) {
          float v = acc[q][i];
#pragma unroll
          for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
          if (lane == 0 && c < c_end) logits[(static_cast<int64_t>(g) * n + i) * C + c] = a.scale * v + b;
        }
      }
    }
  }
}

template <typename TI, typename TO, int NM>
__global__ void __launch_bounds__(256) fa_linear_kernel(FaLinearArgs a, const float* __restrict__ logits) {
  extern __shared__ float sm[];
  const int g = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int n = a.n, C = a.C, F = a.F;
  float* sg = sm;  // [n][C] softmax - onehot
  for (int e = tid; e < n * C; e += 256) sg[e] = logits[static_cast<int64_t>(g) * n * C + e];
  __syncthreads();
  // cross-entropy: one wave per example (max with the first index, as torch.argmax)
  for (int i = wv; i < n; i += 4) {
    float* r = sg + i * C;
    float m = -__builtin_huge_valf();
    int mi = C;
    for (int j = lane; j < C; j += 64)
      if (r[j] > m) { m = r[j]; mi = j; }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float om = __shfl_xor(m, o, 64);
      const int oi = __shfl_xor(mi, o, 64);
      if (om > m || (om == m && oi < mi)) { m = om; mi = oi; }
    }
    float sum = 0.f;
    for (int j = lane; j < C; j += 64) sum += __expf(r[j] - m);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
    int64_t t = a.y[static_cast<int64_t>(g) * n + i];
    t = t < 0 ? 0 : (t >= C ? C - 1 : t);  // (labels are valid classes; clamped for memory safety)
    const float xt = r[t];  // (read by every lane before any lane rewrites the row)
    if (lane == 0 && blockIdx.y == 0 && blockIdx.z == 0) {
      a.loss[static_cast<int64_t>(g) * n + i] = m + __logf(sum) - xt;
      a.correct[static_cast<int64_t>(g) * n + i] = mi == t ? 1.f : 0.f;
    }
    const float inv = 1.f / sum;
    for (int j = lane; j < C; j += 64) r[j] = __expf(r[j] - m) * inv - (j == t ? 1.f : 0.f);
  }
  __syncthreads();
  const int f = blockIdx.y * 256 + tid;
  // this block's classes (blockIdx.z: a chunk of a.ccs), its feature-gradient slab
  const int cb = blockIdx.z * a.ccs, ce = min(C, cb + a.ccs);
  const float sn = a.scale / n, ka = a.alpha * sn;
  float* dst = a.dst + g * a.dld;
  const float* src = a.src != nullptr ? a.src + g * a.sld : dst;
  const float* Wg = a.W + g * a.wld + a.woff;
  if (f < F) {
    const TI* feat = static_cast<const TI*>(a.feat) + g * a.fsg;
    float x[NM], d[NM];
#pragma unroll
    for (int i = 0; i < NM; ++i) {
      x[i] = i < n ? fa_ld(feat, i * a.fsn + f) : 0.f;
      d[i] = 0.f;
    }
    constexpr int U = 16;  // rows in flight (the loop is load-latency bound)
    // (later steps update the rows the forward read: one load serves both)
    const bool own = src + a.woff == Wg;
    for (int c0 = cb; c0 < ce; c0 += U) {
      float w[U], sv[U];
#pragma unroll
      for (int q = 0; q < U; ++q) w[q] = c0 + q < ce ? Wg[static_cast<int64_t>(c0 + q) * F + f] : 0.f;
#pragma unroll
      for (int q = 0; q < U; ++q)
        sv[q] = own ? w[q]
                    : ((a.beta != 0.f && c0 + q < ce) ? src[a.woff + static_cast<int64_t>(c0 + q) * F + f] : 0.f);
#pragma unroll
      for (int q = 0; q < U; ++q) {
        const int c = c0 + q;
        if (c >= ce) break;
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < NM; ++i) {
          if (i < n) {
            const float gv = sg[i * C + c];
            d[i] = fmaf(gv, w[q], d[i]);
            s = fmaf(gv, x[i], s);
          }
        }
        const int64_t o = a.woff + static_cast<int64_t>(c) * F + f;
        const float nw = a.beta * sv[q] + ka * s;
        dst[o] = nw;
        if (a.mirror != nullptr) a.mirror[g * a.mld + o] = f2bf(nw);
      }
    }
    TO* df = static_cast<TO*>(a.dfeat) + blockIdx.z * a.dss + g * a.dsg;
#pragma unroll
    for (int i = 0; i < NM; ++i) {
      if (i < n) {
        if constexpr (sizeof(TO) == 2) df[i * a.dsn + f] = f2bf(sn * d[i]);
        else df[i * a.dsn + f] = sn * d[i];
      }
    }
  }
  if (a.boff >= 0 && blockIdx.y == 0) {
    const float kb = a.alpha / n;
    for (int c = cb + tid; c < ce; c += 256) {
      float s = 0.f;
      for (int i = 0; i < n; ++i) s += sg[i * C + c];
      const int64_t o = a.boff + c;
      const float nw = a.beta != 0.f ? a.beta * src[o] + kb * s : kb * s;
      dst[o] = nw;
      if (a.mirror != nullptr) a.mirror[g * a.mld + o] = f2bf(nw);
    }
  }
}

// ------------------------------------------------------------ Fixup scalars
// Per-client scalar affine maps of the Fixup models (models/fixup.py: x + b,
// x * s + b, relu, + residual), the scalars read from the clients' fp32 rows
// (S / B [g * ld]; nullptr: none; ld 0: one pair for every group).  Activations bf16, channel-stacked
// ([pixels][G C]: group of element e = (e mod G C) / C) or client-major (the
// stem's input: group = e / per); 8 elements a thread, one group each.
__device__ __forceinline__ int64_t fa_mem(const FaAffine& a, int g, int64_t eg) {
  // element eg of group g -> memory offset
  if (a.C > 0) {
    const int64_t p = eg / a.C;
    return p * a.GC + static_cast<int64_t>(g) * a.C + (eg - p * a.C);
  }
  return static_cast<int64_t>(g) * a.per + eg;
}

__global__ void __launch_bounds__(256) fa_affine_kernel(FaAffine a) {
  const int64_t n8 = a.G * a.per / 8;
  for (int64_t q = blockIdx.x * 256ll + threadIdx.x; q < n8; q += static_cast<int64_t>(gridDim.x) * 256) {
    const int64_t e = q * 8;
    const int g = a.C > 0 ? static_cast<int>((e % a.GC) / a.C) : static_cast<int>(e / a.per);
    const float sc = a.S != nullptr ? a.S[g * a.ld] : 1.f;
    const float bi = a.B != nullptr ? a.B[g * a.ld] : 0.f;
    const float po = a.P != nullptr ? a.P[g * a.ld] : 0.f;
    const u4 xv = *reinterpret_cast<const u4*>(a.x + e);
    u4 av = {0u, 0u, 0u, 0u};
    if (a.add != nullptr) av = *reinterpret_cast<const u4*>(a.add + e);
    u4 o;
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      float v0 = fmaf(__uint_as_float(xv[h] << 16), sc, bi), v1 = fmaf(__uint_as_float(xv[h] & 0xffff0000u), sc, bi);
      if (a.add != nullptr) {
        v0 += __uint_as_float(av[h] << 16);
        v1 += __uint_as_float(av[h] & 0xffff0000u);
      }
      if (a.relu) {
        v0 = fmaxf(v0, 0.f);
        v1 = fmaxf(v1, 0.f);
      }
      v0 += po;  // (relu(.) + post bias; 0 without one)
      v1 += po;
      o[h] = static_cast<uint32_t>(f2bf(v0)) | (static_cast<uint32_t>(f2bf(v1)) << 16);
    }
    *reinterpret_cast<u4*>(a.y + e) = o;
  }
}

// backward: dpre = dy (masked by y > 0 with relu), out1 = dpre * s (+ add2),
// out2 = dpre; block (chunk, g) sums dpre and dpre * xs (no xs: dy itself,
// unmasked) over its elements of group g (fixed-order tree):
// part[(chunk * G + g) * 2 + {0, 1}]
__global__ void __launch_bounds__(256) fa_affine_bwd_kernel(FaAffine a, FaAffineBwd b) {
  __shared__ float red[2][256];
  const int g = blockIdx.y, tid = threadIdx.x;
  const int64_t e0 = static_cast<int64_t>(blockIdx.x) * b.chunk;
  const int64_t e1 = min(e0 + b.chunk, a.per);
  const float sc = a.S != nullptr ? a.S[g * a.ld] : 1.f;
  const float bi = a.B != nullptr ? a.B[g * a.ld] : 0.f;
  const bool sum_dy = b.xs == nullptr || b.mask_x;  // second sum: dy unmasked
  float s1 = 0.f, s2 = 0.f;
  for (int64_t eg = e0 + 8 * tid; eg < e1; eg += 8 * 256) {
    const int64_t m = fa_mem(a, g, eg);
    const u4 dv = *reinterpret_cast<const u4*>(b.dy + m);
    u4 yv = {0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu}, xv = {0u, 0u, 0u, 0u}, av = {0u, 0u, 0u, 0u};
    if (b.yrelu != nullptr) yv = *reinterpret_cast<const u4*>(b.yrelu + m);
    if (b.xs != nullptr) xv = *reinterpret_cast<const u4*>(b.xs + m);
    if (b.add2 != nullptr) av = *reinterpret_cast<const u4*>(b.add2 + m);
    u4 o1, o2;
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      float d[2] = {__uint_as_float(dv[h] << 16), __uint_as_float(dv[h] & 0xffff0000u)};
      if (sum_dy) s2 += d[0] + d[1];  // (no scale input / post bias: the second sum is of dy unmasked)
      if (b.mask_x) {  // relu'(pre), pre = x s + b recomputed as the forward did
        if (!(fmaf(__uint_as_float(xv[h] << 16), sc, bi) > 0.f)) d[0] = 0.f;
        if (!(fmaf(__uint_as_float(xv[h] & 0xffff0000u), sc, bi) > 0.f)) d[1] = 0.f;
      } else if (b.yrelu != nullptr) {  // relu'(pre) from the output: y > 0
        if (!(__uint_as_float(yv[h] << 16) > 0.f)) d[0] = 0.f;
        if (!(__uint_as_float(yv[h] & 0xffff0000u) > 0.f)) d[1] = 0.f;
      }
      s1 += d[0] + d[1];
      if (!sum_dy)
        s2 = fmaf(d[0], __uint_as_float(xv[h] << 16), fmaf(d[1], __uint_as_float(xv[h] & 0xffff0000u), s2));
      float r0 = d[0] * sc, r1 = d[1] * sc;
      if (b.add2 != nullptr) {
        r0 += __uint_as_float(av[h] << 16);
        r1 += __uint_as_float(av[h] & 0xffff0000u);
      }
      o1[h] = static_cast<uint32_t>(f2bf(r0)) | (static_cast<uint32_t>(f2bf(r1)) << 16);
      o2[h] = static_cast<uint32_t>(f2bf(d[0])) | (static_cast<uint32_t>(f2bf(d[1])) << 16);
    }
    if (b.out1 != nullptr) *reinterpret_cast<u4*>(b.out1 + m) = o1;
    if (b.out2 != nullptr) *reinterpret_cast<u4*>(b.out2 + m) = o2;
  }
  red[0][tid] = s1;
  red[1][tid] = s2;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) {
      red[0][tid] += red[0][tid + o];
      red[1][tid] += red[1][tid + o];
    }
    __syncthreads();
  }
  if (tid == 0) {
    b.part[(static_cast<int64_t>(blockIdx.x) * a.G + g) * 2] = red[0][0];
    b.part[(static_cast<int64_t>(blockIdx.x) * a.G + g) * 2 + 1] = red[1][0];
  }
}

// the scalars' SGD step: grad = sum over the chunks in order; dst[boff] (the
// bias: sum dpre) / dst[soff] (the scale: sum dpre x) = beta src + alpha grad
__global__ void __launch_bounds__(256) fa_scalar_sgd_kernel(const float* __restrict__ part, int chunks, int G,
                                                            float* __restrict__ dst, int64_t ld, int64_t boff,
                                                            int64_t soff, float beta, float alpha,
                                                            const float* __restrict__ src, int64_t sld) {
  const int g = blockIdx.x * 256 + threadIdx.x;
  if (g >= G) return;
  float t1 = 0.f, t2 = 0.f;
  for (int c = 0; c < chunks; ++c) {
    t1 += part[(static_cast<int64_t>(c) * G + g) * 2];
    t2 += part[(static_cast<int64_t>(c) * G + g) * 2 + 1];
  }
  const float* sr = src != nullptr ? src + g * sld : dst + g * ld;
  if (boff >= 0) dst[g * ld + boff] = beta != 0.f ? beta * sr[boff] + alpha * t1 : alpha * t1;
  if (soff >= 0) dst[g * ld + soff] = beta != 0.f ? beta * sr[soff] + alpha * t2 : alpha * t2;
}

// one group's partial sums [chunks][2] -> out[0..1], one block, fixed order
// (strided per-thread sums, then a tree): the merged-batch Fixup scalars'
// gradients (ops/fixup.py)
__global__ void __launch_bounds__(256) fx_part_sum_kernel(const float* __restrict__ part, int chunks,
                                                          float* __restrict__ out) {
  __shared__ float red[2][256];
  const int tid = threadIdx.x;
  float t1 = 0.f, t2 = 0.f;
  for (int c = tid; c < chunks; c += 256) {
    t1 += part[2 * c];
    t2 += part[2 * c + 1];
  }
  red[0][tid] = t1;
  red[1][tid] = t2;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) {
      red[0][tid] += red[0][tid + o];
      red[1][tid] += red[1][tid + o];
    }
    __syncthreads();
  }
  if (tid < 2) out[tid] = red[tid][0];
}

}  // namespace

void launch_fx_part_sum(const float* part, int chunks, float* out, hipStream_t stream) {
  COMMEFF_LAUNCH(fx_part_sum_kernel, dim3(1), dim3(256), 0, stream, part, chunks, out);
}

void launch_weight_image(const float* W, int64_t ld, int G, int K, int C, int RS, int Kc, int kind,
                         uint16_t* dst, hipStream_t stream) {
  const int64_t per = kind == 2 ? static_cast<int64_t>(K) * Kc : static_cast<int64_t>(K) * C * RS;
  if (per * G == 0) return;
  COMMEFF_LAUNCH(weight_image_kernel, dim3(grid_for(per * G)), dim3(256), 0, stream, W, ld, G, K, C, RS, Kc,
                 kind, dst);
}

void launch_row_sgd(float* W, int64_t ld, const float* src, int64_t sld, const float* Gr, int64_t gld, int G,
                    int64_t d4, float clip, float lr, float wd, float* part, uint16_t* Wb, hipStream_t stream) {
  if (G == 0 || d4 == 0) return;
  if (clip > 0.f)
    COMMEFF_LAUNCH(row_sumsq_kernel, dim3(kRowParts, G), dim3(256), 0, stream, Gr, gld, d4, part);
  int bx = static_cast<int>((d4 + 1023) / 1024);
  const int cap = (8192 + G - 1) / G;
  if (bx > cap) bx = cap;
  COMMEFF_LAUNCH(row_sgd_kernel, dim3(bx < 1 ? 1 : bx, G), dim3(256), 0, stream, W, ld, src, sld, Gr, gld, d4,
                 part, clip, lr, wd, Wb);
}

int row_sgd_parts() { return kRowParts; }

void launch_fedavg_upload(float* out, const float* w0, const float* W, int64_t ld, int G, int64_t d, float n,
                          const int32_t* perm, hipStream_t stream, int64_t dout) {
  if (d == 0) return;
  COMMEFF_LAUNCH(upload_kernel, dim3(grid_for(d)), dim3(256), 0, stream, out, w0, W, ld, G, d, n, perm,
                 dout < 0 ? d : dout);
}

void launch_gather_rows(float* dst, uint16_t* dstb, const float* src, const int32_t* perm, int64_t d,
                        hipStream_t stream, int64_t dsrc) {
  if (d == 0) return;
  COMMEFF_LAUNCH(gather_rows_kernel, dim3(grid_for(d)), dim3(256), 0, stream, dst, dstb, src, perm, d,
                 dsrc < 0 ? d : dsrc);
}

void launch_bcast_rows(float* W, int64_t ld, const float* src, int G, int64_t d4, hipStream_t stream) {
  if (G == 0 || d4 == 0) return;
  int bx = static_cast<int>((d4 + 255) / 256);
  const int cap = (8192 + G - 1) / G;
  if (bx > cap) bx = cap;
  COMMEFF_LAUNCH(bcast_rows_kernel, dim3(bx, G), dim3(256), 0, stream, W, ld, src, d4);
}

void launch_cast_rows(uint16_t* Wb, const float* W, int64_t ld, int G, int64_t off, int64_t n, hipStream_t stream) {
  if (G == 0 || n == 0) return;
  int bx = static_cast<int>((n + 255) / 256);
  const int cap = (8192 + G - 1) / G;
  if (bx > cap) bx = cap;
  COMMEFF_LAUNCH(cast_rows_kernel, dim3(bx, G), dim3(256), 0, stream, Wb, W, ld, off, n);
}

void launch_dgrad_image(const uint16_t* src, int64_t ld, int G, int K, int C, uint16_t* dst, hipStream_t stream) {
  if (G == 0) return;
  COMMEFF_LAUNCH(dgrad_image_kernel, dim3(9 * C / 64, K / 64, G), dim3(256), 0, stream, src, ld, K, C, dst);
}

void launch_avgmax_head_fwd(const uint16_t* x, int n, int HW, int G, int C, float* feat, uint8_t* codes,
                            hipStream_t stream) {
  const int64_t total = static_cast<int64_t>(n) * G * C;
  if (total == 0) return;
  COMMEFF_LAUNCH(avgmax_head_fwd_kernel, dim3(grid_for(total)), dim3(256), 0, stream, x, n, HW, G, C, feat,
                 codes);
}

void launch_avgmax_head_bwd(const float* df, const uint8_t* codes, int n, int HW, int G, int C, uint16_t* dx,
                            hipStream_t stream, int S) {
  const int64_t total = static_cast<int64_t>(n) * HW * G * C;
  if (total == 0) return;
  COMMEFF_LAUNCH(avgmax_head_bwd_kernel, dim3(grid_for(total)), dim3(256), 0, stream, df, codes, n, HW, G, C,
                 dx, S);
}

void launch_ew_bf16(const uint16_t* a, const uint16_t* b, uint16_t* y, int64_t n8, int mode, hipStream_t stream) {
  if (n8 == 0) return;
  COMMEFF_LAUNCH(ew_bf16_kernel, dim3(grid_for(n8)), dim3(256), 0, stream, a, b, y, n8, mode);
}

int64_t fa_linear_lds_bytes(int n, int C, int F) {
  const int64_t a = static_cast<int64_t>(n) * F * 4, b = static_cast<int64_t>(n) * C * 4;
  return a > b ? a : b;
}

template <int NM>
void fa_linear_launch(const FaLinearArgs& a, int G, bool feat_bf16, bool dfeat_bf16, float* logits,
                      hipStream_t stream) {
  const int l1 = a.n * a.F * 4, l2 = a.n * a.C * 4;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(fa_logits_kernel<float, NM>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, kFaMaxLds);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(fa_logits_kernel<uint16_t, NM>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, kFaMaxLds);
    attr = true;
  }
  const dim3 g1(G, (a.C + kFaCls - 1) / kFaCls), g2(G, (a.F + 255) / 256, (a.C + a.ccs - 1) / a.ccs);
  const float* lg = logits;
  if (feat_bf16) {
    COMMEFF_LAUNCH((fa_logits_kernel<uint16_t, NM>), g1, dim3(256), l1, stream, a, logits);
    if (dfeat_bf16) COMMEFF_LAUNCH((fa_linear_kernel<uint16_t, uint16_t, NM>), g2, dim3(256), l2, stream, a, lg);
    else COMMEFF_LAUNCH((fa_linear_kernel<uint16_t, float, NM>), g2, dim3(256), l2, stream, a, lg);
  } else {
    COMMEFF_LAUNCH((fa_logits_kernel<float, NM>), g1, dim3(256), l1, stream, a, logits);
    if (dfeat_bf16) COMMEFF_LAUNCH((fa_linear_kernel<float, uint16_t, NM>), g2, dim3(256), l2, stream, a, lg);
    else COMMEFF_LAUNCH((fa_linear_kernel<float, float, NM>), g2, dim3(256), l2, stream, a, lg);
  }
}

void launch_fa_linear_ce(FaLinearArgs a, int G, bool feat_bf16, bool dfeat_bf16, float* logits, hipStream_t stream) {
  if (G == 0 || a.n == 0) return;
  if (a.ccs <= 0) a.ccs = a.C;
  // (registers for the examples: a 32-wide budget for 5 examples spilled)
  if (a.n <= 8) fa_linear_launch<8>(a, G, feat_bf16, dfeat_bf16, logits, stream);
  else if (a.n <= 16) fa_linear_launch<16>(a, G, feat_bf16, dfeat_bf16, logits, stream);
  else fa_linear_launch<kFaMaxN>(a, G, feat_bf16, dfeat_bf16, logits, stream);
}

void launch_fa_affine(const FaAffine& a, hipStream_t stream) {
  const int64_t n8 = a.G * a.per / 8;
  if (n8 == 0) return;
  COMMEFF_LAUNCH(fa_affine_kernel, dim3(grid_for(n8)), dim3(256), 0, stream, a);
}

void launch_fa_affine_bwd(const FaAffine& a, const FaAffineBwd& b, int chunks, hipStream_t stream) {
  if (a.G == 0 || chunks == 0) return;
  COMMEFF_LAUNCH(fa_affine_bwd_kernel, dim3(chunks, a.G), dim3(256), 0, stream, a, b);
}

void launch_fa_scalar_sgd(const float* part, int chunks, int G, float* dst, int64_t ld, int64_t boff, int64_t soff,
                          float beta, float alpha, const float* src, int64_t sld, hipStream_t stream) {
  if (G == 0) return;
  COMMEFF_LAUNCH(fa_scalar_sgd_kernel, dim3((G + 255) / 256), dim3(256), 0, stream, part, chunks, G, dst, ld, boff,
                 soff, beta, alpha, src, sld);
}

}  // namespace commeff
