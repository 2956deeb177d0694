// Ghost batch norm (per-client batch statistics) for gfx950, NHWC bf16.
//
// The engine merges a round's clients into one forward/backward; with
// BatchNorm each client's examples must still be normalised with that
// client's own batch statistics, as in the reference where every client runs
// its own forward (/root/reference/CommEfficient/fed_worker.py:162-176,
// models/resnets.py BatchNorm2d).  The batch is G equal groups of
// M = (N/G)*H*W pixels; statistics are per (group, channel).
//
// Forward  (3 launches): partial shifted sums per (group, pixel slab) ->
//          per-(group, channel) mean / rstd and y = x A + B coefficients
//          (optionally y = relu(x A + B + residual): a ResNet block's tail)
//          (+ running-stat update with the group-averaged moments, fixed
//          order) -> y, 16-byte loads/stores.
// Backward (3 launches): partial sums of dy and dy*xhat per (group, slab) ->
//          per-(group, channel) coefficients, dweight / dbias (fixed-order
//          sums over groups: deterministic) -> dx = w rstd (dy - mean(dy) -
//          xhat mean(dy xhat)) = P dy + Q x + R.
// Sums are shifted by the group's first pixel (E[(x-K)^2] - E[x-K]^2 keeps
// fp32 accurate when |mean| >> std).  Replaces ~40 PyTorch kernels (reshape
// copies, reductions, elementwise, autograd) per BN layer.
#include <hip/hip_runtime.h>
#include <cstdint>
#include "kernels.h"

namespace commeff {
namespace {

typedef uint32_t u4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float lo_bf(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float hi_bf(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }
__device__ __forceinline__ void unpack8(const u4 v, float (&f)[8]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    f[2 * q] = lo_bf(v[q]);
    f[2 * q + 1] = hi_bf(v[q]);
  }
}
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  typedef __bf16 b2 __attribute__((ext_vector_type(2)));
  const b2 t = {static_cast<__bf16>(a), static_cast<__bf16>(b)};
  return __builtin_bit_cast(uint32_t, t);
}

// keep the bf16 lanes of d whose bit in the 1-bit ReLU mask m is set
__device__ __forceinline__ u4 relu_bits8(u4 d, uint32_t m) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t keep = (((m >> (2 * q)) & 1u) ? 0x0000ffffu : 0u) | (((m >> (2 * q + 1)) & 1u) ? 0xffff0000u : 0u);
    d[q] &= keep;
  }
  return d;
}

// bit j set: bf16 lane j of the packed y is > 0 (what relu_mask8 keeps)
__device__ __forceinline__ uint32_t pos_bits8(const u4 y) {
  uint32_t m = 0u;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t lo = y[q] & 0xffffu, hi = y[q] >> 16;
    m |= ((lo & 0x8000u) == 0u && lo != 0u ? 1u : 0u) << (2 * q);
    m |= ((hi & 0x8000u) == 0u && hi != 0u ? 1u : 0u) << (2 * q + 1);
  }
  return m;
}

// thread layout of the partial-sum kernels: CL = C/8 chunk lanes (16 bytes =
// 8 channels each) x PL = 256/CL pixel lanes; a block covers pixel slab s of
// group g, every channel.
template <bool BWD>
__global__ void __launch_bounds__(256)
bn_partial_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ dy,
                  const uint8_t* __restrict__ ybits, const float* __restrict__ stat, int C, int M,
                  int S, float* __restrict__ part, int CB) {
  // part[(g*S + s)*2*C + {0: sum, C: sum2}][c]; blockIdx.y: a block of CB
  // channels (CB = C up to 2048 channels; the channel-stacked clients of
  // parallel/fedavg_native.py have G*C of them)
  __shared__ float red[2][256][8];
  const int g = blockIdx.x / S, s = blockIdx.x - g * S;
  const int cb0 = blockIdx.y * CB;
  x += cb0;
  if (BWD) {
    dy += cb0;
    stat += cb0;
  }
  part += cb0;
  const int CL = CB >> 3, PL = 256 / CL;
  const int cl = threadIdx.x % CL, pl = threadIdx.x / CL;
  const bool active = pl < PL;
  const int per = (M + S - 1) / S;
  const int p0 = s * per, p1 = min(M, p0 + per);
  const size_t gbase = static_cast<size_t>(g) * M;
  float a[8], b[8], k[8], r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = b[j] = k[j] = r[j] = 0.f;
  if (!BWD) {
    // shift: the group's first pixel
    const u4 kv = *reinterpret_cast<const u4*>(x + gbase * C + cl * 8);
    unpack8(kv, k);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      k[j] = stat[(static_cast<size_t>(g) * 2) * C + cl * 8 + j];      // mean
      r[j] = stat[(static_cast<size_t>(g) * 2 + 1) * C + cl * 8 + j];  // rstd
    }
  }
  if (active && !BWD) {
    // forward: 4 pixels per step, their loads in flight together (one 16-byte
    // load per pixel: 2 left this pass at ~3 TB/s)
    for (int p = p0 + pl; p < p1; p += 4 * PL) {
      u4 xv[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int pq = p + q * PL;
        xv[q] = pq < p1 ? *reinterpret_cast<const u4*>(x + (gbase + pq) * C + cl * 8) : u4{0u, 0u, 0u, 0u};
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (p + q * PL >= p1) break;
        float f[8];
        unpack8(xv[q], f);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float u = f[j] - k[j];
          a[j] += u;
          b[j] += u * u;
        }
      }
    }
  }
  if (active && BWD) {
    // 4 pixels per step: their 8 x / dy loads (and ReLU bytes) in flight
    // together (2 pixels: 3.6 TB/s, 82 % of the waves waiting on memory,
    // profiles/r4_pmc_imagenet.txt)
    for (int p = p0 + pl; p < p1; p += 4 * PL) {
      u4 xv[4], dv[4];
      uint32_t mb[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int pq = p + q * PL;
        const size_t o = (gbase + pq) * C + cl * 8;
        const bool in = pq < p1;
        xv[q] = in ? *reinterpret_cast<const u4*>(x + o) : u4{0u, 0u, 0u, 0u};
        dv[q] = in ? *reinterpret_cast<const u4*>(dy + o) : u4{0u, 0u, 0u, 0u};
        mb[q] = (in && ybits != nullptr) ? ybits[(o + cb0) >> 3] : 0xffu;
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        // fused ReLU: dy where y > 0 (1 bit per element); pixels past the
        // slab load zero dy and add nothing
        const u4 dq = ybits != nullptr ? relu_bits8(dv[q], mb[q]) : dv[q];
        float f[8], e[8];
        unpack8(xv[q], f);
        unpack8(dq, e);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          a[j] += e[j];
          b[j] += e[j] * (f[j] - k[j]) * r[j];
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[0][threadIdx.x][j] = a[j];
    red[1][threadIdx.x][j] = b[j];
  }
  __syncthreads();
  // fixed-order combine over the pixel lanes: thread t < CL*8 owns (cl, j)
  for (int t = threadIdx.x; t < CL * 8; t += 256) {
    const int c8 = t >> 3, j = t & 7;
    float sa = 0.f, sb = 0.f;
    for (int q = 0; q < PL; ++q) {
      sa += red[0][q * CL + c8][j];
      sb += red[1][q * CL + c8][j];
    }
    float* o = part + static_cast<size_t>(blockIdx.x) * 2 * C;
    o[c8 * 8 + j] = sa;
    o[C + c8 * 8 + j] = sb;
  }
}

// Finalize kernels: block per 64 channels x 16 lanes.  With >= 16 groups
// thread (c, gl) takes groups gl, gl + 16, ...; with fewer (the per-client
// path: one group) the lanes split each group's slabs instead.  Every
// combine over lanes (per-group sums, running stats, dweight / dbias) runs
// in a fixed order: deterministic.
constexpr int kGL = 16;

// forward: stat[g][0][c] = mean, stat[g][1][c] = rstd (kept for backward),
// ab[g][0][c] = A = w rstd, ab[g][1][c] = B = b - mean A  (y = x A + B)
__global__ void __launch_bounds__(1024)
bn_fwd_finalize_kernel(const uint16_t* __restrict__ x, const float* __restrict__ part,
                       const float* __restrict__ w, const float* __restrict__ bias, int C, int M,
                       int S, int G, float eps, float momentum, float* __restrict__ stat,
                       float* __restrict__ ab, float* __restrict__ run_mean,
                       float* __restrict__ run_var, int64_t* __restrict__ nbt) {
  if (nbt != nullptr && blockIdx.x == 0 && threadIdx.x == 0) *nbt += 1;  // num_batches_tracked
  __shared__ float red[2][kGL][64];
  const int cc = threadIdx.x & 63, gl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cc;
  float msum = 0.f, vsum = 0.f;
  const float wc = c < C && w != nullptr ? w[c] : 1.f, bc = c < C && w != nullptr ? bias[c] : 0.f;
  auto finish = [&](int g, float s1, float s2) __attribute__((always_inline)) {
    const float kk = __uint_as_float(static_cast<uint32_t>(x[static_cast<size_t>(g) * M * C + c]) << 16);
    const float d = s1 / M;
    const float var = fmaxf(s2 / M - d * d, 0.f);
    const float mean = kk + d, rstd = rsqrtf(var + eps);
    const size_t o = static_cast<size_t>(g) * 2 * C + c;
    stat[o] = mean;
    stat[o + C] = rstd;
    ab[o] = wc * rstd;
    ab[o + C] = bc - mean * wc * rstd;
    msum += mean;
    vsum += var;
  };
  if (G < kGL) {
    // few groups (one per client-step on the per-client path): the lanes
    // split the slabs of each group instead, combined in a fixed order
    for (int g = 0; g < G; ++g) {
      float s1 = 0.f, s2 = 0.f;
      if (c < C) {
        for (int s = gl; s < S; s += kGL) {
          const float* p = part + (static_cast<size_t>(g) * S + s) * 2 * C;
          s1 += p[c];
          s2 += p[C + c];
        }
      }
      __syncthreads();  // red reuse
      red[0][gl][cc] = s1;
      red[1][gl][cc] = s2;
      __syncthreads();
      if (gl == 0 && c < C) {
        float t1 = 0.f, t2 = 0.f;
        for (int q = 0; q < kGL; ++q) {
          t1 += red[0][q][cc];
          t2 += red[1][q][cc];
        }
        finish(g, t1, t2);
      }
    }
    __syncthreads();
  } else if (c < C) {
    for (int g = gl; g < G; g += kGL) {
      float s1 = 0.f, s2 = 0.f;
      for (int s = 0; s < S; ++s) {
        const float* p = part + (static_cast<size_t>(g) * S + s) * 2 * C;
        s1 += p[c];
        s2 += p[C + c];
      }
      finish(g, s1, s2);
    }
  }
  red[0][gl][cc] = msum;
  red[1][gl][cc] = vsum;
  __syncthreads();
  if (gl == 0 && c < C && run_mean != nullptr) {
    float ms = 0.f, vs = 0.f;
    for (int q = 0; q < kGL; ++q) {
      ms += red[0][q][cc];
      vs += red[1][q][cc];
    }
    const float unb = M > 1 ? static_cast<float>(M) / static_cast<float>(M - 1) : 1.f;
    run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * (ms / G);
    run_var[c] = (1.f - momentum) * run_var[c] + momentum * (vs / G) * unb;
  }
}

// backward: with k0 = w rstd, k1 = mean(dy), k2 = mean(dy xhat) and
// xhat = (x - mean) rstd, dx = k0 (dy - k1 - xhat k2) = P dy + Q x + R:
// coef[g][0..2][c] = P, Q, R.  dw[c] = sum_g sum(dy xhat), db[c] = sum_g sum(dy);
// grouped weight gradients (parallel/grouped.py): gdw[g * gstride + c] +=
// sum(dy xhat) and gdb[...] += sum(dy) of group g alone
__global__ void __launch_bounds__(1024)
bn_bwd_finalize_kernel(const float* __restrict__ part, const float* __restrict__ stat,
                       const float* __restrict__ w, int C, int M, int S, int G,
                       float* __restrict__ coef, float* __restrict__ dw, float* __restrict__ db,
                       float beta, float* __restrict__ gdw, float* __restrict__ gdb,
                       int64_t gstride) {
  __shared__ float red[2][kGL][64];
  const int cc = threadIdx.x & 63, gl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cc;
  float tw = 0.f, tb = 0.f;
  const float wc = c < C && w != nullptr ? w[c] : 1.f;
  auto finish = [&](int g, float s1, float s2) __attribute__((always_inline)) {
    tb += s1;
    tw += s2;
    if (gdw != nullptr) {  // per-group (per-client) dweight / dbias, accumulated
      gdw[g * gstride + c] += s2;
      gdb[g * gstride + c] += s1;
    }
    const float mean = stat[static_cast<size_t>(g) * 2 * C + c];
    const float rstd = stat[static_cast<size_t>(g) * 2 * C + C + c];
    const float k0 = wc * rstd, k1 = s1 / M, k2 = s2 / M;
    float* o = coef + static_cast<size_t>(g) * 3 * C;
    o[c] = k0;
    o[C + c] = -k0 * k2 * rstd;
    o[2 * C + c] = -k0 * k1 + k0 * k2 * rstd * mean;
  };
  if (G < kGL) {  // lanes split the slabs (see the forward finalize)
    for (int g = 0; g < G; ++g) {
      float s1 = 0.f, s2 = 0.f;
      if (c < C) {
        for (int s = gl; s < S; s += kGL) {
          const float* p = part + (static_cast<size_t>(g) * S + s) * 2 * C;
          s1 += p[c];
          s2 += p[C + c];
        }
      }
      __syncthreads();
      red[0][gl][cc] = s1;
      red[1][gl][cc] = s2;
      __syncthreads();
      if (gl == 0 && c < C) {
        float t1 = 0.f, t2 = 0.f;
        for (int q = 0; q < kGL; ++q) {
          t1 += red[0][q][cc];
          t2 += red[1][q][cc];
        }
        finish(g, t1, t2);
      }
    }
    __syncthreads();
  } else if (c < C) {
    for (int g = gl; g < G; g += kGL) {
      float s1 = 0.f, s2 = 0.f;
      for (int s = 0; s < S; ++s) {
        const float* p = part + (static_cast<size_t>(g) * S + s) * 2 * C;
        s1 += p[c];
        s2 += p[C + c];
      }
      finish(g, s1, s2);
    }
  }
  red[0][gl][cc] = tw;
  red[1][gl][cc] = tb;
  __syncthreads();
  if (gl == 0 && c < C) {
    float sw = 0.f, sb = 0.f;
    for (int q = 0; q < kGL; ++q) {
      sw += red[0][q][cc];
      sb += red[1][q][cc];
    }
    // beta 1: accumulate into an existing .grad (flat-buffer views)
    if (dw != nullptr) dw[c] = beta != 0.f ? dw[c] + sw : sw;
    if (db != nullptr) db[c] = beta != 0.f ? db[c] + sb : sb;
  }
}

// ---- few groups (2 <= G < 16, e.g. 8 clients of a grouped round): the
// finalize kernels above loop over the groups serially inside 1-32 blocks
// (~17 us each at C <= 512, latency-bound).  Here one block per (64
// channels, group): its 16 lanes split the group's slabs, one fixed-order LDS
// combine.  Cross-group sums (running statistics; dweight / dbias when they
// are not grouped) go to small per-group buffers summed in a fixed order by
// one more tiny kernel.
__device__ __forceinline__ void group_slab_sums(const float* __restrict__ part, int C, int S, int g,
                                                int c, int cc, int gl, float (&red)[2][kGL][64],
                                                float* t1, float* t2) {
  float s1 = 0.f, s2 = 0.f;
  if (c < C) {
    for (int s = gl; s < S; s += kGL) {
      const float* p = part + (static_cast<size_t>(g) * S + s) * 2 * C;
      s1 += p[c];
      s2 += p[C + c];
    }
  }
  red[0][gl][cc] = s1;
  red[1][gl][cc] = s2;
  __syncthreads();
  float a = 0.f, b = 0.f;
  for (int q = 0; q < kGL; ++q) {
    a += red[0][q][cc];
    b += red[1][q][cc];
  }
  *t1 = a;
  *t2 = b;
}

// grid (C/64, G).  gmv[g][0][c] = mean, gmv[g][1][c] = var (running stats)
__global__ void __launch_bounds__(1024)
bn_fwd_finalize_group_kernel(const uint16_t* __restrict__ x, const float* __restrict__ part,
                             const float* __restrict__ w, const float* __restrict__ bias, int C,
                             int M, int S, float eps, float* __restrict__ stat,
                             float* __restrict__ ab, float* __restrict__ gmv) {
  __shared__ float red[2][kGL][64];
  const int cc = threadIdx.x & 63, gl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cc, g = blockIdx.y;
  float t1, t2;
  group_slab_sums(part, C, S, g, c, cc, gl, red, &t1, &t2);
  if (gl != 0 || c >= C) return;
  const float wc = w != nullptr ? w[c] : 1.f, bc = w != nullptr ? bias[c] : 0.f;
  const float kk = __uint_as_float(static_cast<uint32_t>(x[static_cast<size_t>(g) * M * C + c]) << 16);
  const float dd = t1 / M;
  const float var = fmaxf(t2 / M - dd * dd, 0.f);
  const float mean = kk + dd, rstd = rsqrtf(var + eps);
  const size_t o = static_cast<size_t>(g) * 2 * C + c;
  stat[o] = mean;
  stat[o + C] = rstd;
  ab[o] = wc * rstd;
  ab[o + C] = bc - mean * wc * rstd;
  gmv[o] = mean;
  gmv[o + C] = var;
}

// grid (C/64, G): group g's mean / var from the moments its producing GEMM
// wrote per 128-row tile (GemmArgs::stats: [tile][slot][mean | M2][C]; slot 0
// = the group of the tile's first row), merged with Chan's parallel formula in
// tile order (16 lanes over strided tiles, then the lanes in order:
// deterministic).  Outputs as bn_fwd_finalize_group_kernel.
__global__ void __launch_bounds__(1024)
bn_fwd_finalize_tiles_kernel(const float* __restrict__ ts, const float* __restrict__ w,
                             const float* __restrict__ bias, int C, int Mtot, int M, float eps,
                             float* __restrict__ stat, float* __restrict__ ab,
                             float* __restrict__ gmv) {
  __shared__ float red[3][kGL][64];
  const int cc = threadIdx.x & 63, gl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cc, g = blockIdx.y;
  const int lo = g * M, hi = lo + M;
  const int b0 = lo / kBnStatTile, b1 = (hi - 1) / kBnStatTile;
  float n = 0.f, mean = 0.f, m2 = 0.f;
  auto merge = [&](float nb, float mb, float qb) __attribute__((always_inline)) {
    if (nb <= 0.f) return;
    const float nn = n + nb, d = mb - mean;
    mean += d * (nb / nn);
    m2 += qb + d * d * (n * nb / nn);
    n = nn;
  };
  if (c < C) {
    for (int b = b0 + gl; b <= b1; b += kGL) {
      const int r0 = b * kBnStatTile, r1 = min(r0 + kBnStatTile, Mtot);
      const int slot = r0 / M == g ? 0 : 1;
      const int nb = min(r1, hi) - max(r0, lo);
      const float* o = ts + static_cast<size_t>(b) * 4 * C + 2 * slot * C;
      merge(static_cast<float>(nb), o[c], o[C + c]);
    }
  }
  red[0][gl][cc] = n;
  red[1][gl][cc] = mean;
  red[2][gl][cc] = m2;
  __syncthreads();
  if (gl != 0 || c >= C) return;
  n = mean = m2 = 0.f;
  for (int q = 0; q < kGL; ++q) merge(red[0][q][cc], red[1][q][cc], red[2][q][cc]);
  const float wc = w != nullptr ? w[c] : 1.f, bc = w != nullptr ? bias[c] : 0.f;
  const float var = fmaxf(m2 / static_cast<float>(M), 0.f);
  const float rstd = rsqrtf(var + eps);
  const size_t o = static_cast<size_t>(g) * 2 * C + c;
  stat[o] = mean;
  stat[o + C] = rstd;
  ab[o] = wc * rstd;
  ab[o + C] = bc - mean * wc * rstd;
  gmv[o] = mean;
  gmv[o + C] = var;
}

// running statistics from the group-averaged moments (fixed group order)
__global__ void __launch_bounds__(256)
bn_running_kernel(const float* __restrict__ gmv, int C, int M, int G, float momentum,
                  float* __restrict__ run_mean, float* __restrict__ run_var,
                  int64_t* __restrict__ nbt) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (nbt != nullptr && c == 0) *nbt += 1;
  if (c >= C || run_mean == nullptr) return;
  float ms = 0.f, vs = 0.f;
  for (int g = 0; g < G; ++g) {
    ms += gmv[static_cast<size_t>(g) * 2 * C + c];
    vs += gmv[static_cast<size_t>(g) * 2 * C + C + c];
  }
  const float unb = M > 1 ? static_cast<float>(M) / static_cast<float>(M - 1) : 1.f;
  run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * (ms / G);
  run_var[c] = (1.f - momentum) * run_var[c] + momentum * (vs / G) * unb;
}

// grid (C/64, G).  Grouped: gdw / gdb rows += the group's sums; else the
// per-group sums go to gsum[g][0..1][c] for bn_dwdb_kernel
__global__ void __launch_bounds__(1024)
bn_bwd_finalize_group_kernel(const float* __restrict__ part, const float* __restrict__ stat,
                             const float* __restrict__ w, int C, int M, int S,
                             float* __restrict__ coef, float* __restrict__ gdw,
                             float* __restrict__ gdb, int64_t gstride, float* __restrict__ gsum) {
  __shared__ float red[2][kGL][64];
  const int cc = threadIdx.x & 63, gl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cc, g = blockIdx.y;
  float s1, s2;
  group_slab_sums(part, C, S, g, c, cc, gl, red, &s1, &s2);
  if (gl != 0 || c >= C) return;
  const float wc = w != nullptr ? w[c] : 1.f;
  const float mean = stat[static_cast<size_t>(g) * 2 * C + c];
  const float rstd = stat[static_cast<size_t>(g) * 2 * C + C + c];
  const float k0 = wc * rstd, k1 = s1 / M, k2 = s2 / M;
  float* o = coef + static_cast<size_t>(g) * 3 * C;
  o[c] = k0;
  o[C + c] = -k0 * k2 * rstd;
  o[2 * C + c] = -k0 * k1 + k0 * k2 * rstd * mean;
  if (gdw != nullptr) {
    gdw[g * gstride + c] += s2;
    gdb[g * gstride + c] += s1;
  } else if (gsum != nullptr) {
    gsum[static_cast<size_t>(g) * 2 * C + c] = s2;
    gsum[static_cast<size_t>(g) * 2 * C + C + c] = s1;
  }
}

__global__ void __launch_bounds__(256)
bn_dwdb_kernel(const float* __restrict__ gsum, int C, int G, float* __restrict__ dw,
               float* __restrict__ db, float beta) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  float sw = 0.f, sb = 0.f;
  for (int g = 0; g < G; ++g) {
    sw += gsum[static_cast<size_t>(g) * 2 * C + c];
    sb += gsum[static_cast<size_t>(g) * 2 * C + C + c];
  }
  if (dw != nullptr) dw[c] = beta != 0.f ? dw[c] + sw : sw;
  if (db != nullptr) db[c] = beta != 0.f ? db[c] + sb : sb;
}

__device__ __forceinline__ void load8f(const float* p, float (&f)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
}

// fwd: y = x A + B ;  bwd: dx = P dy + Q x + R  (per-(group, channel) coefficients)
// ``aux``: forward -- a residual addend (y = act(x A + B + addend)); backward --
// an output for the ReLU-masked dy (the addend's gradient)
// POST (forward): y = relu(x A + B) + aux -- the residual add AFTER the ReLU
// (models/fixup.py PreActBlock: relu(bn2(conv2 .)) + shortcut), the ReLU bits
// of the pre-add value
// the few-group forward's running-statistics update, done by the apply
// kernel's first block (the finalize wrote every group's mean / var to gmv):
// one launch fewer per BN, the channels' group sums in group order (as
// bn_running_kernel)
struct BnRun {
  const float* gmv;
  float* run_mean;
  float* run_var;
  int64_t* nbt;
  int G;  // 0: no update
  float momentum;
};

__device__ __forceinline__ void bn_running_update(const BnRun& r, int C, int M) {
  if (r.nbt != nullptr && threadIdx.x == 0) *r.nbt += 1;
  if (r.run_mean == nullptr) return;
  const float unb = M > 1 ? static_cast<float>(M) / static_cast<float>(M - 1) : 1.f;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float ms = 0.f, vs = 0.f;
    for (int g = 0; g < r.G; ++g) {
      ms += r.gmv[static_cast<size_t>(g) * 2 * C + c];
      vs += r.gmv[static_cast<size_t>(g) * 2 * C + C + c];
    }
    r.run_mean[c] = (1.f - r.momentum) * r.run_mean[c] + r.momentum * (ms / r.G);
    r.run_var[c] = (1.f - r.momentum) * r.run_var[c] + r.momentum * (vs / r.G) * unb;
  }
}

constexpr BnRun kNoRun{nullptr, nullptr, nullptr, nullptr, 0, 0.f};

template <bool BWD, bool POST = false>
__global__ void __launch_bounds__(256)
bn_apply_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ dy,
                const uint8_t* __restrict__ ybits, const float* __restrict__ coef, int C, int M,
                uint32_t nchunks, bool relu, uint16_t* __restrict__ out,
                uint16_t* __restrict__ aux, uint8_t* __restrict__ bits_out, BnRun run) {
  if (!BWD && run.G > 0 && blockIdx.x == 0) bn_running_update(run, C, M);
  const uint32_t CL = static_cast<uint32_t>(C) >> 3;
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < nchunks; i += gridDim.x * 256u) {
    const uint32_t p = i / CL;
    const int c0 = static_cast<int>(i - p * CL) * 8;
    const int g = static_cast<int>(p / static_cast<uint32_t>(M));
    const float* k = coef + static_cast<size_t>(g) * (BWD ? 3 : 2) * C + c0;
    float f[8], A[8], B[8], o[8];
    unpack8(*reinterpret_cast<const u4*>(x + static_cast<size_t>(i) * 8), f);
    load8f(k, A);
    load8f(k + C, B);
    if (!BWD) {
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = f[j] * A[j] + B[j];
      if (!POST && aux != nullptr) {  // fused residual add (before the ReLU)
        float r8[8];
        unpack8(*reinterpret_cast<const u4*>(aux + static_cast<size_t>(i) * 8), r8);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] += r8[j];
      }
      if (relu) {
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = fmaxf(o[j], 0.f);
      }
    } else {
      float d[8], R[8];
      u4 dv = *reinterpret_cast<const u4*>(dy + static_cast<size_t>(i) * 8);
      if (ybits != nullptr) dv = relu_bits8(dv, ybits[i]);
      if (aux != nullptr) *reinterpret_cast<u4*>(aux + static_cast<size_t>(i) * 8) = dv;
      unpack8(dv, d);
      load8f(k + 2 * C, R);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = d[j] * A[j] + f[j] * B[j] + R[j];
    }
    const u4 v = {pack2(o[0], o[1]), pack2(o[2], o[3]), pack2(o[4], o[5]), pack2(o[6], o[7])};
    if (!BWD && bits_out != nullptr) bits_out[i] = static_cast<uint8_t>(pos_bits8(v));
    if (!BWD && POST) {  // residual add after the ReLU (on the bf16-rounded value)
      float r8[8], q[8];
      unpack8(*reinterpret_cast<const u4*>(aux + static_cast<size_t>(i) * 8), r8);
      unpack8(v, q);
      const u4 w = {pack2(q[0] + r8[0], q[1] + r8[1]), pack2(q[2] + r8[2], q[3] + r8[3]),
                    pack2(q[4] + r8[4], q[5] + r8[5]), pack2(q[6] + r8[6], q[7] + r8[7])};
      *reinterpret_cast<u4*>(out + static_cast<size_t>(i) * 8) = w;
    } else {
      *reinterpret_cast<u4*>(out + static_cast<size_t>(i) * 8) = v;
    }
  }
}


// ---- channel-stacked clients (parallel/fedavg_native.py): one "group" of M
// pixels whose C = G * cg channels are G clients' cg channels side by side.
// Statistics are per channel, i.e. per (client, channel); the affine
// parameters of channel c are client c / cg's, read from its fp32 parameter
// row (w[(c / cg) * ld + c % cg]); the weight / bias gradients go straight into
// the clients' gradient rows.  The lanes of a block split the slabs (the
// one-group branch of the kernels above), combined in a fixed order.
__device__ __forceinline__ void cs_slab_sums(const float* __restrict__ part, int C, int S, int c, int cc,
                                             int gl, float (&red)[2][kGL][64], float* t1, float* t2) {
  float s1 = 0.f, s2 = 0.f;
  if (c < C) {
    for (int s = gl; s < S; s += kGL) {
      const float* p = part + static_cast<size_t>(s) * 2 * C;
      s1 += p[c];
      s2 += p[C + c];
    }
  }
  red[0][gl][cc] = s1;
  red[1][gl][cc] = s2;
  __syncthreads();
  float a = 0.f, b = 0.f;
  for (int q = 0; q < kGL; ++q) {
    a += red[0][q][cc];
    b += red[1][q][cc];
  }
  *t1 = a;
  *t2 = b;
}

__global__ void __launch_bounds__(1024)
bn_cs_fwd_finalize_kernel(const uint16_t* __restrict__ x, const float* __restrict__ part,
                          const float* __restrict__ prm, int64_t ld, int64_t woff, int64_t boff, int cg,
                          int C, int M, int S, float eps, float momentum, float* __restrict__ stat,
                          float* __restrict__ ab, float* __restrict__ run_mean,
                          float* __restrict__ run_var, int64_t* __restrict__ nbt) {
  __shared__ float red[2][kGL][64];
  if (nbt != nullptr && blockIdx.x == 0 && threadIdx.x == 0) *nbt += 1;
  const int cc = threadIdx.x & 63, gl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cc;
  float t1, t2;
  cs_slab_sums(part, C, S, c, cc, gl, red, &t1, &t2);
  if (gl != 0 || c >= C) return;
  const int64_t row = static_cast<int64_t>(c / cg) * ld + c % cg;
  const float wc = prm[row + woff], bc = prm[row + boff];
  const float kk = __uint_as_float(static_cast<uint32_t>(x[c]) << 16);
  const float dd = t1 / M;
  const float var = fmaxf(t2 / M - dd * dd, 0.f);
  const float mean = kk + dd, rstd = rsqrtf(var + eps);
  stat[c] = mean;
  stat[C + c] = rstd;
  ab[c] = wc * rstd;
  ab[C + c] = bc - mean * wc * rstd;
  if (run_mean != nullptr) {  // each client's own running statistics
    const float unb = M > 1 ? static_cast<float>(M) / static_cast<float>(M - 1) : 1.f;
    run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * mean;
    run_var[c] = (1.f - momentum) * run_var[c] + momentum * var * unb;
  }
}

__global__ void __launch_bounds__(1024)
bn_cs_bwd_finalize_kernel(const float* __restrict__ part, const float* __restrict__ stat,
                          const float* __restrict__ prm, int64_t ld, int64_t woff, int cg, int C, int M,
                          int S, float* __restrict__ coef, float* __restrict__ grad, int64_t gld,
                          int64_t gwoff, int64_t gboff, float beta, float alpha,
                          const float* __restrict__ wsrc, int64_t sld) {
  __shared__ float red[2][kGL][64];
  const int cc = threadIdx.x & 63, gl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cc;
  float s1, s2;
  cs_slab_sums(part, C, S, c, cc, gl, red, &s1, &s2);
  if (gl != 0 || c >= C) return;
  const float wc = prm[static_cast<int64_t>(c / cg) * ld + c % cg + woff];
  const float mean = stat[c], rstd = stat[C + c];
  const float k0 = wc * rstd, k1 = s1 / M, k2 = s2 / M;
  coef[c] = k0;
  coef[C + c] = -k0 * k2 * rstd;
  coef[2 * C + c] = -k0 * k1 + k0 * k2 * rstd * mean;
  float* gr = grad + static_cast<int64_t>(c / cg) * gld + c % cg;
  // dweight = sum(dy xhat), dbias = sum(dy); beta / alpha: the SGD step applied
  // in place to the weight rows (read above, before this write)
  // (wsrc: beta scales the current weights' rows, sld apart / 0 shared, at
  // the same offsets -- the first local step's server row, not a copy in grad)
  const float* sr = wsrc != nullptr ? wsrc + static_cast<int64_t>(c / cg) * sld + c % cg : gr;
  gr[gwoff] = beta != 0.f ? beta * sr[gwoff] + alpha * s2 : alpha * s2;
  gr[gboff] = beta != 0.f ? beta * sr[gboff] + alpha * s1 : alpha * s1;
}

// ---- small maps (M <= 32 NP pixels: the channel-stacked 8x8 / 4x4 layers):
// statistics, finalize and apply in ONE kernel.  A block owns 64 channels of
// every pixel (8 chunk lanes of 8 channels x 32 pixel lanes), its x (and dy)
// values stay in registers between the passes; the three launches of the
// general path (partial sums, finalize, apply) were ~5 us each, latency-bound,
// on 8-16 MB tensors (FedAvg round 31.62 -> 31.10 ms, same-box A/B).  Two-pass
// moments (mean, then the centred squares) from the registers; fixed-order
// combines over the pixel lanes: deterministic.
template <int NP, bool POST>
__global__ void __launch_bounds__(256)
bn_cs_small_fwd_kernel(const uint16_t* __restrict__ x, const float* __restrict__ prm, int64_t ld,
                       int64_t woff, int64_t boff, int cg, int C, int M, float eps, float momentum,
                       float* __restrict__ stat, float* __restrict__ run_mean, float* __restrict__ run_var,
                       int64_t* __restrict__ nbt, uint16_t* __restrict__ y, uint8_t* __restrict__ bits,
                       const uint16_t* __restrict__ post_add) {
  __shared__ float red[32][65];
  __shared__ float cf[2][64];
  if (nbt != nullptr && blockIdx.x == 0 && threadIdx.x == 0) *nbt += 1;
  const int cl = threadIdx.x & 7, pl = threadIdx.x >> 3;
  const int c0 = blockIdx.x * 64 + cl * 8;
  u4 xv[NP];
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const int p = pl + 32 * i;
    xv[i] = p < M ? *reinterpret_cast<const u4*>(x + static_cast<size_t>(p) * C + c0) : u4{0u, 0u, 0u, 0u};
  }
  // pass 1: the mean
  float a[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = 0.f;
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    float f[8];
    unpack8(xv[i], f);  // (pixels past M hold zeros)
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] += f[j];
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[pl][cl * 8 + j] = a[j];
  __syncthreads();
  if (threadIdx.x < 64) {
    float t = 0.f;
    for (int q = 0; q < 32; ++q) t += red[q][threadIdx.x];
    cf[0][threadIdx.x] = t / M;
  }
  __syncthreads();
  float mean[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    mean[j] = cf[0][cl * 8 + j];
    a[j] = 0.f;
  }
  // pass 2: the centred squares
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    if (pl + 32 * i >= M) break;
    float f[8];
    unpack8(xv[i], f);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float u = f[j] - mean[j];
      a[j] += u * u;
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[pl][cl * 8 + j] = a[j];
  __syncthreads();
  if (threadIdx.x < 64) {
    float t = 0.f;
    for (int q = 0; q < 32; ++q) t += red[q][threadIdx.x];
    const int c = blockIdx.x * 64 + threadIdx.x;
    const float mu = cf[0][threadIdx.x], var = t / M, rstd = rsqrtf(var + eps);
    const int64_t row = static_cast<int64_t>(c / cg) * ld + c % cg;
    const float wc = prm[row + woff], bc = prm[row + boff];
    stat[c] = mu;
    stat[C + c] = rstd;
    cf[0][threadIdx.x] = wc * rstd;
    cf[1][threadIdx.x] = bc - mu * wc * rstd;
    if (run_mean != nullptr) {
      const float unb = M > 1 ? static_cast<float>(M) / static_cast<float>(M - 1) : 1.f;
      run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * mu;
      run_var[c] = (1.f - momentum) * run_var[c] + momentum * var * unb;
    }
  }
  __syncthreads();
  float A[8], B[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    A[j] = cf[0][cl * 8 + j];
    B[j] = cf[1][cl * 8 + j];
  }
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const int p = pl + 32 * i;
    if (p >= M) break;
    float f[8], o[8];
    unpack8(xv[i], f);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = fmaxf(f[j] * A[j] + B[j], 0.f);
    const u4 v = {pack2(o[0], o[1]), pack2(o[2], o[3]), pack2(o[4], o[5]), pack2(o[6], o[7])};
    const size_t e = static_cast<size_t>(p) * C + c0;
    if (bits != nullptr) bits[e >> 3] = static_cast<uint8_t>(pos_bits8(v));
    if (POST) {  // residual add after the ReLU, on the bf16-rounded value
      float r8[8], q[8];
      unpack8(*reinterpret_cast<const u4*>(post_add + e), r8);
      unpack8(v, q);
      *reinterpret_cast<u4*>(y + e) = u4{pack2(q[0] + r8[0], q[1] + r8[1]), pack2(q[2] + r8[2], q[3] + r8[3]),
                                          pack2(q[4] + r8[4], q[5] + r8[5]), pack2(q[6] + r8[6], q[7] + r8[7])};
    } else {
      *reinterpret_cast<u4*>(y + e) = v;
    }
  }
}

template <int NP>
__global__ void __launch_bounds__(256)
bn_cs_small_bwd_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ dy,
                       const uint8_t* __restrict__ ybits, const float* __restrict__ stat,
                       const float* __restrict__ prm, int64_t ld, int64_t woff, int cg, int C, int M,
                       float* __restrict__ grad, int64_t gld, int64_t gwoff, int64_t gboff, float beta,
                       float alpha, const float* __restrict__ wsrc, int64_t sld, uint16_t* __restrict__ dx) {
  __shared__ float red[2][32][65];
  __shared__ float cf[3][64];
  const int cl = threadIdx.x & 7, pl = threadIdx.x >> 3;
  const int c0 = blockIdx.x * 64 + cl * 8;
  u4 xv[NP], dv[NP];
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const int p = pl + 32 * i;
    const size_t e = static_cast<size_t>(p) * C + c0;
    xv[i] = p < M ? *reinterpret_cast<const u4*>(x + e) : u4{0u, 0u, 0u, 0u};
    dv[i] = p < M ? *reinterpret_cast<const u4*>(dy + e) : u4{0u, 0u, 0u, 0u};
    if (p < M && ybits != nullptr) dv[i] = relu_bits8(dv[i], ybits[e >> 3]);
  }
  float mean[8], rstd[8], s1[8], s2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    mean[j] = stat[c0 + j];
    rstd[j] = stat[C + c0 + j];
    s1[j] = s2[j] = 0.f;
  }
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    float f[8], d[8];
    unpack8(xv[i], f);
    unpack8(dv[i], d);  // (pixels past M: zero dy, nothing added)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      s1[j] += d[j];
      s2[j] += d[j] * (f[j] - mean[j]) * rstd[j];
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[0][pl][cl * 8 + j] = s1[j];
    red[1][pl][cl * 8 + j] = s2[j];
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    float t1 = 0.f, t2 = 0.f;
    for (int q = 0; q < 32; ++q) {
      t1 += red[0][q][threadIdx.x];
      t2 += red[1][q][threadIdx.x];
    }
    const int c = blockIdx.x * 64 + threadIdx.x;
    const float wc = prm[static_cast<int64_t>(c / cg) * ld + c % cg + woff];
    const float mu = stat[c], rs = stat[C + c];
    const float k0 = wc * rs, k1 = t1 / M, k2 = t2 / M;
    cf[0][threadIdx.x] = k0;
    cf[1][threadIdx.x] = -k0 * k2 * rs;
    cf[2][threadIdx.x] = -k0 * k1 + k0 * k2 * rs * mu;
    float* gr = grad + static_cast<int64_t>(c / cg) * gld + c % cg;
    const float* sr = wsrc != nullptr ? wsrc + static_cast<int64_t>(c / cg) * sld + c % cg : gr;
    gr[gwoff] = beta != 0.f ? beta * sr[gwoff] + alpha * t2 : alpha * t2;
    gr[gboff] = beta != 0.f ? beta * sr[gboff] + alpha * t1 : alpha * t1;
  }
  __syncthreads();
  float P[8], Q[8], R[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    P[j] = cf[0][cl * 8 + j];
    Q[j] = cf[1][cl * 8 + j];
    R[j] = cf[2][cl * 8 + j];
  }
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const int p = pl + 32 * i;
    if (p >= M) break;
    float f[8], d[8], o[8];
    unpack8(xv[i], f);
    unpack8(dv[i], d);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = d[j] * P[j] + f[j] * Q[j] + R[j];
    *reinterpret_cast<u4*>(dx + static_cast<size_t>(p) * C + c0) =
        u4{pack2(o[0], o[1]), pack2(o[2], o[3]), pack2(o[4], o[5]), pack2(o[6], o[7])};
  }
}

int apply_grid(int64_t n) {
  int64_t b = (n + 255) / 256;
  if (b > 8192) b = 8192;
  return static_cast<int>(b < 1 ? 1 : b);
}

}  // namespace

// floats of the ``part`` scratch: the partial sums + (few groups) the
// per-group moments / dweight-dbias sums behind them
int64_t bn_scratch_floats(int G, int M, int C) {
  return static_cast<int64_t>(G) * bn_slabs(G, M) * 2 * C + static_cast<int64_t>(G) * 2 * C;
}

int bn_slabs(int G, int M) {
  // >= ~512 partial blocks over the whole batch, >= 64 pixels each
  int s = (512 + G - 1) / G;
  const int cap = M / 64 > 1 ? M / 64 : 1;
  if (s > cap) s = cap;
  return s < 1 ? 1 : s;
}

void launch_bn_fwd(const uint16_t* x, const float* w, const float* b, int G, int M, int C,
                   float eps, float momentum, float* run_mean, float* run_var, float* part,
                   float* stat, float* ab, bool relu, int64_t* nbt, uint16_t* y, hipStream_t stream,
                   const uint16_t* addend, uint8_t* relu_bits, const float* tile_stats) {
  const int S = bn_slabs(G, M);
  const int64_t nchunks = static_cast<int64_t>(G) * M * (C / 8);
  if (tile_stats != nullptr) {
    // the producing GEMM wrote per-tile moments: no partial pass over x
    float* gmv = part + static_cast<size_t>(G) * S * 2 * C;
    COMMEFF_LAUNCH(bn_fwd_finalize_tiles_kernel, dim3((C + 63) / 64, G), dim3(64 * kGL), 0, stream,
                   tile_stats, w, b, C, G * M, M, eps, stat, ab, gmv);
    COMMEFF_LAUNCH(bn_running_kernel, dim3((C + 255) / 256), dim3(256), 0, stream, gmv, C, M, G,
                   momentum, run_mean, run_var, nbt);
    COMMEFF_LAUNCH(bn_apply_kernel<false>, dim3(apply_grid(nchunks)), dim3(256), 0, stream, x, nullptr,
                   nullptr, ab, C, M, static_cast<uint32_t>(nchunks), relu, y,
                   const_cast<uint16_t*>(addend), relu ? relu_bits : nullptr, kNoRun);
    return;
  }
  COMMEFF_LAUNCH(bn_partial_kernel<false>, dim3(G * S), dim3(256), 0, stream, x, nullptr, nullptr,
                     nullptr, C, M, S, part, C);
  if (G >= 2 && G < kGL) {
    // per-group mean / var behind the partial sums (bn_scratch_floats)
    float* gmv = part + static_cast<size_t>(G) * S * 2 * C;
    COMMEFF_LAUNCH(bn_fwd_finalize_group_kernel, dim3((C + 63) / 64, G), dim3(64 * kGL), 0, stream,
                   x, part, w, b, C, M, S, eps, stat, ab, gmv);
    const BnRun run{gmv, run_mean, run_var, nbt, G, momentum};
    COMMEFF_LAUNCH(bn_apply_kernel<false>, dim3(apply_grid(nchunks)), dim3(256), 0, stream, x, nullptr,
                   nullptr, ab, C, M, static_cast<uint32_t>(nchunks), relu, y,
                   const_cast<uint16_t*>(addend), relu ? relu_bits : nullptr, run);
    return;
  } else {
    COMMEFF_LAUNCH(bn_fwd_finalize_kernel, dim3((C + 63) / 64), dim3(64 * kGL), 0, stream, x, part,
                       w, b, C, M, S, G, eps, momentum, stat, ab, run_mean, run_var, nbt);
  }
  COMMEFF_LAUNCH(bn_apply_kernel<false>, dim3(apply_grid(nchunks)), dim3(256), 0, stream, x, nullptr,
                     nullptr, ab, C, M, static_cast<uint32_t>(nchunks), relu, y,
                     const_cast<uint16_t*>(addend), relu ? relu_bits : nullptr, kNoRun);
}

void launch_bn_bwd(const uint16_t* x, const uint16_t* dy, const uint8_t* y_relu, const float* stat,
                   const float* w, int G, int M, int C, float* part, float* coef, float* dw, float* db,
                   float beta, uint16_t* dx, hipStream_t stream, float* gdw, float* gdb,
                   int64_t gstride, uint16_t* dadd) {
  const int S = bn_slabs(G, M);
  COMMEFF_LAUNCH(bn_partial_kernel<true>, dim3(G * S), dim3(256), 0, stream, x, dy, y_relu, stat, C, M,
                     S, part, C);
  if (G >= 2 && G < kGL) {
    float* gsum = part + static_cast<size_t>(G) * S * 2 * C;  // see bn_scratch_floats
    const bool grouped = gdw != nullptr;
    COMMEFF_LAUNCH(bn_bwd_finalize_group_kernel, dim3((C + 63) / 64, G), dim3(64 * kGL), 0, stream,
                       part, stat, w, C, M, S, coef, gdw, gdb, gstride,
                       (!grouped && (dw != nullptr || db != nullptr)) ? gsum : nullptr);
    if (!grouped && (dw != nullptr || db != nullptr))
      COMMEFF_LAUNCH(bn_dwdb_kernel, dim3((C + 255) / 256), dim3(256), 0, stream, gsum, C, G, dw, db,
                         beta);
  } else {
    COMMEFF_LAUNCH(bn_bwd_finalize_kernel, dim3((C + 63) / 64), dim3(64 * kGL), 0, stream, part, stat,
                       w, C, M, S, G, coef, dw, db, beta, gdw, gdb, gstride);
  }
  const int64_t nchunks = static_cast<int64_t>(G) * M * (C / 8);
  COMMEFF_LAUNCH(bn_apply_kernel<true>, dim3(apply_grid(nchunks)), dim3(256), 0, stream, x, dy, y_relu,
                     coef, C, M, static_cast<uint32_t>(nchunks), false, dx, dadd, nullptr, kNoRun);
}

// channel block of the partial kernels: the largest power-of-two multiple of
// 8 dividing C, at most 2048 (C / 8 lanes of 16 bytes x 256 / (C / 8) pixels),
// halved (down to 64) while the S x C / CB grid has fewer than 1024 blocks --
// the small maps of the deep layers (S = 1..5 slabs) otherwise ran 25..125
// blocks walking every pixel serially (17.8 us per backward partial at 4x4)
static int cs_channel_block(int C, int S) {
  int cb = 8;
  while (cb * 2 <= 2048 && C % (cb * 2) == 0) cb *= 2;
  while (cb > 64 && static_cast<int64_t>(S) * (C / cb) < 1024) cb /= 2;
  return cb;
}

int64_t bn_cs_scratch_floats(int M, int C) { return static_cast<int64_t>(bn_slabs(1, M)) * 2 * C; }

void launch_bn_cs_fwd(const uint16_t* x, const float* prm, int64_t ld, int64_t woff, int64_t boff, int cg,
                      int M, int C, float eps, float momentum, float* run_mean, float* run_var,
                      int64_t* nbt, float* part, float* stat, float* ab, uint16_t* y, uint8_t* relu_bits,
                      const uint16_t* post_add, hipStream_t stream) {
  if (M <= 320 && M >= 1 && C % 64 == 0) {  // one fused kernel (small maps)
#define CS_SMALL_FWD(NP)                                                                                     \
  {                                                                                                          \
    if (post_add != nullptr)                                                                                 \
      COMMEFF_LAUNCH((bn_cs_small_fwd_kernel<NP, true>), dim3(C / 64), dim3(256), 0, stream, x, prm, ld, woff, \
                     boff, cg, C, M, eps, momentum, stat, run_mean, run_var, nbt, y, relu_bits, post_add);     \
    else                                                                                                     \
      COMMEFF_LAUNCH((bn_cs_small_fwd_kernel<NP, false>), dim3(C / 64), dim3(256), 0, stream, x, prm, ld,     \
                     woff, boff, cg, C, M, eps, momentum, stat, run_mean, run_var, nbt, y, relu_bits, nullptr); \
  }
    if (M <= 128) CS_SMALL_FWD(4) else CS_SMALL_FWD(10)
#undef CS_SMALL_FWD
    return;
  }
  const int S = bn_slabs(1, M), CB = cs_channel_block(C, S);
  COMMEFF_LAUNCH(bn_partial_kernel<false>, dim3(S, C / CB), dim3(256), 0, stream, x, nullptr, nullptr,
                 nullptr, C, M, S, part, CB);
  COMMEFF_LAUNCH(bn_cs_fwd_finalize_kernel, dim3((C + 63) / 64), dim3(64 * kGL), 0, stream, x, part, prm,
                 ld, woff, boff, cg, C, M, S, eps, momentum, stat, ab, run_mean, run_var, nbt);
  const int64_t nchunks = static_cast<int64_t>(M) * (C / 8);
  if (post_add != nullptr)
    COMMEFF_LAUNCH((bn_apply_kernel<false, true>), dim3(apply_grid(nchunks)), dim3(256), 0, stream, x, nullptr,
                   nullptr, ab, C, M, static_cast<uint32_t>(nchunks), true, y, const_cast<uint16_t*>(post_add),
                   relu_bits, kNoRun);
  else
    COMMEFF_LAUNCH(bn_apply_kernel<false>, dim3(apply_grid(nchunks)), dim3(256), 0, stream, x, nullptr,
                   nullptr, ab, C, M, static_cast<uint32_t>(nchunks), true, y, nullptr, relu_bits, kNoRun);
}

void launch_bn_cs_bwd(const uint16_t* x, const uint16_t* dy, const uint8_t* y_relu, const float* stat,
                      const float* prm, int64_t ld, int64_t woff, int cg, int M, int C, float* part,
                      float* coef, float* grad, int64_t gld, int64_t gwoff, int64_t gboff, uint16_t* dx,
                      hipStream_t stream, float beta, float alpha, const float* wsrc, int64_t sld) {
  if (M <= 320 && M >= 1 && C % 64 == 0) {  // one fused kernel (small maps)
    if (M <= 128)
      COMMEFF_LAUNCH(bn_cs_small_bwd_kernel<4>, dim3(C / 64), dim3(256), 0, stream, x, dy, y_relu, stat, prm, ld,
                     woff, cg, C, M, grad, gld, gwoff, gboff, beta, alpha, wsrc, sld, dx);
    else
      COMMEFF_LAUNCH(bn_cs_small_bwd_kernel<10>, dim3(C / 64), dim3(256), 0, stream, x, dy, y_relu, stat, prm,
                     ld, woff, cg, C, M, grad, gld, gwoff, gboff, beta, alpha, wsrc, sld, dx);
    return;
  }
  const int S = bn_slabs(1, M), CB = cs_channel_block(C, S);
  COMMEFF_LAUNCH(bn_partial_kernel<true>, dim3(S, C / CB), dim3(256), 0, stream, x, dy, y_relu, stat, C,
                 M, S, part, CB);
  COMMEFF_LAUNCH(bn_cs_bwd_finalize_kernel, dim3((C + 63) / 64), dim3(64 * kGL), 0, stream, part, stat, prm,
                 ld, woff, cg, C, M, S, coef, grad, gld, gwoff, gboff, beta, alpha, wsrc, sld);
  const int64_t nchunks = static_cast<int64_t>(M) * (C / 8);
  COMMEFF_LAUNCH(bn_apply_kernel<true>, dim3(apply_grid(nchunks)), dim3(256), 0, stream, x, dy, y_relu,
                 coef, C, M, static_cast<uint32_t>(nchunks), false, dx, nullptr, nullptr, kNoRun);
}

}  // namespace commeff
