// GPT-2 block junction kernels (pre-LN transformer, bf16 activations):
//
//   resid_ln_fwd   h = x + drop(p + bias)   (or h = drop(x) without a branch)
//                  y = LayerNorm(h) * gamma + beta,  mean / rstd per row saved
//   resid_ln_bwd   dh = LN'(gy) + gh,  dp = drop'(dh),
//                  per-block column partials of gy*xhat, gy, dp
//                  (dgamma, dbeta, dbias of the branch's projection)
//   bias_gelu_fwd  f = gelu_tanh(u + b)
//   bias_act_bwd   du = gf * gelu_tanh'(u + b) (or du = gf), per-block column
//                  partials of du (the bias gradient of the producing GEMM)
//   colsum_final   deterministic fixed-order sum of the block partials
//
// These replace, per GPT-2 sublayer, HF's separate residual add, dropout,
// LayerNorm, GELU, dropout-backward, LayerNorm-backward (3 kernels) and
// bias-gradient reduction kernels (reference model: HF GPT2DoubleHeadsModel,
// /root/reference/CommEfficient/gpt2_train.py:4-6,262-273).  The GEMMs stay on
// hipBLASLt and attention on the fused SDPA kernels (ops/transformer.py).
//
// Layout: one row (token) of H = 256*V features is owned by a half-wave (32
// lanes, V 16-byte vectors of 8 bf16 per lane, lane-interleaved so every
// vector step of the half-wave reads 512 contiguous bytes); 8 rows per
// 256-thread block.  Row reductions are 5 xor-shuffles inside the half-wave.
// Dropout draws one 32-bit hash of (seed, element index) per element, so the
// backward regenerates the mask instead of storing it.
#include <hip/hip_runtime.h>
#include <cstdint>
#include "kernels.h"

namespace commeff {
namespace {

struct alignas(16) V8 {
  uint32_t w[4];
};

__device__ __forceinline__ void unpack8(const V8& v, float f[8]) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    f[2 * k] = __uint_as_float(v.w[k] << 16);
    f[2 * k + 1] = __uint_as_float(v.w[k] & 0xffff0000u);
  }
}

__device__ __forceinline__ uint32_t bf16_bits(float f) {
  const __bf16 b = static_cast<__bf16>(f);
  return static_cast<uint32_t>(__builtin_bit_cast(uint16_t, b));
}

__device__ __forceinline__ V8 pack8(const float f[8]) {
  V8 v;
#pragma unroll
  for (int k = 0; k < 4; ++k) v.w[k] = bf16_bits(f[2 * k]) | (bf16_bits(f[2 * k + 1]) << 16);
  return v;
}

// round to bf16 and back (the value a bf16 tensor would hold)
__device__ __forceinline__ float rbf(float f) { return __uint_as_float(bf16_bits(f) << 16); }

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

// keep element `idx` of a dropout site with drop threshold `thresh` (= p * 2^32)
__device__ __forceinline__ bool keep_elem(uint64_t idx, uint32_t seed, uint32_t thresh) {
  const uint32_t hi = mix32(static_cast<uint32_t>(idx >> 32) + seed);
  return mix32(static_cast<uint32_t>(idx) ^ hi) >= thresh;
}

__device__ __forceinline__ float half_wave_sum(float v) {
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 32);
  return v;
}

constexpr float kGeluK = 0.7978845608028654f;  // sqrt(2/pi)
constexpr float kGeluC = 0.044715f;

__device__ __forceinline__ float gelu_tanh(float x) {
  const float t = tanhf(kGeluK * (x + kGeluC * x * x * x));
  return 0.5f * x * (1.f + t);
}

__device__ __forceinline__ float gelu_tanh_grad(float x) {
  const float x2 = x * x;
  const float t = tanhf(kGeluK * (x + kGeluC * x2 * x));
  return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * kGeluK * (1.f + 3.f * kGeluC * x2);
}

// ------------------------------------------------------------ resid + LN fwd
template <int V>
__global__ void __launch_bounds__(256)
resid_ln_fwd_kernel(const V8* __restrict__ x, const V8* __restrict__ p, const V8* __restrict__ bias,
                    const V8* __restrict__ gamma, const V8* __restrict__ beta, V8* __restrict__ h_out,
                    V8* __restrict__ y_out, float* __restrict__ mean_out, float* __restrict__ rstd_out,
                    int64_t M, uint32_t thresh, float scale, uint32_t seed, float eps) {
  constexpr int HV = V * 32;  // 16-byte vectors per row
  constexpr float invH = 1.f / (HV * 8);
  const int lane = threadIdx.x & 31;
  const int64_t row = static_cast<int64_t>(blockIdx.x) * 8 + (threadIdx.x >> 5);
  if (row >= M) return;  // the whole half-wave leaves together
  const int64_t rbase = row * HV;
  float v[V][8];
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < V; ++q) {
    const int cv = lane + q * 32;
    unpack8(x[rbase + cv], v[q]);
    const uint64_t ebase = static_cast<uint64_t>(rbase + cv) * 8;
    if (p != nullptr) {
      float pv[8], bv[8];
      unpack8(p[rbase + cv], pv);
      if (bias != nullptr) {
        unpack8(bias[cv], bv);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) bv[e] = 0.f;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float t = rbf(pv[e] + bv[e]);  // the projection output (bf16 GEMM + bias)
        if (thresh != 0u) t = keep_elem(ebase + e, seed, thresh) ? rbf(t * scale) : 0.f;
        v[q][e] = rbf(v[q][e] + t);
      }
    } else if (thresh != 0u) {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        v[q][e] = keep_elem(ebase + e, seed, thresh) ? rbf(v[q][e] * scale) : 0.f;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) s += v[q][e];
  }
  const float mu = half_wave_sum(s) * invH;
  float ss = 0.f;
#pragma unroll
  for (int q = 0; q < V; ++q)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float d = v[q][e] - mu;
      ss += d * d;
    }
  const float rs = rsqrtf(half_wave_sum(ss) * invH + eps);
#pragma unroll
  for (int q = 0; q < V; ++q) {
    const int cv = lane + q * 32;
    if (h_out != nullptr) h_out[rbase + cv] = pack8(v[q]);
    float g[8], b[8], y[8];
    unpack8(gamma[cv], g);
    unpack8(beta[cv], b);
#pragma unroll
    for (int e = 0; e < 8; ++e) y[e] = (v[q][e] - mu) * rs * g[e] + b[e];
    y_out[rbase + cv] = pack8(y);
  }
  if (lane == 0) {
    mean_out[row] = mu;
    rstd_out[row] = rs;
  }
}

// ------------------------------------------------------------ resid + LN bwd
// part: [gridDim.x][3][H] fp32 column partials (gy*xhat, gy, dp)
template <int V>
__global__ void __launch_bounds__(256)
resid_ln_bwd_kernel(const V8* __restrict__ gy, const V8* __restrict__ gh, const V8* __restrict__ h,
                    const float* __restrict__ mean, const float* __restrict__ rstd,
                    const V8* __restrict__ gamma, V8* __restrict__ dh_out, V8* __restrict__ dp_out,
                    float* __restrict__ part, int64_t M, uint32_t thresh, float scale, uint32_t seed) {
  constexpr int HV = V * 32;
  constexpr int H = HV * 8;
  constexpr float invH = 1.f / H;
  __shared__ float red[8][H];
  const int lane = threadIdx.x & 31;
  const int sub = threadIdx.x >> 5;
  float g[V][8];
#pragma unroll
  for (int q = 0; q < V; ++q) unpack8(gamma[lane + q * 32], g[q]);
  float ag[V][8], ab[V][8], ap[V][8];
#pragma unroll
  for (int q = 0; q < V; ++q)
#pragma unroll
    for (int e = 0; e < 8; ++e) ag[q][e] = ab[q][e] = ap[q][e] = 0.f;

  for (int64_t row = static_cast<int64_t>(blockIdx.x) * 8 + sub; row < M;
       row += static_cast<int64_t>(gridDim.x) * 8) {
    const int64_t rbase = row * HV;
    const float mu = mean[row], rs = rstd[row];
    float xh[V][8], dy[V][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int q = 0; q < V; ++q) {
      const int cv = lane + q * 32;
      float hv[8];
      unpack8(h[rbase + cv], hv);
      unpack8(gy[rbase + cv], dy[q]);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        xh[q][e] = (hv[e] - mu) * rs;
        const float dx = dy[q][e] * g[q][e];
        s1 += dx;
        s2 += dx * xh[q][e];
        ag[q][e] += dy[q][e] * xh[q][e];
        ab[q][e] += dy[q][e];
      }
    }
    s1 = half_wave_sum(s1) * invH;
    s2 = half_wave_sum(s2) * invH;
#pragma unroll
    for (int q = 0; q < V; ++q) {
      const int cv = lane + q * 32;
      float r[8];
      if (gh != nullptr) {
        unpack8(gh[rbase + cv], r);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) r[e] = 0.f;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) r[e] = rbf(rs * (dy[q][e] * g[q][e] - s1 - xh[q][e] * s2) + r[e]);
      dh_out[rbase + cv] = pack8(r);
      if (dp_out != nullptr) {
        const uint64_t ebase = static_cast<uint64_t>(rbase + cv) * 8;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          if (thresh != 0u) r[e] = keep_elem(ebase + e, seed, thresh) ? rbf(r[e] * scale) : 0.f;
          ap[q][e] += r[e];
        }
        dp_out[rbase + cv] = pack8(r);
      }
    }
  }
  // fixed-order block reduction of the 8 half-wave partials per column
  float* dst = part + static_cast<int64_t>(blockIdx.x) * 3 * H;
#pragma unroll
  for (int which = 0; which < 3; ++which) {
#pragma unroll
    for (int q = 0; q < V; ++q)
#pragma unroll
      for (int e = 0; e < 8; ++e)
        red[sub][(lane + q * 32) * 8 + e] = which == 0 ? ag[q][e] : (which == 1 ? ab[q][e] : ap[q][e]);
    __syncthreads();
    for (int c = threadIdx.x; c < H; c += 256) {
      float t = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) t += red[k][c];
      dst[which * H + c] = t;
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------ bias + GELU
__global__ void __launch_bounds__(256)
bias_gelu_fwd_kernel(const V8* __restrict__ u, const V8* __restrict__ b, V8* __restrict__ f,
                     int64_t nvec, int NV) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= nvec) return;
  float uv[8], bv[8], o[8];
  unpack8(u[i], uv);
  unpack8(b[i % NV], bv);
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = gelu_tanh(rbf(uv[e] + bv[e]));
  f[i] = pack8(o);
}

template <bool GELU>
__device__ __forceinline__ void bias_act_row(const V8& gv, const V8& uv, const float bv[8], V8* du,
                                             int64_t i, float acc[8]) {
  float g[8];
  unpack8(gv, g);
  if (GELU) {
    float x[8];
    unpack8(uv, x);
#pragma unroll
    for (int e = 0; e < 8; ++e) g[e] = rbf(g[e] * gelu_tanh_grad(rbf(x[e] + bv[e])));
    du[i] = pack8(g);
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] += g[e];
}

// one thread per 8-column vector (blockDim = NV), rows strided by the grid,
// four rows per step (their loads issued before any is used);
// part: [gridDim.x][N] fp32 column partials of du
template <bool GELU>
__global__ void __launch_bounds__(1024)
bias_act_bwd_kernel(const V8* __restrict__ gf, const V8* __restrict__ u, const V8* __restrict__ b,
                    V8* __restrict__ du, float* __restrict__ part, int64_t M, int NV) {
  const int cv = threadIdx.x;
  const int64_t G = gridDim.x;
  float acc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = 0.f;
  float bv[8];
  if (GELU) {
    unpack8(b[cv], bv);
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) bv[e] = 0.f;
  }
  int64_t row = blockIdx.x;
  constexpr int kR = 4;  // rows per step, every load issued before any is used
  for (; row + (kR - 1) * G < M; row += kR * G) {
    V8 gv[kR], uv[kR];
#pragma unroll
    for (int k = 0; k < kR; ++k) {
      const int64_t i = (row + k * G) * NV + cv;
      gv[k] = gf[i];
      uv[k] = GELU ? u[i] : gv[k];
    }
#pragma unroll
    for (int k = 0; k < kR; ++k) bias_act_row<GELU>(gv[k], uv[k], bv, du, (row + k * G) * NV + cv, acc);
  }
  for (; row < M; row += G) {
    const int64_t i0 = row * NV + cv;
    const V8 g0 = gf[i0];
    bias_act_row<GELU>(g0, GELU ? u[i0] : g0, bv, du, i0, acc);
  }
  float* dst = part + static_cast<int64_t>(blockIdx.x) * NV * 8 + cv * 8;
  *reinterpret_cast<float4*>(dst) = make_float4(acc[0], acc[1], acc[2], acc[3]);
  *reinterpret_cast<float4*>(dst + 4) = make_float4(acc[4], acc[5], acc[6], acc[7]);
}

// out_q[c] = sum_b part[b*stride + q*N + c]: 16 columns per 1024-thread
// block (Q*N/16 blocks: ~150-200 for GPT-2, the kernel is latency-bound);
// lane l of wave w reads column l % 16 of rows w*per + l/16 + 4i (every load
// of the lane in flight at once), sums them in row order, then the 4 row
// phases (xor-shuffles 16, 32) and the 16 waves (LDS, wave order) combine in a
// fixed order -- the result is deterministic
__global__ void __launch_bounds__(1024)
colsum_final_kernel(const float* __restrict__ part, int G, int Q, int64_t N, int64_t stride,
                    ColsumOut out) {
  __shared__ float red[16][16];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int cl = lane & 15, ph = lane >> 4;
  const int64_t col = static_cast<int64_t>(blockIdx.x) * 16 + cl;  // over Q*N
  const bool ok = col < Q * N;
  const int per = (G + 15) / 16;
  const int b0 = w * per;
  const int b1 = b0 + per < G ? b0 + per : G;
  float acc = 0.f;
  if (ok) {
    const float* src = part + col;
    constexpr int kU = 16;
    for (int b = b0 + ph; b < b1; b += 4 * kU) {
      float t[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int bb = b + 4 * u;
        t[u] = bb < b1 ? src[static_cast<int64_t>(bb) * stride] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < kU; ++u) acc += t[u];
    }
  }
  acc += __shfl_xor(acc, 16, 64);
  acc += __shfl_xor(acc, 32, 64);
  if (ph == 0) red[w][cl] = acc;
  __syncthreads();
  if (w == 0 && ph == 0 && ok) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) t += red[k][cl];
    const int q = static_cast<int>(col / N);
    const int64_t c = col - q * N;
    void* o = q == 0 ? out.p[0] : (q == 1 ? out.p[1] : out.p[2]);
    const int mode = q == 0 ? out.mode[0] : (q == 1 ? out.mode[1] : out.mode[2]);
    if (o != nullptr) {
      if (mode == 0)
        static_cast<uint16_t*>(o)[c] = static_cast<uint16_t>(bf16_bits(t));
      else if (mode == 1)
        static_cast<float*>(o)[c] = t;
      else
        static_cast<float*>(o)[c] += t;
    }
  }
}

uint32_t drop_threshold(float p) {
  if (p <= 0.f) return 0u;
  const double t = static_cast<double>(p) * 4294967296.0;
  return t >= 4294967295.0 ? 0xffffffffu : static_cast<uint32_t>(t);
}

// LN backward blocks (= column-partial rows for colsum_final); 1536 blocks
// measured slower than 512 for a GPT-2 round (658 vs 589 us / 25 calls)
int ln_grid(int64_t M) {
  const int64_t b = (M + 7) / 8;
  return static_cast<int>(b < 512 ? (b > 0 ? b : 1) : 512);
}

}  // namespace

bool resid_ln_supported(int64_t H) { return H % 256 == 0 && H / 256 >= 1 && H / 256 <= 6; }

void launch_resid_ln_fwd(const void* x, const void* p, const void* bias, const void* gamma,
                         const void* beta, void* h_out, void* y_out, float* mean, float* rstd,
                         int64_t M, int64_t H, float p_drop, uint32_t seed, float eps,
                         hipStream_t stream) {
  if (M == 0) return;
  const uint32_t th = drop_threshold(p_drop);
  const float scale = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  const dim3 grid(static_cast<uint32_t>((M + 7) / 8));
#define RLN_FWD(VV)                                                                              \
  COMMEFF_LAUNCH(resid_ln_fwd_kernel<VV>, grid, dim3(256), 0, stream,                        \
                     static_cast<const V8*>(x), static_cast<const V8*>(p),                       \
                     static_cast<const V8*>(bias), static_cast<const V8*>(gamma),                \
                     static_cast<const V8*>(beta), static_cast<V8*>(h_out),                      \
                     static_cast<V8*>(y_out), mean, rstd, M, th, scale, seed, eps)
  switch (H / 256) {
    case 1: RLN_FWD(1); break;
    case 2: RLN_FWD(2); break;
    case 3: RLN_FWD(3); break;
    case 4: RLN_FWD(4); break;
    case 5: RLN_FWD(5); break;
    case 6: RLN_FWD(6); break;
    default: break;
  }
#undef RLN_FWD
}

int resid_ln_bwd_blocks(int64_t M) { return ln_grid(M); }

void launch_resid_ln_bwd(const void* gy, const void* gh, const void* h, const float* mean,
                         const float* rstd, const void* gamma, void* dh_out, void* dp_out,
                         float* part, int64_t M, int64_t H, float p_drop, uint32_t seed,
                         hipStream_t stream) {
  const uint32_t th = drop_threshold(p_drop);
  const float scale = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  const dim3 grid(static_cast<uint32_t>(ln_grid(M)));
#define RLN_BWD(VV)                                                                              \
  COMMEFF_LAUNCH(resid_ln_bwd_kernel<VV>, grid, dim3(256), 0, stream,                        \
                     static_cast<const V8*>(gy), static_cast<const V8*>(gh),                     \
                     static_cast<const V8*>(h), mean, rstd, static_cast<const V8*>(gamma),       \
                     static_cast<V8*>(dh_out), static_cast<V8*>(dp_out), part, M, th, scale,     \
                     seed)
  switch (H / 256) {
    case 1: RLN_BWD(1); break;
    case 2: RLN_BWD(2); break;
    case 3: RLN_BWD(3); break;
    case 4: RLN_BWD(4); break;
    case 5: RLN_BWD(5); break;
    case 6: RLN_BWD(6); break;
    default: break;
  }
#undef RLN_BWD
}

void launch_bias_gelu_fwd(const void* u, const void* b, void* f, int64_t M, int64_t N,
                          hipStream_t stream) {
  const int64_t nvec = M * N / 8;
  if (nvec == 0) return;
  COMMEFF_LAUNCH(bias_gelu_fwd_kernel, dim3(static_cast<uint32_t>((nvec + 255) / 256)),
                     dim3(256), 0, stream, static_cast<const V8*>(u), static_cast<const V8*>(b),
                     static_cast<V8*>(f), nvec, static_cast<int>(N / 8));
}

int bias_act_bwd_blocks(int64_t M) {
  return static_cast<int>(M < 512 ? (M > 0 ? M : 1) : 512);
}

void launch_bias_act_bwd(const void* gf, const void* u, const void* b, void* du, float* part,
                         int64_t M, int64_t N, bool gelu, hipStream_t stream) {
  const dim3 grid(static_cast<uint32_t>(bias_act_bwd_blocks(M)));
  const int NV = static_cast<int>(N / 8);
  if (gelu)
    COMMEFF_LAUNCH(bias_act_bwd_kernel<true>, grid, dim3(NV), 0, stream,
                       static_cast<const V8*>(gf), static_cast<const V8*>(u),
                       static_cast<const V8*>(b), static_cast<V8*>(du), part, M, NV);
  else
    COMMEFF_LAUNCH(bias_act_bwd_kernel<false>, grid, dim3(NV), 0, stream,
                       static_cast<const V8*>(gf), nullptr, nullptr, nullptr, part, M, NV);
}

void launch_colsum_final(const float* part, int G, int Q, int64_t N, int64_t stride,
                         const ColsumOut& out, hipStream_t stream) {
  const int64_t cols = Q * N;
  COMMEFF_LAUNCH(colsum_final_kernel, dim3(static_cast<uint32_t>((cols + 15) / 16)),
                     dim3(1024), 0, stream, part, G, Q, N, stride, out);
}

}  // namespace commeff

// ---------------------------------------------------- token rows <-> heads
// GPT-2 attention layout changes with padding removal folded in.  Token rows
// are the real (unpadded) tokens, [Mr, P*H]; the attention runs on padded
// per-head tensors [N, nh, L, hd].  inv[n*L + t] = token row of position
// (n, t) or -1 for a pad (nullptr: identity, no padding); tok[i] = n*L + t of
// token row i (nullptr: identity).
namespace commeff {
namespace {

// one block per padded position: out[pos, :] = src[inv[pos], :] or 0 at a pad
// (the padded row layout [N, L, K] is the attention's [N, L, heads, hd]
// memory layout: q/k/v/dO are its head views without another copy)
__global__ void __launch_bounds__(256)
pad_rows_kernel(const V8* __restrict__ src, int64_t src_ld8, int K8, const int32_t* __restrict__ inv,
                V8* __restrict__ out) {
  const int64_t pos = blockIdx.x;
  const int64_t r = inv != nullptr ? inv[pos] : pos;
  for (int v = threadIdx.x; v < K8; v += 256) {
    V8 val;
    if (r >= 0) {
      val = src[r * src_ld8 + v];
    } else {
      val.w[0] = val.w[1] = val.w[2] = val.w[3] = 0u;
    }
    out[pos * K8 + v] = val;
  }
}

// one block per token row i: out[i, p*H + h*hd + d] = src_p[n, h, t, d]
__global__ void __launch_bounds__(256)
heads_to_rows_kernel(HeadSrcs src, int P, int H8, int hd8, int64_t L,
                     const int32_t* __restrict__ tok, V8* __restrict__ out) {
  const int64_t i = blockIdx.x;
  const int64_t pos = tok != nullptr ? tok[i] : i;
  const int64_t n = pos / L, t = pos - n * L;
  for (int v = threadIdx.x; v < P * H8; v += 256) {
    const int p = v / H8;
    const int c = v - p * H8;
    const int h = c / hd8, d = c - h * hd8;
    const int64_t* st = p == 0 ? src.stride[0] : (p == 1 ? src.stride[1] : src.stride[2]);
    const V8* s = static_cast<const V8*>(p == 0 ? src.p[0] : (p == 1 ? src.p[1] : src.p[2]));
    out[i * P * H8 + v] = s[(n * st[0] + h * st[1] + t * st[2]) / 8 + d];
  }
}

}  // namespace

void launch_pad_rows(const void* src, int64_t src_ld, int64_t K, const int32_t* inv, int64_t rows,
                     void* out, hipStream_t stream) {
  if (rows == 0) return;
  COMMEFF_LAUNCH(pad_rows_kernel, dim3(static_cast<uint32_t>(rows)), dim3(256), 0, stream,
                     static_cast<const V8*>(src), src_ld / 8, static_cast<int>(K / 8), inv,
                     static_cast<V8*>(out));
}

void launch_heads_to_rows(const HeadSrcs& src, int P, int64_t H, int64_t hd, int64_t L,
                          const int32_t* tok, int64_t Mr, void* out, hipStream_t stream) {
  if (Mr == 0) return;
  COMMEFF_LAUNCH(heads_to_rows_kernel, dim3(static_cast<uint32_t>(Mr)), dim3(256), 0, stream,
                     src, P, static_cast<int>(H / 8), static_cast<int>(hd / 8), L, tok,
                     static_cast<V8*>(out));
}

}  // namespace commeff
