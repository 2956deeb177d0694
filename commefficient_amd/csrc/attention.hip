// Fused causal self-attention for short sequences (GPT-2 PersonaChat rows:
// L <= 128 tokens, head dim 64) on the bf16 MFMA (v_mfma_f32_32x32x16_bf16),
// one 4-wave workgroup per (sequence, head), everything in LDS.
//
// Reference model: HF GPT2Attention (SDPA, is_causal, attention dropout) of
// GPT2DoubleHeadsModel, /root/reference/CommEfficient/gpt2_train.py:4-6.
// At these lengths the generic flash kernels spend ~215 us per layer (fwd +
// bwd, 64 sequences x 12 heads) on tile overheads; here a sequence's whole
// Q, K, V (3 x 16 KB) and its score matrix sit in LDS, so a layer moves
// ~130 MB and does ~6 GFLOP.
//
// Token rows stay UNPADDED: sequence n owns rows [start[n], start[n] + len[n])
// of qkv [M, 3H] (q | k | v, head h at columns h*64) and of o / do [M, H];
// dqkv [M, 3H] comes back in the same layout (no padding, no head
// transposes, no q/k/v concatenation).
//
// Forward:  S = Q K^T * scale (causal tiles only), row softmax (2 threads per
//           row, LSE saved), P_drop = dropout(P) (32-bit counter hash of
//           (seed, (seq*heads + h)*128*128 + i*128 + j), the backward
//           regenerates it), O = P_drop V.
// Backward: D_i = dO_i . O_i; S, dP_drop = dO V^T recomputed in registers;
//           P = exp(S - LSE), dS = P (dP - D) * scale (dP = dropout'(dP_drop));
//           dV = P_drop^T dO, dK = dS^T Q, dQ = dS K.  Operands that an MFMA
//           needs K-major are written to LDS transposed (scalar 2-byte stores
//           straight from the accumulator layout).
// MFMA operand convention (as conv.hip): C[m][n] = sum_k A[m][k] * Bt[n][k],
// lane l holds A row (l & 31), k = 8 (l >> 5) .. +8 of a 16-wide k step, the
// same for Bt; accumulator element e of lane l is C[(e & 3) + 8 (e >> 2) +
// 4 (l >> 5)][l & 31].
#include <hip/hip_runtime.h>
#include <cstdint>
#include "kernels.h"
#include "conv_common.h"

namespace commeff {
namespace {

constexpr int HD = 64;       // head dim
constexpr int LM = 128;      // max sequence length
constexpr int RS = HD + 8;   // row stride (elements) of [LM][HD] bf16 tiles
constexpr int TS = LM + 8;   // row stride of [HD][LM] and [LM][LM] bf16 tiles
constexpr int SS = LM + 4;   // row stride of the fp32 score tile
constexpr int OS = HD + 4;   // row stride of the fp32 output staging tile

__device__ __forceinline__ uint16_t bfbits(float f) {
  const __bf16 b = static_cast<__bf16>(f);
  return __builtin_bit_cast(uint16_t, b);
}
__device__ __forceinline__ float bfval(uint16_t h) { return __uint_as_float(static_cast<uint32_t>(h) << 16); }

__device__ __forceinline__ uint32_t amix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ bool akeep(uint64_t idx, uint32_t seed, uint32_t thresh) {
  const uint32_t hi = amix32(static_cast<uint32_t>(idx >> 32) + seed);
  return amix32(static_cast<uint32_t>(idx) ^ hi) >= thresh;
}

__device__ __forceinline__ int crow(int e, int hi) { return (e & 3) + 8 * (e >> 2) + 4 * hi; }

__device__ __forceinline__ f32x16_t zero16() {
  f32x16_t z;
#pragma unroll
  for (int e = 0; e < 16; ++e) z[e] = 0.f;
  return z;
}

// ------------------------------------------------------------------ forward
// LDS: Q, K [LM][RS], V^T [HD][TS] and the fp32 score tile (122 KB).  (A
// variant with the softmax in registers -- 54 KB, 2 workgroups per CU, row
// reductions by 10 xor-shuffles per row -- measured 460 vs 366 us/round.)
__global__ void __launch_bounds__(256) attn_fwd_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint16_t* sQ = reinterpret_cast<uint16_t*>(smem);          // [LM][RS]
  uint16_t* sK = sQ + LM * RS;                                 // [LM][RS]
  uint16_t* sVt = sK + LM * RS;                                // [HD][TS]
  float* sS = reinterpret_cast<float*>(sVt + HD * TS);         // [LM][SS]
  uint16_t* sP = sQ;                                           // [LM][TS] over Q, K
  float* sO = sS;                                              // [LM][OS] over S
  const int bh = blockIdx.x;
  const int n = bh / a.nh, h = bh - n * a.nh;
  const int L = a.len[n];
  if (L <= 0) return;
  const int64_t r0 = a.start[n];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, hi = lane >> 5, lr = lane & 31;
  const int H = a.nh * HD;

  {  // all of this thread's 16-byte pieces in flight before any LDS store
    v4u q[4], k[4], v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int c = tid + 256 * u, i = c >> 3, ch = c & 7;
      q[u] = k[u] = v[u] = v4u{0u, 0u, 0u, 0u};
      if (i < L) {
        const uint16_t* row = a.qkv + (r0 + i) * (3 * H) + h * HD + ch * 8;
        q[u] = *reinterpret_cast<const v4u*>(row);
        k[u] = *reinterpret_cast<const v4u*>(row + H);
        v[u] = *reinterpret_cast<const v4u*>(row + 2 * H);
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int c = tid + 256 * u, i = c >> 3, ch = c & 7;
      *reinterpret_cast<v4u*>(sQ + i * RS + ch * 8) = q[u];
      *reinterpret_cast<v4u*>(sK + i * RS + ch * 8) = k[u];
#pragma unroll
      for (int e = 0; e < 8; ++e)
        sVt[(ch * 8 + e) * TS + i] = static_cast<uint16_t>((v[u][e >> 1] >> (16 * (e & 1))) & 0xffffu);
    }
  }
  __syncthreads();

  if (32 * w < L) {
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) {
      if (ct > w) break;  // causal: these key tiles are all masked for this strip
      f32x16_t acc = zero16();
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const bf16x8_t af = *reinterpret_cast<const bf16x8_t*>(sQ + (32 * w + lr) * RS + 16 * ks + 8 * hi);
        const bf16x8_t bf = *reinterpret_cast<const bf16x8_t*>(sK + (32 * ct + lr) * RS + 16 * ks + 8 * hi);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bf, acc, 0, 0, 0);
      }
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = 32 * w + crow(e, hi), col = 32 * ct + lr;
        sS[row * SS + col] = (col <= row && col < L) ? acc[e] * a.scale : -__builtin_huge_valf();
      }
    }
  }
  __syncthreads();

  // row softmax, 2 threads per row; P_drop -> sP (bf16, zeros past the diagonal)
  {
    const int i = tid >> 1, half = tid & 1;
    const int jmax = i + 1 < L ? i + 1 : L;  // valid keys [0, jmax)
    float p[64];
    float m = -__builtin_huge_valf();
#pragma unroll
    for (int t = 0; t < 64; ++t) {
      const int j = half * 64 + t;
      p[t] = j < jmax ? sS[i * SS + j] : -__builtin_huge_valf();
      m = fmaxf(m, p[t]);
    }
    m = fmaxf(m, __shfl_xor(m, 1, 64));
    float sum = 0.f;
#pragma unroll
    for (int t = 0; t < 64; ++t) {
      const int j = half * 64 + t;
      p[t] = j < jmax ? __expf(p[t] - m) : 0.f;
      sum += p[t];
    }
    sum += __shfl_xor(sum, 1, 64);
    if (i < L && half == 0) a.lse[static_cast<int64_t>(bh) * LM + i] = m + __logf(sum);
    const float inv = 1.f / sum;
    const uint64_t ib = (static_cast<uint64_t>(bh) * LM + i) * LM + half * 64;
#pragma unroll
    for (int t = 0; t < 64; t += 2) {
      float v0 = p[t] * inv, v1 = p[t + 1] * inv;
      if (a.thresh != 0u) {
        v0 = akeep(ib + t, a.seed, a.thresh) ? v0 * a.dscale : 0.f;
        v1 = akeep(ib + t + 1, a.seed, a.thresh) ? v1 * a.dscale : 0.f;
      }
      *reinterpret_cast<uint32_t*>(sP + i * TS + half * 64 + t) =
          static_cast<uint32_t>(bfbits(v0)) | (static_cast<uint32_t>(bfbits(v1)) << 16);
    }
  }
  __syncthreads();

  if (32 * w < L) {
    f32x16_t acc[2] = {zero16(), zero16()};
    for (int ks = 0; ks < 2 * w + 2; ++ks) {
      const bf16x8_t af = *reinterpret_cast<const bf16x8_t*>(sP + (32 * w + lr) * TS + 16 * ks + 8 * hi);
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {
        const bf16x8_t bf = *reinterpret_cast<const bf16x8_t*>(sVt + (32 * ct + lr) * TS + 16 * ks + 8 * hi);
        acc[ct] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bf, acc[ct], 0, 0, 0);
      }
    }
    // sO aliases sS: every wave's softmax reads finished at the barrier above
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
#pragma unroll
      for (int e = 0; e < 16; ++e) sO[(32 * w + crow(e, hi)) * OS + 32 * ct + lr] = acc[ct][e];
  }
  __syncthreads();
  for (int c = tid; c < L * 8; c += 256) {
    const int i = c >> 3, ch = c & 7;
    const float* src = sO + i * OS + ch * 8;
    v4u out;
#pragma unroll
    for (int q = 0; q < 4; ++q) out[q] = pack_bf16(src[2 * q], src[2 * q + 1]);
    *reinterpret_cast<v4u*>(a.o + (r0 + i) * H + h * HD + ch * 8) = out;
  }
}

// ----------------------------------------------------------------- backward
__global__ void __launch_bounds__(256) attn_bwd_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  // R1 (whole kernel): transposed Q, K, dO + per-row D and LSE
  uint16_t* sQt = reinterpret_cast<uint16_t*>(smem);   // [HD][TS]
  uint16_t* sKt = sQt + HD * TS;
  uint16_t* sdOt = sKt + HD * TS;
  float* sD = reinterpret_cast<float*>(sdOt + HD * TS);  // [LM]
  float* sL = sD + LM;                                   // [LM]
  unsigned char* r2 = reinterpret_cast<unsigned char*>(sL + LM);
  // R2 phase 1: row-major Q, K, V, dO
  uint16_t* sQ = reinterpret_cast<uint16_t*>(r2);
  uint16_t* sK = sQ + LM * RS;
  uint16_t* sV = sK + LM * RS;
  uint16_t* sdO = sV + LM * RS;
  // R2 phase 3: P_drop^T, dS, dS^T  ([LM][TS] each)
  uint16_t* sPdT = reinterpret_cast<uint16_t*>(r2);
  uint16_t* sdS = sPdT + LM * TS;
  uint16_t* sdSt = sdS + LM * TS;
  // R2 phase 5: dQ, dK, dV staged as bf16 [LM][RS]
  uint16_t* sG = reinterpret_cast<uint16_t*>(r2);

  const int bh = blockIdx.x;
  const int n = bh / a.nh, h = bh - n * a.nh;
  const int L = a.len[n];
  if (L <= 0) return;
  const int64_t r0 = a.start[n];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, hi = lane >> 5, lr = lane & 31;
  const int H = a.nh * HD;

  // ---- phase 1: loads (rows past L are zero), all pieces in flight first
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    v4u q[2], k[2], v[2], g[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int c = tid + 256 * (2 * half + u), i = c >> 3, ch = c & 7;
      q[u] = k[u] = v[u] = g[u] = v4u{0u, 0u, 0u, 0u};
      if (i < L) {
        const uint16_t* row = a.qkv + (r0 + i) * (3 * H) + h * HD + ch * 8;
        q[u] = *reinterpret_cast<const v4u*>(row);
        k[u] = *reinterpret_cast<const v4u*>(row + H);
        v[u] = *reinterpret_cast<const v4u*>(row + 2 * H);
        g[u] = *reinterpret_cast<const v4u*>(a.dout + (r0 + i) * H + h * HD + ch * 8);
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int c = tid + 256 * (2 * half + u), i = c >> 3, ch = c & 7;
      *reinterpret_cast<v4u*>(sQ + i * RS + ch * 8) = q[u];
      *reinterpret_cast<v4u*>(sK + i * RS + ch * 8) = k[u];
      *reinterpret_cast<v4u*>(sV + i * RS + ch * 8) = v[u];
      *reinterpret_cast<v4u*>(sdO + i * RS + ch * 8) = g[u];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int d = ch * 8 + e, sh = 16 * (e & 1);
        sQt[d * TS + i] = static_cast<uint16_t>((q[u][e >> 1] >> sh) & 0xffffu);
        sKt[d * TS + i] = static_cast<uint16_t>((k[u][e >> 1] >> sh) & 0xffffu);
        sdOt[d * TS + i] = static_cast<uint16_t>((g[u][e >> 1] >> sh) & 0xffffu);
      }
    }
  }
  {  // D_i = dO_i . O_i (2 threads per row), LSE_i
    const int i = tid >> 1, half = tid & 1;
    float s = 0.f;
    if (i < L) {
      const uint16_t* orow = a.o + (r0 + i) * H + h * HD + half * 32;
      const uint16_t* grow = a.dout + (r0 + i) * H + h * HD + half * 32;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const v4u ov = *reinterpret_cast<const v4u*>(orow + 8 * q);
        const v4u gv = *reinterpret_cast<const v4u*>(grow + 8 * q);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int sh = 16 * (e & 1);
          s += bfval(static_cast<uint16_t>((ov[e >> 1] >> sh) & 0xffffu)) *
               bfval(static_cast<uint16_t>((gv[e >> 1] >> sh) & 0xffffu));
        }
      }
    }
    s += __shfl_xor(s, 1, 64);
    if (half == 0) {
      sD[i] = s;
      sL[i] = i < L ? a.lse[static_cast<int64_t>(bh) * LM + i] : 0.f;
    }
  }
  __syncthreads();

  // ---- phase 2: S, dP_drop for this wave's 32 query rows; P_drop, dS in registers
  f32x16_t pd[4], ds[4];
#pragma unroll
  for (int ct = 0; ct < 4; ++ct) {
    pd[ct] = zero16();
    ds[ct] = zero16();
  }
  const bool active = 32 * w < L;
  if (active) {
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) {
      if (ct > w) break;
      f32x16_t s = zero16(), dp = zero16();
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int ko = 16 * ks + 8 * hi;
        const bf16x8_t qa = *reinterpret_cast<const bf16x8_t*>(sQ + (32 * w + lr) * RS + ko);
        const bf16x8_t kb = *reinterpret_cast<const bf16x8_t*>(sK + (32 * ct + lr) * RS + ko);
        const bf16x8_t ga = *reinterpret_cast<const bf16x8_t*>(sdO + (32 * w + lr) * RS + ko);
        const bf16x8_t vb = *reinterpret_cast<const bf16x8_t*>(sV + (32 * ct + lr) * RS + ko);
        s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(qa, kb, s, 0, 0, 0);
        dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ga, vb, dp, 0, 0, 0);
      }
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = 32 * w + crow(e, hi), col = 32 * ct + lr;
        const bool valid = col <= row && row < L;
        const float P = valid ? __expf(s[e] * a.scale - sL[row]) : 0.f;
        bool keep = true;
        if (a.thresh != 0u)
          keep = akeep((static_cast<uint64_t>(bh) * LM + row) * LM + col, a.seed, a.thresh);
        const float dP = keep ? dp[e] * a.dscale : 0.f;
        pd[ct][e] = keep ? P * a.dscale : 0.f;
        ds[ct][e] = P * (dP - sD[row]) * a.scale;
      }
    }
  }
  __syncthreads();  // every wave is done with the row-major R2 tiles

  // ---- phase 3: zero R2, then scatter P_drop^T, dS, dS^T (bf16)
  {
    v4u* z = reinterpret_cast<v4u*>(r2);
    const v4u zz = {0u, 0u, 0u, 0u};
    for (int c = tid; c < 3 * LM * TS / 8; c += 256) z[c] = zz;
  }
  __syncthreads();
  if (active) {
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) {
      if (ct > w) break;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = 32 * w + crow(e, hi), col = 32 * ct + lr;
        const uint16_t pb = bfbits(pd[ct][e]), db = bfbits(ds[ct][e]);
        sPdT[col * TS + row] = pb;
        sdS[row * TS + col] = db;
        sdSt[col * TS + row] = db;
      }
    }
  }
  __syncthreads();

  // ---- phase 4: dQ (query rows of this wave), dK, dV (key rows of this wave)
  f32x16_t gq[2] = {zero16(), zero16()}, gk[2] = {zero16(), zero16()}, gv[2] = {zero16(), zero16()};
  if (active) {
    for (int ks = 0; ks < 2 * w + 2; ++ks) {  // keys j <= this strip's rows
      const bf16x8_t af = *reinterpret_cast<const bf16x8_t*>(sdS + (32 * w + lr) * TS + 16 * ks + 8 * hi);
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {
        const bf16x8_t bf = *reinterpret_cast<const bf16x8_t*>(sKt + (32 * ct + lr) * TS + 16 * ks + 8 * hi);
        gq[ct] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bf, gq[ct], 0, 0, 0);
      }
    }
    const int kend = (L + 15) / 16;
    for (int ks = 2 * w; ks < kend; ++ks) {  // queries i >= this strip's keys
      const int ko = 16 * ks + 8 * hi;
      const bf16x8_t pa = *reinterpret_cast<const bf16x8_t*>(sPdT + (32 * w + lr) * TS + ko);
      const bf16x8_t sa = *reinterpret_cast<const bf16x8_t*>(sdSt + (32 * w + lr) * TS + ko);
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {
        const bf16x8_t gb = *reinterpret_cast<const bf16x8_t*>(sdOt + (32 * ct + lr) * TS + ko);
        const bf16x8_t qb = *reinterpret_cast<const bf16x8_t*>(sQt + (32 * ct + lr) * TS + ko);
        gv[ct] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pa, gb, gv[ct], 0, 0, 0);
        gk[ct] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(sa, qb, gk[ct], 0, 0, 0);
      }
    }
  }
  __syncthreads();  // R2 reads done: stage the gradients there

  // ---- phase 5: stage dQ | dK | dV as bf16 rows, then 16-byte stores
  if (active) {
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = 32 * w + crow(e, hi), col = 32 * ct + lr;
        sG[row * RS + col] = bfbits(gq[ct][e]);
        sG[(LM + row) * RS + col] = bfbits(gk[ct][e]);
        sG[(2 * LM + row) * RS + col] = bfbits(gv[ct][e]);
      }
  }
  __syncthreads();
  for (int c = tid; c < 3 * L * 8; c += 256) {
    const int part = c / (L * 8), rem = c - part * L * 8;
    const int i = rem >> 3, ch = rem & 7;
    const v4u val = *reinterpret_cast<const v4u*>(sG + (part * LM + i) * RS + ch * 8);
    *reinterpret_cast<v4u*>(a.dqkv + (r0 + i) * (3 * H) + part * H + h * HD + ch * 8) = val;
  }
}

constexpr size_t kFwdLds = (2 * LM * RS + HD * TS) * 2 + LM * SS * 4;
constexpr size_t kBwdLds = 3 * HD * TS * 2 + 2 * LM * 4 + 3 * LM * TS * 2;
static_assert(2 * LM * RS >= LM * TS, "P must fit over Q and K");
static_assert(LM * SS >= LM * OS, "O staging must fit over S");
static_assert(3 * LM * TS >= 4 * LM * RS, "row tiles must fit in R2");
static_assert(kBwdLds <= 160 * 1024, "backward LDS");

uint32_t attn_thresh(float p) {
  if (p <= 0.f) return 0u;
  const double t = static_cast<double>(p) * 4294967296.0;
  return t >= 4294967295.0 ? 0xffffffffu : static_cast<uint32_t>(t);
}

}  // namespace

void launch_attn_fwd(AttnArgs a, int64_t nseq, float p_drop, hipStream_t stream) {
  if (nseq == 0) return;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(attn_fwd_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(kFwdLds));
    attr = true;
  }
  a.thresh = attn_thresh(p_drop);
  a.dscale = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  hipLaunchKernelGGL(attn_fwd_kernel, dim3(static_cast<uint32_t>(nseq * a.nh)), dim3(256), kFwdLds,
                     stream, a);
}

void launch_attn_bwd(AttnArgs a, int64_t nseq, float p_drop, hipStream_t stream) {
  if (nseq == 0) return;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(attn_bwd_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(kBwdLds));
    attr = true;
  }
  a.thresh = attn_thresh(p_drop);
  a.dscale = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  hipLaunchKernelGGL(attn_bwd_kernel, dim3(static_cast<uint32_t>(nseq * a.nh)), dim3(256), kBwdLds,
                     stream, a);
}

}  // namespace commeff
