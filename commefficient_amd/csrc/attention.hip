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
//           (seed, ((seq*heads + h)*1024 + i)*1024 + j), the backward
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
constexpr int LM = 128;      // max sequence length of the short (all-in-LDS) kernels
// dropout index: idx = ((seq*heads + h)*DS + i)*DS + j with DS = 1024 (the
// maximum sequence length)
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
// dropout keep(idx) = amix32(lo32(idx) ^ amix32(hi32(idx) + seed)) >= thresh
// (ops/transformer.py _ref_attn), evaluated with the high word hoisted out of
// the element loops: with DS*DS = 2^20, idx = ((bh*DS + i)*DS + j) has high
// word bh >> 12 and low word (bh << 20) + (i << 10) + j (mod 2^32)
__device__ __forceinline__ uint32_t akeep_hs(int bh, uint32_t seed) {
  return amix32((static_cast<uint32_t>(bh) >> 12) + seed);
}
__device__ __forceinline__ uint32_t akeep_lo(int bh, int i, int j) {
  return (static_cast<uint32_t>(bh) << 20) + (static_cast<uint32_t>(i) << 10) + static_cast<uint32_t>(j);
}
__device__ __forceinline__ bool akeep_fast(uint32_t lo, uint32_t hs, uint32_t thresh) {
  return amix32(lo ^ hs) >= thresh;
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
  const int L = min(a.len[n], LM);
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
    const uint32_t hs = akeep_hs(bh, a.seed), ib = akeep_lo(bh, i, half * 64);
#pragma unroll
    for (int t = 0; t < 64; t += 2) {
      float v0 = p[t] * inv, v1 = p[t + 1] * inv;
      if (a.thresh != 0u) {
        v0 = akeep_fast(ib + t, hs, a.thresh) ? v0 * a.dscale : 0.f;
        v1 = akeep_fast(ib + t + 1, hs, a.thresh) ? v1 * a.dscale : 0.f;
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
  const int L = min(a.len[n], LM);
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
          keep = akeep_fast(akeep_lo(bh, row, col), akeep_hs(bh, a.seed), a.thresh);
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


// ============================================================ long sequences
// Flash-style kernels for sequences longer than LM (up to DS = 1024 tokens,
// GPT-2's n_positions): a workgroup owns 128 rows of one (sequence, head) --
// 32 per wave -- and streams the other operand through a double-buffered LDS
// ring in 64-row tiles (the next tile's global loads are in flight while the
// current one is used; one block barrier per tile), with an online softmax.
//   forward   (query rows):  S = Q K^T per 64-key tile into a per-wave fp32
//             tile, row max / rescale / exp / dropout by 2 threads per row
//             (P_drop written over the row's S), O = alpha O + P_drop V;
//             O / l and LSE at the end;
//   backward  dQ kernel (query rows): S, dP = dO V^T per 64-key tile, dS
//             straight from the accumulators into a per-wave transposed
//             image, dQ += dS K; it also writes D_i = dO_i . O_i;
//             dK/dV kernel (key rows): S^T = K Q^T, dP^T = V dO^T per
//             64-query tile, dV += P_drop^T dO, dK += dS^T Q.
// Every operand that an MFMA needs transposed (V for P V, K for dS K, Q and
// dO for the key-row products, dS / P_drop as A operands) is read with the
// gfx950 transposing LDS read ds_read_b64_tr_b16 from the row-major tile (or
// from 8-byte stores of the accumulator columns): no scalar transposing
// stores.  Every output element is written once by one workgroup:
// deterministic, no atomics.  Dropout masks use the same (seq, head, i, j)
// hash as the short kernels, so the two families are interchangeable.
constexpr int QB = 128;  // rows per workgroup
constexpr int TT = 64;   // streamed tile rows
constexpr int T2 = 72;   // bf16 row stride of [64][64] tiles

// global pieces of one 64 x 64 bf16 tile (rows t0 + i of a row block at
// token row r0; rows >= L are zero): two 16-byte pieces per thread
struct TilePieces {
  v4u v[2];
};
__device__ __forceinline__ TilePieces tile_fetch(const uint16_t* base, int64_t ld, int64_t r0, int t0,
                                                 int L, int tid) {
  TilePieces p;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int c = tid + 256 * u, i = c >> 3, ch = c & 7;
    p.v[u] = v4u{0u, 0u, 0u, 0u};
    if (t0 + i < L) p.v[u] = *reinterpret_cast<const v4u*>(base + (r0 + t0 + i) * ld + ch * 8);
  }
  return p;
}
__device__ __forceinline__ void tile_store(uint16_t* dst, const TilePieces& p, int tid) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int c = tid + 256 * u, i = c >> 3, ch = c & 7;
    *reinterpret_cast<v4u*>(dst + i * T2 + ch * 8) = p.v[u];
  }
}

// A-operand fragments of 32 rows x 64 columns straight from global memory
// (lane: row lr, k = 16 ks + 8 hi); rows >= L are zero
__device__ __forceinline__ void frag_load(bf16x8_t f[4], const uint16_t* base, int64_t ld, int64_t row,
                                          bool valid, int hi) {
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    v4u v = v4u{0u, 0u, 0u, 0u};
    if (valid) v = *reinterpret_cast<const v4u*>(base + row * ld + 16 * ks + 8 * hi);
    f[ks] = __builtin_bit_cast(bf16x8_t, v);
  }
}

// Transposing-read operand (cdna_hip_programming.md T10): 32 columns
// [cb, cb + 32) x 16 rows [16 ks, 16 ks + 16) of a bf16 image with row
// stride LD elements, as the MFMA operand whose lane holds column
// cb + (lane & 31) and k = 8 (lane >> 5) + j.  Lane 4q + p of each 16-lane
// group addresses row q (+4 for the second read), columns 4p .. 4p + 3.
template <int LD>
__device__ __forceinline__ bf16x8_t tr_op(const uint16_t* img, int cb, int ks, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int col = cb + 16 * (g & 1) + 4 * p;
  const int row = 16 * ks + 8 * (g >> 1) + q;
  const unsigned char* b = reinterpret_cast<const unsigned char*>(img);
  return tr_read(b + (row * LD + col) * 2, b + ((row + 4) * LD + col) * 2);
}

// 32 rows x 64 columns staged bf16 in a per-wave [32][stride] tile -> token
// rows r0 + g0 + row (< L) of a [M, ld] bf16 matrix
template <int STRIDE>
__device__ __forceinline__ void rows_store(uint16_t* out, int64_t ld, int64_t r0, int g0, int L,
                                           const uint16_t* stage, int lane) {
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int c = lane + 64 * u, row = c >> 3, ch = c & 7;
    if (g0 + row < L)
      *reinterpret_cast<v4u*>(out + (r0 + g0 + row) * ld + ch * 8) =
          *reinterpret_cast<const v4u*>(stage + row * STRIDE + ch * 8);
  }
}

template <int STRIDE>
__device__ __forceinline__ void stage_acc(uint16_t* stage, const f32x16_t acc[2], int hi, int lr,
                                          const float* rowscale) {
#pragma unroll
  for (int ct = 0; ct < 2; ++ct)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int row = crow(e, hi);
      const float v = rowscale ? acc[ct][e] * rowscale[row] : acc[ct][e];
      stage[row * STRIDE + 32 * ct + lr] = bfbits(v);
    }
}



// Forward, transposed formulation: the same tiles and online softmax with the
// scores computed as S^T = K Q^T, so the accumulator lane (query lr, half hi)
// holds 16 keys of ITS query: the row max / sum are lane-local plus one
// xor-shuffle with lane ^ 32, P never leaves the registers (it is the B
// operand of O^T += V^T P^T: an accumulator's keys 8 (ks & 1) .. + 7 are the
// operand's k slots, and the V^T operand is read with the SAME key order --
// transposing reads of rows kb + 4 hi + 0..3 and kb + 8 + 4 hi + 0..3), and the
// O rescale by alpha and the final 1 / l are lane-local.  No per-wave S / P /
// alpha images: 37 KB of LDS (the K / V ring) and no wave-level LDS round
// trips between the two MFMA phases.
template <int LD>
__device__ __forceinline__ bf16x8_t tr_op_perm(const uint16_t* img, int cb, int kb, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int col = cb + 16 * (g & 1) + 4 * p;
  const int row = kb + 4 * (g >> 1) + q;
  const unsigned char* b = reinterpret_cast<const unsigned char*>(img);
  return tr_read(b + (row * LD + col) * 2, b + ((row + 8) * LD + col) * 2);
}

__global__ void __launch_bounds__(256, 3) attn_long_fwd_t_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint16_t* sK = reinterpret_cast<uint16_t*>(smem);   // [2][TT][T2]
  uint16_t* sV = sK + 2 * TT * T2;                     // [2][TT][T2]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, hi = lane >> 5, lr = lane & 31;
  const int tiles = a.lse_ld / QB;
  const int bh = blockIdx.x / tiles, q0 = (blockIdx.x - bh * tiles) * QB;
  const int n = bh / a.nh, h = bh - n * a.nh;
  const int L = min(a.len[n], a.lse_ld);
  if (q0 >= L) return;
  const int64_t r0 = a.start[n];
  const int H = a.nh * HD;
  const int64_t ld3 = 3 * static_cast<int64_t>(H);
  const int wq0 = q0 + 32 * w;
  const bool wvalid = wq0 < L;
  const int qi = wq0 + lr;  // this lane's query
  const uint16_t* kbase = a.qkv + H + h * HD;
  const uint16_t* vbase = a.qkv + 2 * H + h * HD;
  bf16x8_t qf[4];  // B operand: query lr, dims 16 ks + 8 hi ..
  frag_load(qf, a.qkv + h * HD, ld3, r0 + qi, qi < L, hi);
  f32x16_t o[2] = {zero16(), zero16()};  // O^T: dims 32 dt + crow(e, hi), query lr
  float m_run = -__builtin_huge_valf(), l_run = 0.f;
  const uint32_t hs = akeep_hs(bh, a.seed);
  const int nkt = (min(q0 + QB, L) - 1) / TT + 1;
  {
    const TilePieces pk = tile_fetch(kbase, ld3, r0, 0, L, tid);
    const TilePieces pv = tile_fetch(vbase, ld3, r0, 0, L, tid);
    tile_store(sK, pk, tid);
    tile_store(sV, pv, tid);
  }
  __syncthreads();
  for (int kt = 0; kt < nkt; ++kt) {
    const uint16_t* cK = sK + (kt & 1) * TT * T2;
    const uint16_t* cV = sV + (kt & 1) * TT * T2;
    TilePieces pk, pv;
    const bool more = kt + 1 < nkt;
    if (more) {  // next tile's loads in flight during this tile's math
      pk = tile_fetch(kbase, ld3, r0, (kt + 1) * TT, L, tid);
      pv = tile_fetch(vbase, ld3, r0, (kt + 1) * TT, L, tid);
    }
    if (wvalid && kt * TT <= wq0 + 31) {
      f32x16_t s[2];
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {  // keys 32 ct ..
        s[ct] = zero16();
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
          const bf16x8_t kf = *reinterpret_cast<const bf16x8_t*>(cK + (32 * ct + lr) * T2 + 16 * ks + 8 * hi);
          s[ct] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[ks], s[ct], 0, 0, 0);
        }
      }
      float mt = -__builtin_huge_valf();
#pragma unroll
      for (int ct = 0; ct < 2; ++ct)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int j = kt * TT + 32 * ct + crow(e, hi);
          const float v = (j <= qi && qi < L) ? s[ct][e] * a.scale : -__builtin_huge_valf();
          s[ct][e] = v;
          mt = fmaxf(mt, v);
        }
      mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
      const float m_new = fmaxf(m_run, mt);
      const bool live = m_new > -__builtin_huge_valf();
      const float alpha = live ? __expf(m_run - m_new) : 1.f;
      float sum = 0.f;
      bf16x8_t pf[4];  // B operand of O^T: keys of k-step ks = accumulator ct = ks >> 1, e = 8 (ks & 1) ..
#pragma unroll
      for (int ct = 0; ct < 2; ++ct)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          float p = live ? __expf(s[ct][e] - m_new) : 0.f;
          sum += p;
          if (a.thresh != 0u) {
            const int j = kt * TT + 32 * ct + crow(e, hi);
            p = akeep_fast(akeep_lo(bh, qi, j), hs, a.thresh) ? p * a.dscale : 0.f;
          }
          pf[2 * ct + (e >> 3)][e & 7] = static_cast<__bf16>(p);
        }
      l_run = l_run * alpha + sum;
      m_run = live ? m_new : m_run;
#pragma unroll
      for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int e = 0; e < 16; ++e) o[dt][e] *= alpha;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
#pragma unroll
        for (int dt = 0; dt < 2; ++dt)
          o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_op_perm<T2>(cV, 32 * dt, 16 * ks, lane), pf[ks],
                                                          o[dt], 0, 0, 0);
    }
    if (more) {  // the other buffer was last read before the previous barrier
      tile_store(sK + ((kt + 1) & 1) * TT * T2, pk, tid);
      tile_store(sV + ((kt + 1) & 1) * TT * T2, pv, tid);
    }
    __syncthreads();
  }
  if (wvalid && qi < L) {
    const float l = l_run + __shfl_xor(l_run, 32, 64);
    const float inv = 1.f / l;
    if (hi == 0) a.lse[static_cast<int64_t>(bh) * a.lse_ld + qi] = m_run + __logf(l);
    uint16_t* orow = a.o + (r0 + qi) * H + h * HD;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int grp = 0; grp < 4; ++grp) {  // dims 32 dt + 8 grp + 4 hi .. + 3
        uint2 v;
        v.x = pack_bf16(o[dt][4 * grp] * inv, o[dt][4 * grp + 1] * inv);
        v.y = pack_bf16(o[dt][4 * grp + 2] * inv, o[dt][4 * grp + 3] * inv);
        *reinterpret_cast<uint2*>(orow + 32 * dt + 8 * grp + 4 * hi) = v;
      }
  }
}

// dQ (+ D), transposed formulation (as attn_long_fwd_t_kernel): S^T = K Q^T
// and dP^T = V dO^T put one query per lane, so LSE_i and D_i are lane-local,
// dS^T = P^T (dP^T - D) never leaves the registers, and dQ^T += K^T dS^T reads
// K^T with the permuted key order of the register operand.  LDS: the K / V
// ring only.
__global__ void __launch_bounds__(256, 3) attn_long_dq_t_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint16_t* sK = reinterpret_cast<uint16_t*>(smem);
  uint16_t* sV = sK + 2 * TT * T2;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, hi = lane >> 5, lr = lane & 31;
  const int tiles = a.lse_ld / QB;
  const int bh = blockIdx.x / tiles, q0 = (blockIdx.x - bh * tiles) * QB;
  const int n = bh / a.nh, h = bh - n * a.nh;
  const int L = min(a.len[n], a.lse_ld);
  if (q0 >= L) return;
  const int64_t r0 = a.start[n];
  const int H = a.nh * HD;
  const int64_t ld3 = 3 * static_cast<int64_t>(H);
  const int wq0 = q0 + 32 * w;
  const bool wvalid = wq0 < L;
  const int qi = wq0 + lr;
  const bool qok = qi < L;
  const uint16_t* kbase = a.qkv + H + h * HD;
  const uint16_t* vbase = a.qkv + 2 * H + h * HD;
  bf16x8_t qf[4], gf[4];  // B operands: query lr, dims 16 ks + 8 hi ..
  frag_load(qf, a.qkv + h * HD, ld3, r0 + qi, qok, hi);
  frag_load(gf, a.dout + h * HD, H, r0 + qi, qok, hi);
  float Di = 0.f, Li = 0.f;
  {  // D_i = dO_i . O_i (lanes lr and lr + 32: 32 dims each) and LSE_i
    if (qok) {
      const uint16_t* orow = a.o + (r0 + qi) * H + h * HD + hi * 32;
      const uint16_t* grow = a.dout + (r0 + qi) * H + h * HD + hi * 32;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const v4u ov = *reinterpret_cast<const v4u*>(orow + 8 * q);
        const v4u gv = *reinterpret_cast<const v4u*>(grow + 8 * q);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int sh = 16 * (e & 1);
          Di += bfval(static_cast<uint16_t>((ov[e >> 1] >> sh) & 0xffffu)) *
                bfval(static_cast<uint16_t>((gv[e >> 1] >> sh) & 0xffffu));
        }
      }
      Li = a.lse[static_cast<int64_t>(bh) * a.lse_ld + qi];
    }
    Di += __shfl_xor(Di, 32, 64);
    if (qok && hi == 0) a.dbuf[static_cast<int64_t>(bh) * a.lse_ld + qi] = Di;
  }
  const uint32_t hs = akeep_hs(bh, a.seed);
  f32x16_t gq[2] = {zero16(), zero16()};  // dQ^T: dims 32 dt + crow(e, hi), query lr
  const int nkt = (min(q0 + QB, L) - 1) / TT + 1;
  {
    const TilePieces pk = tile_fetch(kbase, ld3, r0, 0, L, tid);
    const TilePieces pv = tile_fetch(vbase, ld3, r0, 0, L, tid);
    tile_store(sK, pk, tid);
    tile_store(sV, pv, tid);
  }
  __syncthreads();
  for (int kt = 0; kt < nkt; ++kt) {
    const uint16_t* cK = sK + (kt & 1) * TT * T2;
    const uint16_t* cV = sV + (kt & 1) * TT * T2;
    TilePieces pk, pv;
    const bool more = kt + 1 < nkt;
    if (more) {
      pk = tile_fetch(kbase, ld3, r0, (kt + 1) * TT, L, tid);
      pv = tile_fetch(vbase, ld3, r0, (kt + 1) * TT, L, tid);
    }
    if (wvalid && kt * TT <= wq0 + 31) {
      bf16x8_t df[4];  // dS^T as the B operand of k-step ks (permuted key order)
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {  // keys 32 ct ..
        f32x16_t s = zero16(), dp = zero16();
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
          const int ko = (32 * ct + lr) * T2 + 16 * ks + 8 * hi;
          s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*reinterpret_cast<const bf16x8_t*>(cK + ko), qf[ks], s, 0, 0, 0);
          dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*reinterpret_cast<const bf16x8_t*>(cV + ko), gf[ks], dp, 0, 0, 0);
        }
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int j = kt * TT + 32 * ct + crow(e, hi);
          const bool valid = j <= qi && qok;
          const float P = valid ? __expf(s[e] * a.scale - Li) : 0.f;
          bool keep = true;
          if (a.thresh != 0u) keep = akeep_fast(akeep_lo(bh, qi, j), hs, a.thresh);
          const float dP = keep ? dp[e] * a.dscale : 0.f;
          df[2 * ct + (e >> 3)][e & 7] = static_cast<__bf16>(P * (dP - Di) * a.scale);
        }
      }
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
#pragma unroll
        for (int dt = 0; dt < 2; ++dt)
          gq[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_op_perm<T2>(cK, 32 * dt, 16 * ks, lane), df[ks],
                                                           gq[dt], 0, 0, 0);
    }
    if (more) {
      tile_store(sK + ((kt + 1) & 1) * TT * T2, pk, tid);
      tile_store(sV + ((kt + 1) & 1) * TT * T2, pv, tid);
    }
    __syncthreads();
  }
  if (wvalid && qok) {
    uint16_t* drow = a.dqkv + (r0 + qi) * ld3 + h * HD;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int grp = 0; grp < 4; ++grp) {  // dims 32 dt + 8 grp + 4 hi .. + 3
        uint2 v;
        v.x = pack_bf16(gq[dt][4 * grp], gq[dt][4 * grp + 1]);
        v.y = pack_bf16(gq[dt][4 * grp + 2], gq[dt][4 * grp + 3]);
        *reinterpret_cast<uint2*>(drow + 32 * dt + 8 * grp + 4 * hi) = v;
      }
  }
}



// dK, dV with the scores in query-row form: S = Q K^T and dP = dO V^T put one
// KEY per lane (column lr), so P_drop and dS are, as they come out of the
// accumulators, the B operands of dV^T += dO^T P_drop and dK^T += Q^T dS (key
// n = lane, query k in the accumulator's permuted order; dO^T / Q^T read with
// the same order).  LSE / D per query row come from the staged [2][64] rows.
// LDS: the Q / dO ring + LSE / D (38 KB), no per-wave P / dS images.
__global__ void __launch_bounds__(256, 2) attn_long_dkdv_s_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint16_t* sQ = reinterpret_cast<uint16_t*>(smem);
  uint16_t* sG = sQ + 2 * TT * T2;
  float* sL = reinterpret_cast<float*>(sG + 2 * TT * T2);  // [2][TT]
  float* sD = sL + 2 * TT;                                  // [2][TT]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, hi = lane >> 5, lr = lane & 31;
  const int tiles = a.lse_ld / QB;
  const int bh = blockIdx.x / tiles, k0 = (blockIdx.x - bh * tiles) * QB;
  const int n = bh / a.nh, h = bh - n * a.nh;
  const int L = min(a.len[n], a.lse_ld);
  if (k0 >= L) return;
  const int64_t r0 = a.start[n];
  const int H = a.nh * HD;
  const int64_t ld3 = 3 * static_cast<int64_t>(H);
  const int wk0 = k0 + 32 * w;
  const bool wvalid = wk0 < L;
  const int kj = wk0 + lr;  // this lane's key
  const uint16_t* qbase = a.qkv + h * HD;
  const uint16_t* gbase = a.dout + h * HD;
  const float* lrow = a.lse + static_cast<int64_t>(bh) * a.lse_ld;
  const float* drow = a.dbuf + static_cast<int64_t>(bh) * a.lse_ld;
  bf16x8_t kf[4], vf[4];  // B operands: key lr, dims 16 ks + 8 hi ..
  frag_load(kf, a.qkv + H + h * HD, ld3, r0 + kj, kj < L, hi);
  frag_load(vf, a.qkv + 2 * H + h * HD, ld3, r0 + kj, kj < L, hi);
  const uint32_t hs = akeep_hs(bh, a.seed);
  f32x16_t gk[2] = {zero16(), zero16()}, gv[2] = {zero16(), zero16()};  // dims 32 dt + crow, key lr
  {
    const TilePieces pq = tile_fetch(qbase, ld3, r0, k0, L, tid);
    const TilePieces pg = tile_fetch(gbase, H, r0, k0, L, tid);
    tile_store(sQ, pq, tid);
    tile_store(sG, pg, tid);
    if (tid < TT) {
      const int i = k0 + tid;
      sL[tid] = i < L ? lrow[i] : 0.f;
      sD[tid] = i < L ? drow[i] : 0.f;
    }
  }
  __syncthreads();
  for (int qs = k0, it = 0; qs < L; qs += TT, ++it) {
    const int b = it & 1;
    const uint16_t* cQ = sQ + b * TT * T2;
    const uint16_t* cG = sG + b * TT * T2;
    const float* cL = sL + b * TT;
    const float* cD = sD + b * TT;
    TilePieces pq, pg;
    float nl = 0.f, nd = 0.f;
    const bool more = qs + TT < L;
    if (more) {
      pq = tile_fetch(qbase, ld3, r0, qs + TT, L, tid);
      pg = tile_fetch(gbase, H, r0, qs + TT, L, tid);
      if (tid < TT) {
        const int i = qs + TT + tid;
        nl = i < L ? lrow[i] : 0.f;
        nd = i < L ? drow[i] : 0.f;
      }
    }
    if (wvalid && qs + TT - 1 >= wk0) {
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {  // queries 32 ct .. : k-steps 2 ct, 2 ct + 1
        f32x16_t s = zero16(), dp = zero16();
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
          const int qo = (32 * ct + lr) * T2 + 16 * ks + 8 * hi;
          s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*reinterpret_cast<const bf16x8_t*>(cQ + qo), kf[ks], s, 0, 0, 0);
          dp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*reinterpret_cast<const bf16x8_t*>(cG + qo), vf[ks], dp, 0, 0, 0);
        }
        bf16x8_t pfr[2], sfr[2];  // P_drop / dS as B operands (permuted query order)
#pragma unroll
        for (int grp = 0; grp < 4; ++grp) {
          const int qr = 32 * ct + 8 * grp + 4 * hi;  // tile rows qr .. qr + 3 (e = 4 grp ..)
          const float4 l4 = *reinterpret_cast<const float4*>(cL + qr);
          const float4 d4 = *reinterpret_cast<const float4*>(cD + qr);
          const float lv[4] = {l4.x, l4.y, l4.z, l4.w}, dv[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const int e = 4 * grp + t;
            const int i = qs + qr + t;  // query
            const bool valid = kj <= i && i < L;
            const float P = valid ? __expf(s[e] * a.scale - lv[t]) : 0.f;
            bool keep = true;
            if (a.thresh != 0u) keep = akeep_fast(akeep_lo(bh, i, kj), hs, a.thresh);
            const float dP = keep ? dp[e] * a.dscale : 0.f;
            pfr[e >> 3][e & 7] = static_cast<__bf16>(keep ? P * a.dscale : 0.f);
            sfr[e >> 3][e & 7] = static_cast<__bf16>(P * (dP - dv[t]) * a.scale);
          }
        }
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int dt = 0; dt < 2; ++dt) {
            const int kb = 32 * ct + 16 * u;
            gv[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_op_perm<T2>(cG, 32 * dt, kb, lane), pfr[u],
                                                             gv[dt], 0, 0, 0);
            gk[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_op_perm<T2>(cQ, 32 * dt, kb, lane), sfr[u],
                                                             gk[dt], 0, 0, 0);
          }
      }
    }
    if (more) {
      tile_store(sQ + (b ^ 1) * TT * T2, pq, tid);
      tile_store(sG + (b ^ 1) * TT * T2, pg, tid);
      if (tid < TT) {
        sL[(b ^ 1) * TT + tid] = nl;
        sD[(b ^ 1) * TT + tid] = nd;
      }
    }
    __syncthreads();
  }
  if (wvalid && kj < L) {
    uint16_t* krow = a.dqkv + (r0 + kj) * ld3 + H + h * HD;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int grp = 0; grp < 4; ++grp) {  // dims 32 dt + 8 grp + 4 hi .. + 3
        uint2 k2, v2;
        k2.x = pack_bf16(gk[dt][4 * grp], gk[dt][4 * grp + 1]);
        k2.y = pack_bf16(gk[dt][4 * grp + 2], gk[dt][4 * grp + 3]);
        v2.x = pack_bf16(gv[dt][4 * grp], gv[dt][4 * grp + 1]);
        v2.y = pack_bf16(gv[dt][4 * grp + 2], gv[dt][4 * grp + 3]);
        *reinterpret_cast<uint2*>(krow + 32 * dt + 8 * grp + 4 * hi) = k2;
        *reinterpret_cast<uint2*>(krow + H + 32 * dt + 8 * grp + 4 * hi) = v2;
      }
  }
}

constexpr size_t kLongFwdTLds = 4 * TT * T2 * 2;  // the K / V ring only
constexpr size_t kLongDkdvSLds = 4 * TT * T2 * 2 + 4 * TT * 4;  // Q / dO ring + LSE / D
static_assert(kLongDkdvSLds <= 80 * 1024 && kLongFwdTLds <= 80 * 1024, "2 workgroups per CU");

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
  if (a.lse_ld > LM) {  // long sequences: flash-style kernel
    static bool lattr = false;
    if (!lattr) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(attn_long_fwd_t_kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(kLongFwdTLds));
      lattr = true;
    }
    a.thresh = attn_thresh(p_drop);
    a.dscale = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
    const dim3 grid(static_cast<uint32_t>(nseq * a.nh * (a.lse_ld / QB)));
    COMMEFF_LAUNCH(attn_long_fwd_t_kernel, grid, dim3(256), kLongFwdTLds, stream, a);
    return;
  }
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(attn_fwd_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(kFwdLds));
    attr = true;
  }
  a.thresh = attn_thresh(p_drop);
  a.dscale = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  COMMEFF_LAUNCH(attn_fwd_kernel, dim3(static_cast<uint32_t>(nseq * a.nh)), dim3(256), kFwdLds,
                     stream, a);
}

void launch_attn_bwd(AttnArgs a, int64_t nseq, float p_drop, hipStream_t stream) {
  if (nseq == 0) return;
  if (a.lse_ld > LM) {  // long sequences: dQ (+ D) kernel, then dK / dV kernel
    static bool tattr = false;
    if (!tattr) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(attn_long_dq_t_kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(kLongFwdTLds));
      tattr = true;
    }
    a.thresh = attn_thresh(p_drop);
    a.dscale = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
    const dim3 grid(static_cast<uint32_t>(nseq * a.nh * (a.lse_ld / QB)));
    COMMEFF_LAUNCH(attn_long_dq_t_kernel, grid, dim3(256), kLongFwdTLds, stream, a);
    {
      static bool sattr = false;
      if (!sattr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(attn_long_dkdv_s_kernel),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(kLongDkdvSLds));
        sattr = true;
      }
      COMMEFF_LAUNCH(attn_long_dkdv_s_kernel, grid, dim3(256), kLongDkdvSLds, stream, a);
    }
    return;
  }
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(attn_bwd_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(kBwdLds));
    attr = true;
  }
  a.thresh = attn_thresh(p_drop);
  a.dscale = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  COMMEFF_LAUNCH(attn_bwd_kernel, dim3(static_cast<uint32_t>(nseq * a.nh)), dim3(256), kBwdLds,
                     stream, a);
}

}  // namespace commeff
