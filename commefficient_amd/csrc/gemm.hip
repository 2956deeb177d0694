// Dense bf16 GEMMs of the model layers on the gfx950 MFMA:
//
//   C[M][N] = act(A[M][K] . op(B) + bias[N]) (+ beta * C)      fp32 accumulation
//     NT: B stored [N][K] (K contiguous)  -- Linear forward with the weight as
//         [out][in], 1x1-conv forward ([K_out][C_in]), GPT-2 input gradients
//         (dY [T][out] . W[in][out]^T), the tied LM head (hid . wte^T);
//     NN: B stored [K][N] (N contiguous)  -- HF Conv1D forward (X . W[in][out]),
//         1x1-conv input gradients (dY . W[K_out][C_in]).
//   act: none or tanh-GELU (GPT-2 MLP; the pre-activation is stored too).
//
// Replaces the hipBLASLt (Cijk_*) GEMMs of the GPT-2 blocks (reference model:
// /root/reference/CommEfficient/gpt2_train.py:262-273, HF GPT2DoubleHeads) and
// of the ResNet bottlenecks' 1x1 convs (models/resnets.py:76-130).
//
// Tile: BM = 128 rows x BN (128 or 64) columns per 4-wave block (waves 2 x 2,
// 64 x BN/2 each, 32x32x16 MFMAs), 64-deep K-steps through a two-stage LDS
// ring filled by LDS DMA (global_load_lds, 16 bytes a lane, no staging
// registers), one raw s_barrier per K-step, two blocks per CU (the measured
// best trade of ring depth for occupancy on the conv kernels, conv.hip).  A
// (and B for NT) is staged [rows][64 k] with the XOR swizzle applied on the
// SOURCE address (the DMA writes lane-linearly) and read with ds_read_b128;
// B for NN is staged K-major [64 k][BN] and read with the transposing
// ds_read_b64_tr_b16.  Rows past M load a zero page and are not stored.
// Tile -> block mapping is XCD-aware.  The epilogue stages the fp32 tile
// through LDS and writes 16-byte rows.
#include <hip/hip_runtime.h>
#include <cstdint>
#include "kernels.h"
#include "conv_common.h"

namespace commeff {
namespace {

constexpr int GK = 64;  // K-step

__device__ __attribute__((aligned(16))) uint32_t g_mm_zero[4] = {0u, 0u, 0u, 0u};

__device__ __forceinline__ void mm_glds16(const void* src, unsigned char* lds) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

__device__ __forceinline__ float gelu_tanh(float x) {
  const float u = 0.7978845608028654f * (x + 0.044715f * x * x * x);
  return 0.5f * x * (1.f + tanhf(u));
}

// v[0..7] += bias[n..n+7] (fp32 or bf16 bias vector)
__device__ __forceinline__ void add_bias(const GemmArgs& a, int n, float v[8]) {
  if (a.bias != nullptr) {
    const float4 b0 = *reinterpret_cast<const float4*>(a.bias + n);
    const float4 b1 = *reinterpret_cast<const float4*>(a.bias + n + 4);
    v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w;
    v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
  } else if (a.bias16 != nullptr) {
    const v4u b = *reinterpret_cast<const v4u*>(a.bias16 + n);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] += bf2f((b[j >> 1] >> (16 * (j & 1))) & 0xffffu);
  }
}

template <int BN, bool NN>
struct MmCfg {
  static constexpr int BM = 128, NT = 256;
  static constexpr int A_BYTES = BM * GK * 2;          // [128 rows][64 k]
  static constexpr int B_BYTES = BN * GK * 2;          // NT: [BN rows][64 k]; NN: [64 k][BN]
  static constexpr int STAGE = A_BYTES + B_BYTES;
  static constexpr int ALD = A_BYTES / 16 / NT;        // 4
  static constexpr int BLD = B_BYTES / 16 / NT;        // 4 or 2
  static constexpr int LD = BN + 4;                    // epilogue fp32 row stride
  static constexpr int EPI = BM * LD * 4;
  static constexpr int LDS = 2 * STAGE > EPI ? 2 * STAGE : EPI;
};

template <int BN, bool NN, int ACT, bool F32, bool ST = false, bool IMP = false>
__global__ void __launch_bounds__(256) gemm_kernel(GemmArgs a0) {
  using Cfg = MmCfg<BN, NN>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int NI = BN / 64, ALD = Cfg::ALD, BLD = Cfg::BLD;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1, hi = lane >> 5, lr = lane & 31;
  int bid = xcd_remap(blockIdx.x, gridDim.x);
  // (NT: N need not be a tile multiple -- B rows past N load the zero page,
  // column chunks past N are not stored; the tied LM head's 50,257 rows)
  const int ntn = (a0.N + BN - 1) / BN;
  GemmArgs a = a0;
  if (a0.G > 1) {  // group of this block (its tiles are consecutive)
    const int per_g = ((a0.M + Cfg::BM - 1) / Cfg::BM) * ntn;
    const int grp = bid / per_g;
    bid -= grp * per_g;
    a.A += grp * a0.sa;
    a.B += grp * a0.sb;
    a.C = static_cast<unsigned char*>(a0.C) + grp * a0.sc * (F32 ? 4 : 2);
  }
  const int m0 = (bid / ntn) * Cfg::BM, n0 = (bid % ntn) * BN;
  const int KT = a.K / GK;
  const uint16_t* zero = reinterpret_cast<const uint16_t*>(g_mm_zero);

  // A pieces: slot s = i*256 + tid -> (row s >> 3, swizzled chunk)
  const uint16_t* a_ptr[ALD];
  int imp_h0[ALD], imp_w0[ALD];  // IMP: the output pixel's input origin (oh s - pad, ow s - pad)
#pragma unroll
  for (int i = 0; i < ALD; ++i) {
    const int s = i * 256 + tid, row = s >> 3, lc = (s & 7) ^ sw_rd128(row);
    if constexpr (IMP) {
      const int p = m0 + row, ohw = a.imp_OH * a.imp_OW;
      const int n = p / ohw, rem = p - n * ohw, oh = rem / a.imp_OW, ow = rem - oh * a.imp_OW;
      imp_h0[i] = oh * a.imp_s - a.imp_pad;
      imp_w0[i] = ow * a.imp_s - a.imp_pad;
      // image n's first pixel row (+ this lane's channel chunk)
      a_ptr[i] = p < a.M ? a.A + static_cast<int64_t>(n) * a.imp_H * a.imp_W * a.lda + lc * 8 : nullptr;
    } else {
      a_ptr[i] = m0 + row < a.M ? a.A + static_cast<int64_t>(m0 + row) * a.lda + lc * 8 : nullptr;
    }
  }
  const uint16_t* b_ptr[BLD];
#pragma unroll
  for (int j = 0; j < BLD; ++j) {
    const int s = j * 256 + tid;
    if constexpr (NN) {  // [64 k][BN]: rows of BN/8 chunks, transposed-read swizzle
      constexpr int CPR = BN / 8;
      const int row = s / CPR, ch = s % CPR;
      const int lc = BN == 128 ? (ch ^ sw_tr256(row)) : (ch ^ sw_tr128(row));
      b_ptr[j] = a.B + static_cast<int64_t>(row) * a.ldb + n0 + lc * 8;
    } else {
      const int row = s >> 3, lc = (s & 7) ^ sw_rd128(row);
      b_ptr[j] = n0 + row < a.N ? a.B + static_cast<int64_t>(n0 + row) * a.ldb + lc * 8 : nullptr;
    }
  }
  auto issue = [&](int stage, int kt) __attribute__((always_inline)) {
    unsigned char* base = smem + stage * Cfg::STAGE + wid * 1024;
    if constexpr (IMP) {
      const int k0 = kt * GK, tap = k0 / a.imp_C, c0 = k0 - tap * a.imp_C;
      const int r = tap / a.imp_R, t = tap - r * a.imp_R;
#pragma unroll
      for (int i = 0; i < ALD; ++i) {
        const int ih = imp_h0[i] + r, iw = imp_w0[i] + t;
        const bool ok = a_ptr[i] != nullptr && ih >= 0 && ih < a.imp_H && iw >= 0 && iw < a.imp_W;
        mm_glds16(ok ? a_ptr[i] + (static_cast<int64_t>(ih) * a.imp_W + iw) * a.lda + c0 : zero, base + i * 4096);
      }
    } else {
#pragma unroll
      for (int i = 0; i < ALD; ++i) mm_glds16(a_ptr[i] != nullptr ? a_ptr[i] + kt * GK : zero, base + i * 4096);
    }
#pragma unroll
    for (int j = 0; j < BLD; ++j) {
      const uint16_t* src = NN ? b_ptr[j] + static_cast<int64_t>(kt) * GK * a.ldb
                               : (b_ptr[j] != nullptr ? b_ptr[j] + kt * GK : zero);
      mm_glds16(src, base + Cfg::A_BYTES + j * 4096);
    }
  };

  // fragment offsets (bytes inside a stage)
  int offA[4][2];
#pragma unroll
  for (int kk = 0; kk < 4; ++kk)
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) {
      const int row = wr * 64 + mi * 32 + lr, chk = 2 * kk + hi;
      offA[kk][mi] = row * 128 + ((chk ^ sw_rd128(row)) << 4);
    }
  int offB[4][NI];   // NT
  int toB[NI][2];    // NN: transposed reads, +kk*16 rows
#pragma unroll
  for (int ni = 0; ni < NI; ++ni) {
    if constexpr (NN) {
      if constexpr (BN == 128) tr_offsets<256>(wc * (BN / 2) + ni * 32, lane, toB[ni]);
      else tr_offsets<128>(wc * (BN / 2) + ni * 32, lane, toB[ni]);
    } else {
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const int row = wc * (BN / 2) + ni * 32 + lr, chk = 2 * kk + hi;
        offB[kk][ni] = row * 128 + ((chk ^ sw_rd128(row)) << 4);
      }
    }
  }
  constexpr int BROW = BN * 2;  // NN image row bytes

  f32x16_t acc[2][NI];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[mi][ni][e] = 0.f;

  if (KT > 0) issue(0, 0);
  for (int kt = 0; kt < KT; ++kt) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt + 1 < KT) issue((kt + 1) & 1, kt + 1);
    const unsigned char* sA = smem + (kt & 1) * Cfg::STAGE;
    const unsigned char* sB = sA + Cfg::A_BYTES;
    bf16x8_t af[2][2], bfr[2][NI];
    auto load = [&](int kk, int buf) __attribute__((always_inline)) {
#pragma unroll
      for (int mi = 0; mi < 2; ++mi) af[buf][mi] = *reinterpret_cast<const bf16x8_t*>(sA + offA[kk][mi]);
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) {
        if constexpr (NN) {
          const int dd = kk * 16 * BROW;
          bfr[buf][ni] = tr_read(sB + toB[ni][0] + dd, sB + toB[ni][1] + dd);
        } else {
          bfr[buf][ni] = *reinterpret_cast<const bf16x8_t*>(sB + offB[kk][ni]);
        }
      }
    };
    load(0, 0);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int cur = kk & 1;
      if (kk + 1 < 4) load(kk + 1, cur ^ 1);
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[cur][mi], bfr[cur][ni], acc[mi][ni], 0, 0, 0);
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  // ---- epilogue: fp32 tile through LDS -> bias / beta / act -> 16-byte rows
  float* ct = reinterpret_cast<float*>(smem);
  constexpr int LD = Cfg::LD;
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = wr * 64 + mi * 32 + (e & 3) + 8 * (e >> 2) + 4 * hi;
        ct[row * LD + wc * (BN / 2) + ni * 32 + lr] = acc[mi][ni][e];
      }
  __syncthreads();
  constexpr int CPR = BN / 8;
  // batch-norm moments of the stored (bf16-rounded) tile (GemmArgs::stats),
  // accumulated in registers by the store loop: this thread's 8 columns
  // (cc = tid % CPR is fixed) over its rows, shifted by the tile's first row
  // (sums of x - K and (x - K)^2), split at a group boundary inside the tile
  constexpr bool kStatsOk = ST && !F32 && ACT == 0;
  const bool st_on = kStatsOk && a.stats != nullptr;
  const int rend = min(Cfg::BM, a.M - m0);
  int rb = rend;
  float K8[8], s1a[8], s2a[8], s1b[8], s2b[8];
  if (st_on) {
    const int g0 = m0 / a.stats_mg;
    rb = min(rend, (g0 + 1) * a.stats_mg - m0);
    const int c8 = (tid % CPR) * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      K8[j] = bf2f(pack_bf16(ct[c8 + j], 0.f) & 0xffffu);
      s1a[j] = s2a[j] = s1b[j] = s2b[j] = 0.f;
    }
  }
  for (int e = tid; e < Cfg::BM * CPR; e += 256) {
    const int row = e / CPR, cc = e - row * CPR, m = m0 + row;
    const int n = n0 + cc * 8;
    if (m >= a.M || n >= a.N) continue;  // (a chunk straddling N fills C's row padding)
    const float4 lo = *reinterpret_cast<const float4*>(ct + row * LD + cc * 8);
    const float4 up = *reinterpret_cast<const float4*>(ct + row * LD + cc * 8 + 4);
    float v[8] = {lo.x, lo.y, lo.z, lo.w, up.x, up.y, up.z, up.w};
    add_bias(a, n, v);
    const int64_t o = static_cast<int64_t>(m) * a.ldc + n;
    if constexpr (F32) {
      float* c = reinterpret_cast<float*>(a.C) + o;
      if (a.beta != 0.f) {
        const float4 c0 = *reinterpret_cast<const float4*>(c), c1 = *reinterpret_cast<const float4*>(c + 4);
        v[0] += a.beta * c0.x; v[1] += a.beta * c0.y; v[2] += a.beta * c0.z; v[3] += a.beta * c0.w;
        v[4] += a.beta * c1.x; v[5] += a.beta * c1.y; v[6] += a.beta * c1.z; v[7] += a.beta * c1.w;
      }
      *reinterpret_cast<float4*>(c) = make_float4(v[0], v[1], v[2], v[3]);
      *reinterpret_cast<float4*>(c + 4) = make_float4(v[4], v[5], v[6], v[7]);
    } else {
      uint16_t* c = reinterpret_cast<uint16_t*>(a.C) + o;
      if (a.beta != 0.f) {
        const v4u old = *reinterpret_cast<const v4u*>(c);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] += a.beta * bf2f((old[j >> 1] >> (16 * (j & 1))) & 0xffffu);
      }
      if constexpr (ACT == 1) {  // tanh-GELU; the pre-activation goes to C2
        v4u pre;
#pragma unroll
        for (int j = 0; j < 4; ++j) pre[j] = pack_bf16(v[2 * j], v[2 * j + 1]);
        *reinterpret_cast<v4u*>(reinterpret_cast<uint16_t*>(a.C2) + o) = pre;
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = gelu_tanh(bf2f((pre[j >> 1] >> (16 * (j & 1))) & 0xffffu));
      }
      v4u out;
#pragma unroll
      for (int j = 0; j < 4; ++j) out[j] = pack_bf16(v[2 * j], v[2 * j + 1]);
      *reinterpret_cast<v4u*>(c) = out;
      if (kStatsOk && st_on) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = bf2f((out[j >> 1] >> (16 * (j & 1))) & 0xffffu) - K8[j];
          if (row < rb) { s1a[j] += d; s2a[j] = fmaf(d, d, s2a[j]); }
          else { s1b[j] += d; s2b[j] = fmaf(d, d, s2b[j]); }
        }
      }
    }
  }
  if constexpr (kStatsOk) {
    if (st_on) {
      // fixed-order combine of the RG row groups through LDS (the tile is no
      // longer needed), then mean = K + S1/n, M2 = S2 - S1^2/n per slot
      static_assert(Cfg::BM == kBnStatTile, "statistics tile rows");
      constexpr int RG = 256 / CPR;
      static_assert(RG * 4 * BN + BN <= Cfg::BM * Cfg::LD, "statistics scratch fits the tile");
      __syncthreads();
      const int rg = tid / CPR, c8 = (tid % CPR) * 8;
      float* red = ct;                  // [RG][4][BN]: S1a, S2a, S1b, S2b
      float* kk = ct + RG * 4 * BN;     // [BN]
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        red[(rg * 4 + 0) * BN + c8 + j] = s1a[j];
        red[(rg * 4 + 1) * BN + c8 + j] = s2a[j];
        red[(rg * 4 + 2) * BN + c8 + j] = s1b[j];
        red[(rg * 4 + 3) * BN + c8 + j] = s2b[j];
        if (rg == 0) kk[c8 + j] = K8[j];
      }
      __syncthreads();
      if (tid < BN) {
        float t[4] = {0.f, 0.f, 0.f, 0.f};
        for (int q = 0; q < RG; ++q)
#pragma unroll
          for (int u = 0; u < 4; ++u) t[u] += red[(q * 4 + u) * BN + tid];
        const float k0 = kk[tid];
        const float na = static_cast<float>(rb), nb = static_cast<float>(rend - rb);
        float* o = a.stats + static_cast<int64_t>(m0 / Cfg::BM) * 4 * a.N + n0 + tid;
        o[0] = na > 0.f ? k0 + t[0] / na : 0.f;
        o[a.N] = na > 0.f ? fmaxf(t[1] - t[0] * t[0] / na, 0.f) : 0.f;
        o[2 * a.N] = nb > 0.f ? k0 + t[2] / nb : 0.f;
        o[3 * a.N] = nb > 0.f ? fmaxf(t[3] - t[2] * t[2] / nb, 0.f) : 0.f;
      }
    }
  }
}

template <int BN, bool NN, int ACT, bool F32, bool ST = false, bool IMP = false>
void launch_gemm_t(const GemmArgs& a, hipStream_t stream) {
  constexpr int lds = MmCfg<BN, NN>::LDS;
  static bool init = false;
  if (!init) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_kernel<BN, NN, ACT, F32, ST, IMP>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    init = true;
  }
  const int tiles = ((a.M + 127) / 128) * ((a.N + BN - 1) / BN) * (a.G > 1 ? a.G : 1);
  COMMEFF_LAUNCH((gemm_kernel<BN, NN, ACT, F32, ST, IMP>), dim3(tiles), dim3(256), lds, stream, a);
}

// split-K NN (mm_nn_splitk): out bf16 [M, N] = sum over the S fp32 partial
// products part [S][M][N] in split order + the K tail [k0, k1) that no split
// covered (the tied LM head's dh: K = 50,257 = 16 splits of 49 K-steps + 81
// rows), one 8-column chunk per thread, fixed order: deterministic
__global__ void __launch_bounds__(256) splitk_tail_kernel(const float* __restrict__ part, int S, int M, int N,
                                                          const uint16_t* __restrict__ A, int64_t lda,
                                                          const uint16_t* __restrict__ B, int64_t ldb, int k0,
                                                          int k1, uint16_t* __restrict__ out, int64_t ldo) {
  const int n8 = N / 8;
  const int64_t q = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (q >= static_cast<int64_t>(M) * n8) return;
  const int m = static_cast<int>(q / n8), c = static_cast<int>(q - static_cast<int64_t>(m) * n8) * 8;
  float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < S; ++s) {
    const float* p = part + (static_cast<int64_t>(s) * M + m) * N + c;
    const float4 lo = *reinterpret_cast<const float4*>(p), hi = *reinterpret_cast<const float4*>(p + 4);
    v[0] += lo.x; v[1] += lo.y; v[2] += lo.z; v[3] += lo.w;
    v[4] += hi.x; v[5] += hi.y; v[6] += hi.z; v[7] += hi.w;
  }
  const uint16_t* ar = A + static_cast<int64_t>(m) * lda;
  for (int k = k0; k < k1; ++k) {
    const float av = bf2f(ar[k]);
    const v4u bv = *reinterpret_cast<const v4u*>(B + static_cast<int64_t>(k) * ldb + c);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = fmaf(av, bf2f((bv[j >> 1] >> (16 * (j & 1))) & 0xffffu), v[j]);
  }
  v4u o;
#pragma unroll
  for (int j = 0; j < 4; ++j) o[j] = pack_bf16(v[2 * j], v[2 * j + 1]);
  *reinterpret_cast<v4u*>(out + static_cast<int64_t>(m) * ldo + c) = o;
}

}  // namespace

void launch_splitk_tail(const float* part, int S, int M, int N, const uint16_t* A, int64_t lda, const uint16_t* B,
                        int64_t ldb, int k0, int k1, uint16_t* out, int64_t ldo, hipStream_t stream) {
  const int64_t n = static_cast<int64_t>(M) * (N / 8);
  if (n == 0) return;
  COMMEFF_LAUNCH(splitk_tail_kernel, dim3(static_cast<uint32_t>((n + 255) / 256)), dim3(256), 0, stream, part, S,
                 M, N, A, lda, B, ldb, k0, k1, out, ldo);
}

bool gemm_supported(int M, int N, int K, bool nn) {
  (void)nn;
  return M >= 1 && N >= 64 && N % 64 == 0 && K >= 64 && K % 64 == 0;
}

// NT with any N >= 64 (C's rows padded to a multiple of 8 columns; no bias /
// activation / statistics on this path)
bool gemm_supported_nedge(int M, int N, int K) { return M >= 1 && N >= 64 && K >= 64 && K % 64 == 0; }

void launch_gemm(const GemmArgs& a, bool nn, int act, bool f32, hipStream_t stream) {
  if (a.M <= 0) return;
  // (256-row tiles with a 4-stage ring, one block per CU, measured equal or
  // slower on the GPT-2 and ResNet-101 shapes: these GEMMs are one wave of
  // tiles whose load / store phases set the time; profiles/r4_experiments.md)
  // 128-wide column tiles when they still give ~every resident slot (2 per CU) a block
  const bool wide = (a.N % 128 == 0 || (!nn && a.N % 64 != 0)) &&
                    static_cast<int64_t>((a.M + 127) / 128) * ((a.N + 127) / 128) * (a.G > 1 ? a.G : 1) >= 384;
  if (a.imp_C > 0) {  // implicit column image A (NT, bf16 out, no activation)
    if (a.stats != nullptr) {  // + BN moments (conv_nt_imp)
      if (wide) launch_gemm_t<128, false, 0, false, true, true>(a, stream);
      else launch_gemm_t<64, false, 0, false, true, true>(a, stream);
      return;
    }
    if (wide) launch_gemm_t<128, false, 0, false, false, true>(a, stream);
    else launch_gemm_t<64, false, 0, false, false, true>(a, stream);
    return;
  }
  if (a.stats != nullptr && !nn && act == 0 && !f32) {  // BN moments in the epilogue (mm_nt_bnstats)
    if (wide) launch_gemm_t<128, false, 0, false, true>(a, stream);
    else launch_gemm_t<64, false, 0, false, true>(a, stream);
    return;
  }
  if (act == 1) {
    if (wide) { if (nn) launch_gemm_t<128, true, 1, false>(a, stream); else launch_gemm_t<128, false, 1, false>(a, stream); }
    else { if (nn) launch_gemm_t<64, true, 1, false>(a, stream); else launch_gemm_t<64, false, 1, false>(a, stream); }
    return;
  }
  if (f32) {
    if (wide) { if (nn) launch_gemm_t<128, true, 0, true>(a, stream); else launch_gemm_t<128, false, 0, true>(a, stream); }
    else { if (nn) launch_gemm_t<64, true, 0, true>(a, stream); else launch_gemm_t<64, false, 0, true>(a, stream); }
    return;
  }
  if (wide) { if (nn) launch_gemm_t<128, true, 0, false>(a, stream); else launch_gemm_t<128, false, 0, false>(a, stream); }
  else { if (nn) launch_gemm_t<64, true, 0, false>(a, stream); else launch_gemm_t<64, false, 0, false>(a, stream); }
}

}  // namespace commeff
