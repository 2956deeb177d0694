// Weight-gradient GEMM for the GPT-2 linears: C[M][N] (fp32) += A^T B with
// A [T][M] and B [T][N] bf16 row-major -- dW[in][out] += sum over the round's
// token rows t of X[t][in] dY[t][out] (HF Conv1D layout), accumulated straight
// into the flat fp32 gradient (ops/transformer.py grad sinks).
//
// Reference model: the GPT2DoubleHeadsModel backward of
// /root/reference/CommEfficient/gpt2_train.py:55-99.
// hipBLASLt runs these shapes (768 x 768 .. 3072 x 768 over ~10k tokens) at
// 144-421 TF/s: 9-36 output tiles of 256 x 256 cannot fill 256 CUs.  Here:
//   * the reduction runs over the ROW index of both operands, so both tiles
//     are staged K-major by LDS DMA (global_load_lds, 16 bytes a lane) into
//     XOR-swizzled [64 tokens][256] images and read with the gfx950
//     transposing read ds_read_b64_tr_b16 in the 32x32x16 operand layout
//     (the same images and reads as conv.hip's wide wgrad kernel);
//   * 256 x 256 tile per 8-wave block (4 x 2 waves of 64 x 128), 64-token
//     K-steps through a two-stage ring, one block per CU (128 KB LDS);
//   * split-K over tokens so tiles x splits ~ one block per CU; each split
//     writes its fp32 partial tile to a slab and a second kernel adds the
//     slabs to C in a fixed order (bitwise deterministic); one split
//     accumulates into C directly.
#include <hip/hip_runtime.h>
#include <cstdint>
#include "kernels.h"
#include "conv_common.h"

namespace commeff {
namespace {

constexpr int GBK = 64;                    // tokens per K-step
constexpr int GHALF = GBK * 128 * 2;       // one [64][128] bf16 image (16 KB)
constexpr int GSTAGE = 4 * GHALF;          // A (2 halves) + B (2 halves)
constexpr int kGemmLds = 2 * GSTAGE;       // two stages: 128 KB

__device__ __attribute__((aligned(16))) uint32_t g_gemm_zero[4] = {0u, 0u, 0u, 0u};

__device__ __forceinline__ void gl16(const void* src, unsigned char* lds) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

// SMALL: a 128 x 128 tile per 4-wave block (2 x 2 waves of 64 x 64, one
// [64][128] image per operand, 64 KB of LDS: two blocks per CU) for the
// narrow weight gradients -- the ResNet-101 64 / 128-channel layers and the
// 7x7 stem's [64 x 152] product -- whose 256 x 256 tiles would be mostly
// padding; split-K over the (large) token / pixel count fills the chip.
template <bool SMALL>
__global__ void __launch_bounds__(SMALL ? 256 : 512) gemm_tn_acc_kernel(GemmTnArgs a) {
  constexpr int NTH = SMALL ? 256 : 512, TILE = SMALL ? 128 : 256, NH = SMALL ? 1 : 2;
  constexpr int NI = SMALL ? 2 : 4, WN = SMALL ? 64 : 128;  // wave tile: 64 x WN
  constexpr int STG = 2 * NH * GHALF;                        // A + B images of one stage
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  // M, N multiples of 8: a partial edge tile loads zeros past M / N and
  // stores only its valid part
  const int ntn = (a.N + TILE - 1) / TILE;
  const int ntiles = ((a.M + TILE - 1) / TILE) * ntn;
  const int per_g = ntiles * a.splits;
  const int grp = bid / per_g, rem = bid - grp * per_g;
  const int tile = rem % ntiles, split = rem / ntiles;
  const int m0 = (tile / ntn) * TILE, n0 = (tile % ntn) * TILE;
  const int pbeg = split * a.steps_per_split * GBK;
  const int pend = min(a.T, pbeg + a.steps_per_split * GBK);
  // group grp: its own T operand rows and its own C (grouped weight gradients)
  // (sa / sb: the channel-stacked clients of parallel/fedavg_native.py share
  // the token rows, each its column block)
  const uint16_t* __restrict__ gA = a.A + grp * (a.sa >= 0 ? a.sa : static_cast<int64_t>(a.T) * a.lda);
  const uint16_t* __restrict__ gB = a.B + grp * (a.sb >= 0 ? a.sb : static_cast<int64_t>(a.T) * a.ldb);
  const int nsteps = pend > pbeg ? (pend - pbeg + GBK - 1) / GBK : 0;
  const uint64_t zero = reinterpret_cast<uint64_t>(g_gemm_zero);

  // piece i (0..3) of this thread: image half h, chunk slot sp of the half
  uint64_t a_ptr[4], b_ptr[4];
  int p_row[4];
  bool a_in[4], b_in[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int h = SMALL ? 0 : i >> 1, sp = SMALL ? i * NTH + tid : (i & 1) * 512 + tid;
    const int row = sp >> 4, lc = (sp & 15) ^ sw_tr256(row);
    p_row[i] = pbeg + row;
    a_in[i] = m0 + h * 128 + lc * 8 < a.M;
    b_in[i] = n0 + h * 128 + lc * 8 < a.N;
    a_ptr[i] = reinterpret_cast<uint64_t>(gA + static_cast<int64_t>(pbeg + row) * a.lda + m0 + h * 128 + lc * 8);
    b_ptr[i] = reinterpret_cast<uint64_t>(gB + static_cast<int64_t>(pbeg + row) * a.ldb + n0 + h * 128 + lc * 8);
  }
  // implicit column image: the chunk's tap (fixed: imp_C % 8 == 0) and its
  // channel offset; the pixel shift is applied per step
  int imp_dr[4], imp_dc[4], imp_co[4];
  if (a.imp_C > 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int h = SMALL ? 0 : i >> 1, sp = SMALL ? i * NTH + tid : (i & 1) * 512 + tid;
      const int row = sp >> 4, lc = (sp & 15) ^ sw_tr256(row);
      const int j = n0 + h * 128 + lc * 8, tap = j / a.imp_C;
      imp_dr[i] = tap / a.imp_R;  // kernel row / column of the tap
      imp_dc[i] = tap % a.imp_R;
      imp_co[i] = j - tap * a.imp_C;
    }
  }
  auto issue = [&](int stage) __attribute__((always_inline)) {
    unsigned char* base = smem + stage * STG + wid * 1024;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bool ok = p_row[i] < pend;  // token rows past the split: zero page
      // (lane-linear LDS destination of the wave's 64 chunks of slot sp)
      const int dst = SMALL ? i * NTH * 16 : (i >> 1) * GHALF + (i & 1) * 8192;
      gl16(reinterpret_cast<const void*>(ok && a_in[i] ? a_ptr[i] : zero), base + dst);
      uint64_t bp = b_ptr[i];
      bool bok = ok && b_in[i];
      if (a.imp_C > 0) {
        // output pixel p -> input pixel (n, oh s - pad + r, ow s - pad + t)
        const int OH = a.imp_OH > 0 ? a.imp_OH : a.imp_H, OW = a.imp_OW > 0 ? a.imp_OW : a.imp_W;
        const int p = p_row[i], ohw = OH * OW;
        const int n = p / ohw, rem = p - n * ohw, oh = rem / OW, ow = rem - oh * OW;
        const int hh = oh * a.imp_s - a.imp_pad + imp_dr[i], ww = ow * a.imp_s - a.imp_pad + imp_dc[i];
        bok = bok && hh >= 0 && hh < a.imp_H && ww >= 0 && ww < a.imp_W;
        bp = reinterpret_cast<uint64_t>(
            gB + (static_cast<int64_t>(n) * a.imp_H * a.imp_W + static_cast<int64_t>(hh) * a.imp_W + ww) * a.ldb +
            imp_co[i]);
      }
      gl16(reinterpret_cast<const void*>(bok ? bp : zero), base + NH * GHALF + dst);
      p_row[i] += GBK;
      a_ptr[i] += static_cast<uint64_t>(GBK) * a.lda * 2;
      b_ptr[i] += static_cast<uint64_t>(GBK) * a.ldb * 2;
    }
  };

  f32x16_t acc[2][NI];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[mi][ni][e] = 0.f;

  if (nsteps > 0) issue(0);
  // transposed-read offsets: A columns m = wr*64 + mi*32 (half wr >> 1 of the
  // big tile), B columns wc*WN + ni*32 (half wc of the big tile)
  int toA[2][2], toB[NI][2];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi) {
    tr_offsets<256>((SMALL ? wr : (wr & 1)) * 64 + mi * 32, lane, toA[mi]);
    toA[mi][0] += (SMALL ? 0 : (wr >> 1)) * GHALF;
    toA[mi][1] += (SMALL ? 0 : (wr >> 1)) * GHALF;
  }
#pragma unroll
  for (int ni = 0; ni < NI; ++ni) {
    tr_offsets<256>((SMALL ? wc * 64 : 0) + ni * 32, lane, toB[ni]);
    toB[ni][0] += NH * GHALF + (SMALL ? 0 : wc) * GHALF;
    toB[ni][1] += NH * GHALF + (SMALL ? 0 : wc) * GHALF;
  }
  int rd = 0;
  for (int st = 0; st < nsteps; ++st) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (st + 1 < nsteps) issue(rd ^ 1);
    const unsigned char* sb = smem + rd * STG;
    bf16x8_t af[2][2], bfr[2][NI];
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) af[0][mi] = tr_read(sb + toA[mi][0], sb + toA[mi][1]);
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) bfr[0][ni] = tr_read(sb + toB[ni][0], sb + toB[ni][1]);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int cur = kk & 1, nxt = cur ^ 1;
      if (kk + 1 < 4) {
        const int dd = (kk + 1) * 16 * 256;
#pragma unroll
        for (int mi = 0; mi < 2; ++mi) af[nxt][mi] = tr_read(sb + toA[mi][0] + dd, sb + toA[mi][1] + dd);
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) bfr[nxt][ni] = tr_read(sb + toB[ni][0] + dd, sb + toB[ni][1] + dd);
      }
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[cur][mi], bfr[cur][ni], acc[mi][ni], 0, 0, 0);
    }
    rd ^= 1;
  }

  const bool direct = a.splits == 1 && !a.slab_only;
  if (SMALL && direct && a.stage) {
    // the 128 x 128 fp32 tile through the (drained) LDS ring, then streamed
    // row-wise: a wave reads / writes two 512-byte rows of C per instruction
    // (16 bytes a lane) and 256-byte rows of the mirror -- the MFMA layout
    // stores 128-byte pieces 4 bytes a lane, with 2-byte mirror stores
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
    float* tl = reinterpret_cast<float*>(smem);
    {
      const int hi = lane >> 5, lr = lane & 31;
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni)
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int r = wr * 64 + mi * 32 + (e & 3) + 8 * (e >> 2) + 4 * hi;
            tl[r * 128 + wc * WN + ni * 32 + lr] = acc[mi][ni][e];
          }
    }
    __syncthreads();
    float* cb = a.C + static_cast<int64_t>(grp) * a.cg;
    uint16_t* mb = a.mirror != nullptr ? a.mirror + static_cast<int64_t>(grp) * a.mcg : nullptr;
    const bool plain = a.beta == 1.f && a.alpha == 1.f, rdc = plain || a.beta != 0.f;
    const float* sb = a.src != nullptr ? a.src + static_cast<int64_t>(grp) * a.scg : cb;
    const int c4 = tid & 31, r0 = tid >> 5;  // 8 rows per pass, 16 passes
    const int n = n0 + c4 * 4;
#pragma unroll
    for (int pb = 0; pb < 16; pb += 8) {
      float4 o[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int m = m0 + (pb + q) * 8 + r0;
        o[q] = rdc && m < a.M && n < a.N ? *reinterpret_cast<const float4*>(sb + static_cast<int64_t>(m) * a.ldc + n)
                                         : float4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int r = (pb + q) * 8 + r0, m = m0 + r;
        if (m >= a.M || n >= a.N) continue;
        const float4 t = *reinterpret_cast<const float4*>(tl + r * 128 + c4 * 4);
        float4 v;
        if (plain) {
          v = float4{o[q].x + t.x, o[q].y + t.y, o[q].z + t.z, o[q].w + t.w};
        } else {
          v = float4{a.beta * o[q].x + a.alpha * t.x, a.beta * o[q].y + a.alpha * t.y,
                     a.beta * o[q].z + a.alpha * t.z, a.beta * o[q].w + a.alpha * t.w};
        }
        typedef float f4v __attribute__((ext_vector_type(4)));
        typedef uint32_t u2v __attribute__((ext_vector_type(2)));
        f4v* cp = reinterpret_cast<f4v*>(cb + static_cast<int64_t>(m) * a.ldc + n);
        const f4v vv = {v.x, v.y, v.z, v.w};
        if (a.nt) __builtin_nontemporal_store(vv, cp); else *cp = vv;
        if (mb != nullptr) {
          const u2v h = {pack_bf16(v.x, v.y), pack_bf16(v.z, v.w)};
          u2v* mp = reinterpret_cast<u2v*>(mb + static_cast<int64_t>(m) * a.ldc + n);
          if (a.nt) __builtin_nontemporal_store(h, mp); else *mp = h;
        }
      }
    }
    return;
  }
  // C row m (lanes: 32 consecutive n) -- one split: accumulate into C; else
  // this split's slab [M][N]
  const int hi = lane >> 5, lr = lane & 31;
  float* out = direct ? a.C + static_cast<int64_t>(grp) * a.cg
                      : a.slab + static_cast<size_t>(grp * a.splits + split) * a.M * a.N;
  const int64_t ld = direct ? a.ldc : a.N;
  // direct + mirror: the fused SGD step of the FedAvg engine (C = the weight
  // rows, beta = 1 - lr wd, alpha = -lr) and the rows' bf16 copy, written here
  // instead of by a cast pass re-reading C
  uint16_t* mir = direct && a.mirror != nullptr ? a.mirror + static_cast<int64_t>(grp) * a.mcg : nullptr;
  const bool plain = a.beta == 1.f && a.alpha == 1.f;
  const bool rdc = direct && (plain || a.beta != 0.f);
  const float* src = direct && a.src != nullptr ? a.src + static_cast<int64_t>(grp) * a.scg : out;
  if (!direct) {  // a split's slab: plain stores
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) {
        const int n = n0 + wc * WN + ni * 32 + lr;
        if (n >= a.N || m0 + wr * 64 + mi * 32 >= a.M) continue;  // padding of an edge tile
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int m = m0 + wr * 64 + mi * 32 + (e & 3) + 8 * (e >> 2) + 4 * hi;
          if (m >= a.M) continue;  // M not a multiple of 32 (the LM head's vocabulary)
          out[static_cast<int64_t>(m) * ld + n] = acc[mi][ni][e];
        }
      }
    return;
  }
  // (batches of NB column blocks: 32 more registers in the 256 x 256 variant
  // -- all NI of them spilled)
  constexpr int NB = SMALL ? NI : 2;
#pragma unroll
  for (int mi = 0; mi < 2; ++mi) {
    if (m0 + wr * 64 + mi * 32 >= a.M) continue;  // padding of an edge tile
#pragma unroll
    for (int nb = 0; nb < NI; nb += NB) {
      // every C value of this batch loaded before its first store: the mirror
      // (another base) may alias C as far as the compiler knows, and
      // interleaved load / store pairs ran one HBM round trip at a time (378 us
      // per FedAvg layer-3 weight update)
      float old[NB][16];
#pragma unroll
      for (int q = 0; q < NB; ++q) {
        const int n = n0 + wc * WN + (nb + q) * 32 + lr;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int m = m0 + wr * 64 + mi * 32 + (e & 3) + 8 * (e >> 2) + 4 * hi;
          old[q][e] = rdc && n < a.N && m < a.M ? src[static_cast<int64_t>(m) * ld + n] : 0.f;
        }
      }
#pragma unroll
      for (int q = 0; q < NB; ++q) {
        const int n = n0 + wc * WN + (nb + q) * 32 + lr;
        if (n >= a.N) continue;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int m = m0 + wr * 64 + mi * 32 + (e & 3) + 8 * (e >> 2) + 4 * hi;
          if (m >= a.M) continue;  // M not a multiple of 32 (the LM head's vocabulary)
          const float c = acc[mi][nb + q][e];
          const float v = plain ? old[q][e] + c : a.beta * old[q][e] + a.alpha * c;
          out[static_cast<int64_t>(m) * ld + n] = v;
          if (mir != nullptr) mir[static_cast<int64_t>(m) * ld + n] = static_cast<uint16_t>(pack_bf16(v, 0.f));
        }
      }
    }
  }
}

// C_g[m][n] += sum over s of slab[g][s][m][n], s in order (float4 per thread)
__global__ void __launch_bounds__(256) gemm_tn_reduce_kernel(float* __restrict__ C, int64_t ldc,
                                                             const float* __restrict__ slab, int M,
                                                             int N, int splits, int G, int64_t cg,
                                                             float beta, float alpha,
                                                             uint16_t* __restrict__ mirror, int64_t mcg,
                                                             const float* __restrict__ src, int64_t scg) {
  const int64_t plane = static_cast<int64_t>(M) * N;
  const int64_t n4 = G * plane / 4;
  for (int64_t q = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; q < n4;
       q += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t eg = q * 4;
    const int g = static_cast<int>(eg / plane);
    const int64_t e = eg - g * plane;
    const int m = static_cast<int>(e / N), n = static_cast<int>(e - static_cast<int64_t>(m) * N);
    const float* sg = slab + static_cast<int64_t>(g) * splits * plane + e;
    float4 s = *reinterpret_cast<const float4*>(sg);
    for (int k = 1; k < splits; ++k) {
      const float4 v = *reinterpret_cast<const float4*>(sg + k * plane);
      s.x += v.x;
      s.y += v.y;
      s.z += v.z;
      s.w += v.w;
    }
    float4* c = reinterpret_cast<float4*>(C + g * cg + static_cast<int64_t>(m) * ldc + n);
    // (src: beta scales those rows instead of C's -- the FedAvg engine's first
    // local step reads the server row)
    float4 cv = src != nullptr && !(beta == 1.f && alpha == 1.f)
                    ? *reinterpret_cast<const float4*>(src + g * scg + static_cast<int64_t>(m) * ldc + n)
                    : *c;
    if (beta == 1.f && alpha == 1.f) {
      cv.x += s.x;
      cv.y += s.y;
      cv.z += s.z;
      cv.w += s.w;
    } else {
      cv.x = (beta != 0.f ? beta * cv.x : 0.f) + alpha * s.x;
      cv.y = (beta != 0.f ? beta * cv.y : 0.f) + alpha * s.y;
      cv.z = (beta != 0.f ? beta * cv.z : 0.f) + alpha * s.z;
      cv.w = (beta != 0.f ? beta * cv.w : 0.f) + alpha * s.w;
    }
    *c = cv;
    if (mirror != nullptr) {
      uint32_t* mp = reinterpret_cast<uint32_t*>(mirror + g * mcg + static_cast<int64_t>(m) * ldc + n);
      mp[0] = pack_bf16(cv.x, cv.y);
      mp[1] = pack_bf16(cv.z, cv.w);
    }
  }
}

}  // namespace

static bool tn_small(int M, int N, int force = -1) { return force >= 0 ? force != 0 : M % 256 != 0 || N % 256 != 0; }

int gemm_tn_splits(int M, int N, int T, int cus, int small) {
  // (small tiles: two blocks per CU)
  const int t = tn_small(M, N, small) ? 128 : 256;
  if (t == 128) cus *= 2;
  const int tiles = ((M + t - 1) / t) * ((N + t - 1) / t);
  const int steps = (T + GBK - 1) / GBK;
  // at most one block per resident slot: tiles x splits past the slot count
  // leaves a second, nearly empty wave of blocks that costs a whole block time
  // (GPT-2's 27 / 9 / 36-tile shapes ran 261-288 blocks on 256 CUs)
  int s = cus / tiles;
  const int max_s = steps / 4 > 0 ? steps / 4 : 1;  // >= 4 K-steps per split
  if (s > max_s) s = max_s;
  if (s < 1) s = 1;
  return s;
}

void launch_gemm_tn_acc(GemmTnArgs a, hipStream_t stream) {
  if (a.M == 0 || a.N == 0 || a.T == 0) return;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_tn_acc_kernel<false>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, kGemmLds);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_tn_acc_kernel<true>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, kGemmLds / 2);
    attr = true;
  }
  const int steps = (a.T + GBK - 1) / GBK;
  a.steps_per_split = (steps + a.splits - 1) / a.splits;
  const bool small = tn_small(a.M, a.N, a.small);
  const int t = small ? 128 : 256;
  const int tiles = ((a.M + t - 1) / t) * ((a.N + t - 1) / t);
  if (a.G < 1) a.G = 1;
  if (small)
    COMMEFF_LAUNCH(gemm_tn_acc_kernel<true>, dim3(static_cast<uint32_t>(tiles * a.splits * a.G)), dim3(256),
                   kGemmLds / 2, stream, a);
  else
    COMMEFF_LAUNCH(gemm_tn_acc_kernel<false>, dim3(static_cast<uint32_t>(tiles * a.splits * a.G)), dim3(512),
                   kGemmLds, stream, a);
  if (a.splits > 1 && !a.slab_only) {
    const int64_t n4 = static_cast<int64_t>(a.G) * a.M * a.N / 4;
    int64_t blocks = (n4 + 255) / 256;
    if (blocks > 2048) blocks = 2048;
    COMMEFF_LAUNCH(gemm_tn_reduce_kernel, dim3(static_cast<uint32_t>(blocks)), dim3(256), 0, stream,
                       a.C, a.ldc, a.slab, a.M, a.N, a.splits, a.G, a.cg, a.beta, a.alpha, a.mirror, a.mcg,
                       a.src, a.scg);
  }
}

}  // namespace commeff
