// 3x3 / stride 1 / pad 1 convolution for gfx950 as implicit GEMMs on the bf16
// MFMA (v_mfma_f32_32x32x16_bf16), NHWC activations, fp32 accumulation.
//
//   forward  y[p, k]  = act( sum_{r,s,c} x[p + (r-1, s-1), c] * w[k, r, s, c] )
//   dgrad    dx       = forward(dy, wt)   with wt[c, r, s, k] = w[k, 2-r, 2-s, c]
//   wgrad    dw[k, r, s, c] = sum_p dy[p, k] * x[p + (r-1, s-1), c]
//
// This replaces the conv3x3 of ResNet-9 ("the
// conv3x3 MFMA GEMM for ResNet-9"); reference model:
// /root/reference/CommEfficient/models/resnet9.py:32-59 (ConvBN).
//
// Forward / dgrad (`conv_fwd_kernel<TBM, BN, NSTAGE>`): GEMM M = pixels,
// N = output channels, K = 9*C (64 channels of one tap per K-step).  Both
// operands are K-contiguous (NHWC rows, [k][r][s][c] weight rows), so the
// TBM x BN x 64 tile goes global -> LDS with global_load_lds_dwordx4 (LDS DMA,
// no staging registers) through an NSTAGE-deep ring with one raw s_barrier
// per step, and is read back with ds_read_b128 in the 32x32x16 operand layout
// from an XOR-swizzled image (the swizzle is applied on the SOURCE side since
// the DMA writes each wave's 1 KB lane-linearly).  Padding taps and tail
// pixels load from a 16-byte zero page (an exec-masked DMA lane would leave
// stale LDS).  Per chunk, a 9-bit tap-validity mask and a base pointer are
// precomputed once, so a K-step costs ~3 VALU per 16-byte chunk.
// The epilogue stages the fp32 tile in LDS and emits 16-byte stores with
// fused ReLU, a ReLU-mask by another tensor (y = 0 where mask <= 0) and a
// residual addend (packed v_cvt_pk_bf16_f32 conversion).
//
// Wgrad (`conv_wgrad_kernel<BN, NSTAGE>`): GEMM M = out channels (128 per
// tile), N = in channels of one tap, K = pixels.  The reduction runs over the
// ROW index of both NHWC images, so the operands are read with the gfx950
// transposing LDS read ds_read_b64_tr_b16 (cdna_hip_programming.md T10) from
// XOR-swizzled images, again filled by LDS DMA.  K is split over blocks; each
// split writes an fp32 slab and a second kernel sums the slabs in a fixed
// order (deterministic) straight into PyTorch's [K][C][3][3] layout.
//
// Tile -> block mapping is XCD-aware: consecutive logical tiles (which share
// activation rows / halos in L2) are placed on the same XCD.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdlib>
#include <stdexcept>
#include "kernels.h"
#include "conv_common.h"

namespace commeff {
namespace {

constexpr int BK = 64;   // K-step (channels for fwd, pixels for wgrad)
constexpr int WBM = 128; // wgrad: out channels per tile

// 16 zero bytes: source of every padding / tail row of a DMA-staged operand
__device__ __attribute__((aligned(16))) uint32_t g_conv_zero[4] = {0u, 0u, 0u, 0u};

// (a plain device function: referenced directly from a kernel template, the
// target builtin makes the host-side instantiation fail)
__device__ __forceinline__ void glds16(const void* src, unsigned char* lds) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Epilogue shared by the conv forward kernels: the fp32 accumulator tile
// (wave (wr, wc) holds rows wr*64.., columns wc*BN/2..) through LDS, fused
// ReLU / mask / residual add or ReLU + 2x2 max-pool, 16-byte bf16 stores.
// NTE threads take part (tid in [0, NTE)); only threads with own = true hold
// accumulator fragments (the in-block split-K kernel's second half does not).
template <int TBM, int BN, bool POOL, int NTE = TBM * 2, int EPR_ = (TBM > 128 ? 128 : TBM)>
__device__ __forceinline__ void conv_fwd_epilogue(const ConvFwdArgs& a, f32x16_t (&acc)[2][BN / 64],
                                                  unsigned char* smem, int m0, int n0, int tid,
                                                  int wr, int wc, int hi, int lr, bool own = true) {
  constexpr int NT = NTE;
  constexpr int NI = BN / 64;
  // ---- epilogue: fp32 tile in LDS -> fused ops -> 16-byte bf16 stores
  // (tiles taller than EPR rows go through LDS in EPR-row passes)
  constexpr int LD = BN + 4;
  constexpr int EPR = EPR_;
  static_assert(EPR % 64 == 0 && TBM % EPR == 0, "epilogue pass rows");
  float* ct = reinterpret_cast<float*>(smem);
  constexpr int CPR = BN / 8;  // 16-byte output chunks per row
#pragma unroll 1
  for (int ps = 0; ps < TBM / EPR; ++ps) {
  if (ps > 0) __syncthreads();  // the previous pass has read ct
  if (own && (wr * 64) / EPR == ps) {
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = wr * 64 - ps * EPR + mi * 32 + (e & 3) + 8 * (e >> 2) + 4 * hi;
        const int col = wc * (BN / 2) + ni * 32 + lr;
        ct[row * LD + col] = acc[mi][ni][e];
      }
  }
  __syncthreads();
  const int mp = m0 + ps * EPR;  // first pixel of this pass
  if constexpr (POOL) {
    // fused ReLU + 2x2 max-pool (csrc/pool.hip semantics): the tile holds
    // whole image-row pairs (TBM % 2W == 0, m0 % 2W == 0), so its pooled
    // outputs are the contiguous pooled pixels [m0/4, (m0+TBM)/4).  Values are
    // compared after bf16 rounding (as the unfused path pools the stored bf16
    // conv output); code = window position of the max, 255 when max <= 0.
    const int W = a.W, OWl = W >> 1;
    const int q0 = mp >> 2;
#pragma unroll 1
    for (int e = tid; e < (EPR / 4) * CPR; e += NT) {
      const int pq = e / CPR, cc = e - pq * CPR;
      const int r2 = pq / OWl, ow = pq - r2 * OWl;
      const int row0 = 2 * r2 * W + 2 * ow;
      if (mp + row0 >= a.P) continue;
      float best[8];
      uint32_t arg[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        best[j] = -__builtin_huge_valf();
        arg[j] = 0;
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const float* src = ct + (row0 + (t >> 1) * W + (t & 1)) * LD + cc * 8;
        const float4 lo = *reinterpret_cast<const float4*>(src);
        const float4 up = *reinterpret_cast<const float4*>(src + 4);
        const uint32_t pk[4] = {pack_bf16(lo.x, lo.y), pack_bf16(lo.z, lo.w), pack_bf16(up.x, up.y),
                                pack_bf16(up.z, up.w)};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float f = bf2f((pk[j >> 1] >> (16 * (j & 1))) & 0xffffu);
          if (f > best[j]) {
            best[j] = f;
            arg[j] = static_cast<uint32_t>(t);
          }
        }
      }
      v4u out;
      uint64_t codes = 0;
#pragma unroll
      for (int j = 0; j < 8; j += 2) {
        const bool p0 = best[j] > 0.f, p1 = best[j + 1] > 0.f;
        // the maxima are bf16 values: exact upper halves
        const uint32_t h0 = p0 ? (__float_as_uint(best[j]) >> 16) : 0u;
        const uint32_t h1 = p1 ? (__float_as_uint(best[j + 1]) >> 16) : 0u;
        out[j >> 1] = h0 | (h1 << 16);
        codes |= static_cast<uint64_t>(p0 ? arg[j] : 255u) << (8 * j);
        codes |= static_cast<uint64_t>(p1 ? arg[j + 1] : 255u) << (8 * (j + 1));
      }
      const size_t o = static_cast<size_t>(q0 + pq) * a.K + n0 + cc * 8;
      *reinterpret_cast<v4u*>(a.y + o) = out;
      *reinterpret_cast<uint64_t*>(a.pool_idx + o) = codes;
    }
    continue;
  }
  const bool relu = a.relu != 0;
#pragma unroll 2
  for (int e = tid; e < EPR * CPR; e += NT) {
    const int row = e / CPR, cc = e - row * CPR;
    const int p = mp + row;
    if (p >= a.P) continue;
    const float4 lo = *reinterpret_cast<const float4*>(ct + row * LD + cc * 8);
    const float4 up = *reinterpret_cast<const float4*>(ct + row * LD + cc * 8 + 4);
    float v[8] = {lo.x, lo.y, lo.z, lo.w, up.x, up.y, up.z, up.w};
    const size_t o = static_cast<size_t>(p) * a.K + n0 + cc * 8;
    if (relu) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = fmaxf(v[j], 0.f);
    }
    if (a.mask != nullptr) {
      const v4u m = *reinterpret_cast<const v4u*>(a.mask + o);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t hb = (m[j >> 1] >> (16 * (j & 1))) & 0xffffu;
        // keep where mask > 0: sign bit clear and not +0
        v[j] = ((hb & 0x8000u) == 0u && hb != 0u) ? v[j] : 0.f;
      }
    }
    if (a.addend != nullptr) {
      if (a.y_pre != nullptr && a.unpool_idx == nullptr) {  // the activation before the residual add
        v4u pre;
        pre[0] = pack_bf16(v[0], v[1]);
        pre[1] = pack_bf16(v[2], v[3]);
        pre[2] = pack_bf16(v[4], v[5]);
        pre[3] = pack_bf16(v[6], v[7]);
        *reinterpret_cast<v4u*>(a.y_pre + o) = pre;
      }
      const v4u m = *reinterpret_cast<const v4u*>(a.addend + o);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += bf2f((m[j >> 1] >> (16 * (j & 1))) & 0xffffu);
    }
    v4u out;
    out[0] = pack_bf16(v[0], v[1]);
    out[1] = pack_bf16(v[2], v[3]);
    out[2] = pack_bf16(v[4], v[5]);
    out[3] = pack_bf16(v[6], v[7]);
    if (a.unpool_idx != nullptr) {
      // relu + max-pool backward: the value goes to its window position t
      // (code byte per channel, 255 = relu-dead), zeros to the other three
      const uint64_t codes = *reinterpret_cast<const uint64_t*>(a.unpool_idx + o);
      const uint32_t q = fdiv(static_cast<uint32_t>(p), a.div_w);
      const int ow = p - static_cast<int>(q) * a.W;
      const uint32_t n = fdiv(q, a.div_h);
      const int oh = static_cast<int>(q - n * static_cast<uint32_t>(a.H));
      const int FW = 2 * a.W;
      const size_t f0 = (static_cast<size_t>(n * 2 * a.H + 2 * oh) * FW + 2 * ow) * a.K + n0 + cc * 8;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        v4u ot;
#pragma unroll
        for (int h = 0; h < 4; ++h) {
          const uint32_t c0 = static_cast<uint32_t>(codes >> (16 * h)) & 0xffu;
          const uint32_t c1 = static_cast<uint32_t>(codes >> (16 * h + 8)) & 0xffu;
          ot[h] = (c0 == static_cast<uint32_t>(t) ? (out[h] & 0xffffu) : 0u) |
                  (c1 == static_cast<uint32_t>(t) ? (out[h] & 0xffff0000u) : 0u);
        }
        *reinterpret_cast<v4u*>(a.y + f0 + static_cast<size_t>((t >> 1) * FW + (t & 1)) * a.K) = ot;
      }
      continue;
    }
    *reinterpret_cast<v4u*>(a.y + o) = out;
    if (a.y_dual != nullptr) {
      const v4u m = *reinterpret_cast<const v4u*>(a.dual_mask + o);
      v4u od;
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        const uint32_t lo = m[h] & 0xffffu, hi = m[h] >> 16;
        // keep where mask > 0: sign bit clear and not +0 (csrc relu_mask)
        od[h] = (((lo & 0x8000u) == 0u && lo != 0u) ? (out[h] & 0xffffu) : 0u) |
                (((hi & 0x8000u) == 0u && hi != 0u) ? (out[h] & 0xffff0000u) : 0u);
      }
      *reinterpret_cast<v4u*>(a.y_dual + o) = od;
    }
  }
  }  // pass
}

// ------------------------------------------------------------ fwd / dgrad
template <int TBM, int BN, int NSTAGE, bool POOL = false>
__global__ void __launch_bounds__(TBM * 2) conv_fwd_kernel(ConvFwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int NT = TBM * 2;                   // (TBM/64) x 2 waves
  constexpr int A_BYTES = TBM * 128, B_BYTES = BN * 128, STAGE = A_BYTES + B_BYTES;
  constexpr int ALD = TBM * 8 / NT;             // A chunks per thread per step (4)
  constexpr int BLD = BN * 8 / NT;              // B chunks per thread per step
  constexpr int NLD = ALD + BLD;
  constexpr int NI = BN / 64;                   // 32-wide MFMA tiles per wave along N
  static_assert(BLD >= 1 && NSTAGE >= 2 && NSTAGE <= 3 && TBM % 64 == 0, "tile config");

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int ntn = a.K / BN;
  const int tn = bid % ntn, tm = bid / ntn;
  const int m0 = tm * TBM, n0 = tn * BN;
  const int C = a.C, H = a.H, W = a.W;
  const int CB = C >> 6;
  const int KT = 9 * CB;

  // A chunk i of this thread: LDS slot s = i*NT + tid -> (row, logical chunk)
  const uint16_t* a_ptr[ALD];
  uint32_t a_ok[ALD];  // bit t: tap t = 3r+s reads inside the image
#pragma unroll
  for (int i = 0; i < ALD; ++i) {
    const int s = i * NT + tid;
    const int row = s >> 3, lc = (s & 7) ^ sw_rd128(row);
    const int p = m0 + row;
    uint32_t ok = 0;
    if (p < a.P) {
      const uint32_t q = fdiv(static_cast<uint32_t>(p), a.div_w);
      const int w = p - static_cast<int>(q) * W;
      const int h = static_cast<int>(q - fdiv(q, a.div_h) * H);
      const uint32_t rok = (h > 0 ? 1u : 0u) | 2u | (h + 1 < H ? 4u : 0u);
      const uint32_t cok = (w > 0 ? 1u : 0u) | 2u | (w + 1 < W ? 4u : 0u);
#pragma unroll
      for (int r = 0; r < 3; ++r)
        if ((rok >> r) & 1u) ok |= cok << (3 * r);
    }
    a_ok[i] = ok;
    a_ptr[i] = a.x + static_cast<size_t>(p < a.P ? p : 0) * C + lc * 8;
  }
  const uint16_t* b_ptr[BLD];
#pragma unroll
  for (int j = 0; j < BLD; ++j) {
    const int s = j * NT + tid;
    const int row = s >> 3, lc = (s & 7) ^ sw_rd128(row);
    b_ptr[j] = a.w + static_cast<size_t>(n0 + row) * 9 * C + lc * 8;
  }
  const uint16_t* zero = reinterpret_cast<const uint16_t*>(g_conv_zero);

  int tap = 0, cb = 0;  // next K-step to issue
  auto issue = [&](int stage) __attribute__((always_inline)) {
    unsigned char* base = smem + stage * STAGE + wid * 1024;
    const int kr = tap / 3, ks = tap - 3 * (tap / 3);
    const int soff = ((kr - 1) * W + (ks - 1)) * C + cb * 64;
#pragma unroll
    for (int i = 0; i < ALD; ++i) {
      const uint16_t* src = ((a_ok[i] >> tap) & 1u) ? a_ptr[i] + soff : zero;
      glds16(src, base + i * NT * 16);
    }
    const int boff = tap * C + cb * 64;
#pragma unroll
    for (int j = 0; j < BLD; ++j) glds16(b_ptr[j] + boff, base + A_BYTES + j * NT * 16);
    if (++cb == CB) { cb = 0; ++tap; }
  };

  f32x16_t acc[2][NI];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[mi][ni][e] = 0.f;

  issue(0);
  if (NSTAGE == 3 && KT > 1) issue(1);
  const int hi = lane >> 5, lr = lane & 31;
  // byte offsets (inside a stage's A / B image) of this lane's fragments
  int offA[4][2], offB[4][NI];
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) {
    const int chk = 2 * kk + hi;
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) {
      const int row = wr * 64 + mi * 32 + lr;
      offA[kk][mi] = row * 128 + ((chk ^ sw_rd128(row)) << 4);
    }
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) {
      const int row = wc * (BN / 2) + ni * 32 + lr;
      offB[kk][ni] = row * 128 + ((chk ^ sw_rd128(row)) << 4);
    }
  }
  int rd = 0, wrs = NSTAGE - 1;  // stage read this step / stage written next
  for (int kt = 0; kt < KT; ++kt) {
    if constexpr (NSTAGE == 3) {
      if (kt + 1 < KT) wait_vmcnt<NLD>(); else wait_vmcnt<0>();
    } else {
      wait_vmcnt<0>();
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt + NSTAGE - 1 < KT) issue(wrs);
    const unsigned char* sA = smem + rd * STAGE;
    const unsigned char* sB = sA + A_BYTES;
    // fragments of sub-step kk+1 are read while the MFMAs of kk run
    bf16x8_t af[2][2], bfr[2][NI];
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) af[0][mi] = *reinterpret_cast<const bf16x8_t*>(sA + offA[0][mi]);
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) bfr[0][ni] = *reinterpret_cast<const bf16x8_t*>(sB + offB[0][ni]);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int cur = kk & 1, nxt = cur ^ 1;
      if (kk + 1 < 4) {
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
          af[nxt][mi] = *reinterpret_cast<const bf16x8_t*>(sA + offA[kk + 1][mi]);
#pragma unroll
        for (int ni = 0; ni < NI; ++ni)
          bfr[nxt][ni] = *reinterpret_cast<const bf16x8_t*>(sB + offB[kk + 1][ni]);
      }
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[cur][mi], bfr[cur][ni], acc[mi][ni], 0, 0, 0);
    }
    rd = rd + 1 == NSTAGE ? 0 : rd + 1;
    wrs = wrs + 1 == NSTAGE ? 0 : wrs + 1;
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  conv_fwd_epilogue<TBM, BN, POOL>(a, acc, smem, m0, n0, tid, wr, wc, hi, lr);
}

// ---------------------------------------------------- fwd / dgrad, halo
// Same GEMM and epilogue as conv_fwd_kernel<128, 128, 2>, but the A operand
// of the 9 taps comes from ONE padded window per 64-channel block instead of
// 9 separately staged 128-row tiles: the tile's 128 output pixels are whole
// image rows (G images x Rg rows x W), the window holds their rows -1..Rg
// and columns -1..W (zero page outside the image), and tap (r, s) reads the
// window shifted by (r-1, s-1).  LDS-DMA pieces per K-step drop from 8 to
// ~5 per thread (the 128 x 128 loop is bound by per-CU load issue).
// LDS: window (<= 288 padded rows, 36 KB) + B ring 2 x 16 KB: 68 KB, 2 blocks/CU.
struct HaloGeom {
  // images / rows per image in a tile, padded width, padded rows (images
  // stacked with ONE shared zero row between them: G * (Rg + 1) + 1), window
  // rows (padded rows x padded width)
  int G, Rg, PW, PR, NPW;
  // window swizzle (halo_swizzle): 16-byte chunk c of padded row (pr, pc) sits
  // at slot c ^ (((pc >> 1) + swa * pr + swb * (pr >> 2)) & 7)
  int swa, swb;
};

// The A fragments' ds_read_b128 lane groups ({0-3,12-15,20-27}, ...) read
// window rows that jump by the padding columns at every image row of the
// tile, so the chunk swizzle must depend on the padded (row, column), not on
// the flat window row: with the flat-row swizzle (row >> 1) & 7 a 16x16 layer
// reads its A fragments in 8 LDS cycles instead of 4, an 8x8 layer in 12
// (a lane-exact model of the four lane groups over every tap, wave and
// sub-step).  Per width the (swa, swb) below make 32/16/8-wide tiles
// conflict-free and 4-wide ones 6 cycles (flat swizzle: 8).
__device__ __forceinline__ int sw_halo(int pr, int pc, const HaloGeom& g) {
  return ((pc >> 1) + g.swa * pr + g.swb * (pr >> 2)) & 7;
}
// TBM = 128 (4 waves, window <= 288 rows) or 256 (8 waves, <= 384 rows:
// 48 KB + B ring 32 KB = 80 KB, still 2 blocks/CU; the B tile then feeds 256
// pixels, halving its pieces per MFMA once more)
template <int TBM>
struct HaloCfg {
  static constexpr int kMaxRows = TBM == 256 ? 384 : 288;
  static constexpr int kWinBytes = kMaxRows * 128;
  static constexpr int kLds = kWinBytes + 2 * 128 * 128;
  static constexpr int kWinLd = (kMaxRows * 8 + TBM * 2 - 1) / (TBM * 2);  // window pieces per thread
};

// SPLIT: one 8-wave block per output tile, two 4-wave groups each running
// half of the 64-channel blocks in its own LDS window + B ring (2 x 68 KB, 1
// block/CU).  The second group's partial tile is added to the first's through
// LDS (fixed order: bitwise deterministic) and all 8 waves run the epilogue.
// For grids that would leave half the resident slots empty (ResNet-9 res3:
// 252 tiles on 256 CUs).  (Measured alternatives: two blocks per tile with a
// last-arriver combine needs device-scope release fences -- L2 writebacks
// across the 8 XCDs, 140 us vs 62 unsplit; partial tiles through an HBM
// workspace + a combine kernel: 44 + 12 us.)
// BN = 64: 64-wide outputs (ResNet-9 layer-1 dgrad, 128 -> 64 channels), wave
// tiles of 64 x 32 (one MFMA column), B ring 2 x 8 KB.
template <int TBM, int BN>
constexpr int halo_lds() { return HaloCfg<TBM>::kWinBytes + 2 * BN * 128; }

// Double-buffered operand fragments.  Without them the compiler (at the
// 128-VGPR budget of 4 waves/SIMD) gave the next sub-step's fragments the
// registers of the current ones, so every 4-MFMA group waited for its own LDS
// reads (s_waitcnt lgkmcnt(0) right before it, disassembly) -- ~45 % of the
// MFMA rate with every global load, barrier and the epilogue removed
// (profiles/r4_experiments.md).  The fragment offsets are one register per
// operand row (sub-step kk flips chunk bits 5-6), the reads of sub-step kk+1
// are pinned above the MFMAs of kk (sched_barrier), and the step's barrier
// sits before the last sub-step's MFMAs, which overlap the next step's first
// reads.
// BT (grouped input gradient straight from the clients' weight rows,
// parallel/fedavg_native.py): the weights are the CONV's rows [Kc][3][3][Cc]
// per group (Kc = a.C, the dgrad's input channels; Cc = a.kg, its outputs),
// read flipped: the B tile of (tap, 64-channel block) is staged k-major
// ([64 k][128 c], 256-byte rows: the rows' own order) and its fragments come
// from transposing LDS reads -- no transposed weight image per step.
// KS: split-K across blocks (a.ksplit blocks per output tile, each a whole
// number of 64-channel blocks): the partial tile goes to a.part, and
// conv_fwd_combine_kernel sums the splits in a fixed order and runs the
// epilogue.  For grids of few tiles -- e.g. the per-rank round of a
// strong-scaled W = 100 round at N = 8 (13 clients): res3's 4x4 maps are 36
// tiles of 72 K-steps for 256 CUs.
template <int TBM, bool POOL, bool SPLIT = false, int BN = 128, bool BT = false, bool KS = false>
__global__ void __launch_bounds__(TBM * 2 * (SPLIT ? 2 : 1))
__attribute__((amdgpu_waves_per_eu((TBM == 256 && !SPLIT) ? 4 : 1)))  // two 8-wave blocks per CU
conv_fwd_halo_kernel(ConvFwdArgs a, HaloGeom hg) {
  static_assert(BN == 128 || (BN == 64 && !SPLIT && !POOL), "halo tile width");
  static_assert(!BT || (!SPLIT && !POOL), "transposed weight rows: plain tiles");
  static_assert(!KS || (!SPLIT && !BT), "cross-block split-K: plain tiles");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_base[];
  // group g (split-K half) of this block: its own window + B ring
  const int half = SPLIT ? static_cast<int>(threadIdx.x) / (TBM * 2) : 0;
  unsigned char* const smem = smem_base + half * halo_lds<TBM, BN>();
  constexpr int NI = BN / 64, NT = TBM * 2, BLD = BN * 8 / NT;
  constexpr int kHaloWinBytes = HaloCfg<TBM>::kWinBytes, kHaloWinLd = HaloCfg<TBM>::kWinLd;
  const int tid = threadIdx.x & (NT - 1), lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const int bid0 = xcd_remap(blockIdx.x, gridDim.x);
  const int kspl = KS ? bid0 % a.ksplit : 0, bid = KS ? bid0 / a.ksplit : bid0;
  const int ntn = a.K / BN;
  const int tn = bid % ntn, tm = bid / ntn;
  const int m0 = tm * TBM, n0 = tn * BN;
  const int C = a.C, H = a.H, W = a.W, HW = H * W;
  const int KT = 9 * (C >> 6);
  int s_beg = SPLIT ? half * (KT / 2) : 0, s_end = SPLIT ? s_beg + KT / 2 : KT;
  if constexpr (KS) {
    s_beg = kspl * (KT / a.ksplit);
    s_end = s_beg + KT / a.ksplit;
  }
  const int img0 = m0 / HW, h0 = (m0 - img0 * HW) / W;  // first image / row of the tile
  // grouped (channel-stacked) images: row stride and this tile's channel group
  const int xs = a.x_stride > 0 ? a.x_stride : C;
  const int cofs = a.kg > 0 ? (n0 / a.kg) * C : 0;
  const int nimg = a.P / HW;
  const uint16_t* zero = reinterpret_cast<const uint16_t*>(g_conv_zero);

  // window pieces of this thread: source offset (elements) or -1 for padding
  int win_off[kHaloWinLd];
#pragma unroll
  for (int i = 0; i < kHaloWinLd; ++i) {
    const int sl = i * NT + tid;
    const int row = sl >> 3;
    int off = -1;
    if (row < hg.NPW) {
      const int pr = row / hg.PW, pc = row - pr * hg.PW, w = pc - 1;
      const int lc = (sl & 7) ^ sw_halo(pr, pc, hg);
      // padded row pr: G == 1 -> image row h0 + pr - 1 (zero outside the
      // image); else pr = g (Rg + 1) + 1 + h, separators (pr % (Rg+1) == 0) zero
      int img = img0, h = h0 + pr - 1;
      if (hg.G > 1) {
        const int q = pr / (hg.Rg + 1), rr = pr - q * (hg.Rg + 1);
        img = img0 + q;
        h = rr - 1;  // -1 on a separator row
      }
      if (img < nimg && h >= 0 && h < H && w >= 0 && w < W) off = ((img * H + h) * W + w) * xs + cofs + lc * 8;
    }
    win_off[i] = off;
  }
  // grouped weights not stored as one [G kg][3][3][C] image (a.w_gs != 0):
  // this tile's group (n0 / kg, block-uniform since kg % BN == 0) reads its
  // own rows w_gs elements apart (> 0), or every group the same rows (< 0)
  const uint16_t* wsrc = a.w;
  if (a.kg > 0 && a.w_gs != 0) {
    const int64_t g = n0 / a.kg;
    wsrc += (a.w_gs > 0 ? g * a.w_gs : int64_t{0}) - g * a.kg * 9 * static_cast<int64_t>(C);
  }
  int b_off[BLD];  // element offsets into a.w (< K * 9 * C)
  const uint16_t* wbt = a.w;  // BT: this group's conv rows
  int bt_c0 = 0;
#pragma unroll
  for (int j = 0; j < BLD; ++j) {
    const int sl = j * NT + tid;
    if constexpr (BT) {  // [64 k rows][BN / 8 chunks of 8 c], transposed-read swizzle
      const int row = BN == 128 ? sl >> 4 : sl >> 3;
      const int lc = BN == 128 ? (sl & 15) ^ sw_tr256(row) : (sl & 7) ^ sw_tr128(row);
      b_off[j] = row * 9 * a.kg + lc * 8;
    } else {
      const int row = sl >> 3, lc = (sl & 7) ^ sw_rd128(row);
      b_off[j] = (n0 + row) * 9 * C + lc * 8;
    }
  }
  if constexpr (BT) {
    const int64_t g = n0 / a.kg;
    wbt = a.w + (a.w_gs > 0 ? g * a.w_gs : int64_t{0});
    bt_c0 = n0 - static_cast<int>(g) * a.kg;
  }
  auto issue_window = [&](int cb) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < kHaloWinLd; ++i) {
      if (i * NT + (tid & ~63) < hg.NPW * 8) {  // wave-uniform: pieces past the window skipped
        const int off = win_off[i];
        glds16(off >= 0 ? a.x + off + cb * 64 : zero, smem + i * NT * 16 + wid * 1024);
      }
    }
  };
  // K-step s = cb * 9 + tap (channel block outer: one window per cb)
  auto issue_b = [&](int step) __attribute__((always_inline)) {
    unsigned char* base = smem + kHaloWinBytes + (step & 1) * (BN * 128) + wid * 1024;
    if constexpr (BT) {
      // rows k = (step / 9) 64 + row, flipped tap 8 - step % 9, columns bt_c0..
      const int64_t boff = static_cast<int64_t>(step / 9) * 64 * 9 * a.kg + (8 - step % 9) * a.kg + bt_c0;
#pragma unroll
      for (int j = 0; j < BLD; ++j) glds16(wbt + (b_off[j] + boff), base + j * NT * 16);
    } else {
      const int boff = (step % 9) * C + (step / 9) * 64;
#pragma unroll
      for (int j = 0; j < BLD; ++j) glds16(wsrc + (b_off[j] + boff), base + j * NT * 16);
    }
  };

  // this lane's output pixels (rows of the A fragments) -> padded window rows
  const int hi = lane >> 5, lr = lane & 31;
  int pbr[2], pbc[2];  // padded (row, column) of the tap-(1, 1) window row
#pragma unroll
  for (int mi = 0; mi < 2; ++mi) {
    const int m = wr * 64 + mi * 32 + lr;
    const int g = m / (hg.Rg * W), rem = m - g * hg.Rg * W;
    const int r = rem / W, w = rem - r * W;
    pbr[mi] = g * (hg.Rg + 1) + r + 1;
    pbc[mi] = w + 1;
  }
  f32x16_t acc[2][NI];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[mi][ni][e] = 0.f;

    int bB[NI];  // sub-step 0 B offsets; sub-step kk: ^ (kk << 5)
    int tB[NI][2];  // BT: transposed-read offsets; sub-step kk: + kk 16 rows
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) {
      const int row = wc * (BN / 2) + ni * 32 + lr;
      bB[ni] = row * 128 + ((hi ^ sw_rd128(row)) << 4);
      if constexpr (BT) tr_offsets<BN * 2>(wc * (BN / 2) + ni * 32, lane, tB[ni]);
    }
    auto a_base = [&](int st, int (&bA)[2]) __attribute__((always_inline)) {
      const int tap = st % 9, dr = tap / 3 - 1, dc = tap % 3 - 1;
#pragma unroll
      for (int mi = 0; mi < 2; ++mi) {
        const int pr = pbr[mi] + dr, pc = pbc[mi] + dc;
        bA[mi] = (pr * hg.PW + pc) * 128 + ((hi ^ sw_halo(pr, pc, hg)) << 4);
      }
    };
    auto load = [&](int st, int kk, const int (&bA)[2], bf16x8_t (&fa)[2], bf16x8_t (&fb)[NI])
        __attribute__((always_inline)) {
      const unsigned char* sB = smem + kHaloWinBytes + (st & 1) * (BN * 128);
#pragma unroll
      for (int mi = 0; mi < 2; ++mi) fa[mi] = *reinterpret_cast<const bf16x8_t*>(smem + (bA[mi] ^ (kk << 5)));
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) {
        if constexpr (BT)
          fb[ni] = tr_read(sB + tB[ni][0] + kk * 16 * BN * 2, sB + tB[ni][1] + kk * 16 * BN * 2);
        else
          fb[ni] = *reinterpret_cast<const bf16x8_t*>(sB + (bB[ni] ^ (kk << 5)));
      }
    };
    auto mma = [&](const bf16x8_t (&fa)[2], const bf16x8_t (&fb)[NI]) __attribute__((always_inline)) {
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[mi], fb[ni], acc[mi][ni], 0, 0, 0);
    };
    issue_window(s_beg / 9);
    issue_b(s_beg);
    wait_vmcnt<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (s_beg + 1 < s_end) issue_b(s_beg + 1);
    int bA[2];
    a_base(s_beg, bA);
    bf16x8_t fa0[2], fb0[NI], fa1[2], fb1[NI];
    load(s_beg, 0, bA, fa0, fb0);
    // MFMAs of one buffer interleaved one-for-one with the reads of the other
    // (an MFMA gap takes 2 ds_read_b128 at no cost, MI355X_MICROARCH.md §LDS):
    // the reads are in flight under the MFMAs that precede their use
    auto interleave = [&]() __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // one MFMA
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // one LDS read
      }
    };
    for (int s = s_beg; s < s_end; ++s) {
      __builtin_amdgcn_sched_barrier(0);
      mma(fa0, fb0);
      load(s, 1, bA, fa1, fb1);
      interleave();
      __builtin_amdgcn_sched_barrier(0);
      mma(fa1, fb1);
      load(s, 2, bA, fa0, fb0);
      interleave();
      __builtin_amdgcn_sched_barrier(0);
      mma(fa0, fb0);
      load(s, 3, bA, fa1, fb1);
      interleave();
      __builtin_amdgcn_sched_barrier(0);
      if (s + 1 < s_end) {
        // this wave's reads of step s are done; at a channel-block boundary every
        // wave's are (barrier) before the next window overwrites the old one
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if ((s + 1) % 9 == 0) {
          __builtin_amdgcn_s_barrier();
          issue_window((s + 1) / 9);
        }
        wait_vmcnt<0>();  // B(s + 1) (and the new window) landed for this wave ...
        __builtin_amdgcn_s_barrier();  // ... and for every wave; slot s & 1 is free
        if (s + 2 < s_end) issue_b(s + 2);
        a_base(s + 1, bA);
        load(s + 1, 0, bA, fa0, fb0);
      }
      __builtin_amdgcn_sched_barrier(0);
      mma(fa1, fb1);
    }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if constexpr (SPLIT) {
    // group 1 parks its fragments in group 0's region (read by nobody now);
    // group 0 adds them lane for lane, then both groups run the epilogue
    float* red = reinterpret_cast<float*>(smem_base);
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int ni = 0; ni < NI; ++ni)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int o = ((mi * NI + ni) * 16 + e) * NT + tid;
          if (half == 1) red[o] = acc[mi][ni][e];
        }
    __syncthreads();
    if (half == 0) {
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni)
#pragma unroll
          for (int e = 0; e < 16; ++e) acc[mi][ni][e] += red[((mi * NI + ni) * 16 + e) * NT + tid];
    }
    __syncthreads();  // red is read before the epilogue overwrites the region
    conv_fwd_epilogue<TBM, BN, POOL, TBM * 4>(a, acc, smem_base, m0, n0, threadIdx.x, wr, wc, hi, lr,
                                              half == 0);
  } else if constexpr (KS) {
    // the partial tile, [tile][split][accumulator register][thread]: a wave's
    // stores and the combine kernel's loads are 256-byte runs
    float* pt = a.part + static_cast<size_t>(bid * a.ksplit + kspl) * (2 * NI * 16) * NT + tid;
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int ni = 0; ni < NI; ++ni)
#pragma unroll
        for (int e = 0; e < 16; ++e) pt[static_cast<size_t>((mi * NI + ni) * 16 + e) * NT] = acc[mi][ni][e];
  } else {
    conv_fwd_epilogue<TBM, BN, POOL>(a, acc, smem, m0, n0, tid, wr, wc, hi, lr);
  }
}

// sum[t][i] = sum over s of part[t][s][i], s in order (deterministic), 16
// bytes a thread: the splits' reduction spread over the whole chip (the
// combine kernel below has only one block per tile)
__global__ void __launch_bounds__(256) conv_fwd_psum_kernel(const float* __restrict__ part, float* __restrict__ sum,
                                                            int tiles, int ks, int n4) {
  const int q = blockIdx.x * 256 + threadIdx.x;  // float4 index over tiles x n4
  if (q >= tiles * n4) return;
  const int t = q / n4, i = q - t * n4;
  const float4* p = reinterpret_cast<const float4*>(part) + static_cast<size_t>(t) * ks * n4 + i;
  float4 a = p[0];
  for (int s = 1; s < ks; ++s) {
    const float4 b = p[static_cast<size_t>(s) * n4];
    a.x += b.x;
    a.y += b.y;
    a.z += b.z;
    a.w += b.w;
  }
  reinterpret_cast<float4*>(sum)[q] = a;
}

// sum of a tile's a.ksplit partials (split order: deterministic) in the
// accumulator layout of conv_fwd_halo_kernel, then its epilogue
template <int TBM, bool POOL, int BN>
__global__ void __launch_bounds__(TBM * 2) conv_fwd_combine_kernel(ConvFwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int NI = BN / 64, NT = TBM * 2, NREG = 2 * NI * 16;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1, hi = lane >> 5, lr = lane & 31;
  const int tile = blockIdx.x, ntn = a.K / BN;
  const int m0 = (tile / ntn) * TBM, n0 = (tile % ntn) * BN;
  f32x16_t acc[2][NI];
  const float* pt = a.part + static_cast<size_t>(tile) * a.ksplit * NREG * NT + tid;
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[mi][ni][e] = pt[static_cast<size_t>((mi * NI + ni) * 16 + e) * NT];
  for (int s = 1; s < a.ksplit; ++s) {
    const float* ps = pt + static_cast<size_t>(s) * NREG * NT;
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int ni = 0; ni < NI; ++ni)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[mi][ni][e] += ps[static_cast<size_t>((mi * NI + ni) * 16 + e) * NT];
  }
  conv_fwd_epilogue<TBM, BN, POOL>(a, acc, smem, m0, n0, tid, wr, wc, hi, lr);
}

// ------------------------------------------------------------------ wgrad
// pixel range [pbeg, pend) of one split: consecutive steps_per_split * BK
// pixels, or (grouped) the split's share of its group's pixels -- rows past
// pend are masked, so a range need not start or end on a K-step
__device__ __forceinline__ void wgrad_split_range(const ConvWgradArgs& a, int split, int* pbeg,
                                                  int* pend) {
  if (a.group_px > 0) {
    const int g = split / a.splits_per_group, s = split - g * a.splits_per_group;
    const int g0 = g * a.group_px;
    *pbeg = g0 + s * a.steps_per_split * BK;
    *pend = min(g0 + a.group_px, *pbeg + a.steps_per_split * BK);
    return;
  }
  *pbeg = split * a.steps_per_split * BK;
  *pend = min(a.P, *pbeg + a.steps_per_split * BK);
}

// PAIR (C == 64, BN == 128): a tile's 128 columns are TWO taps x 64 input
// channels (taps 2q, 2q+1; the 10th tap of the last pair is a zero operand
// that is never stored), so 64-channel layers run the 128-wide wave tiles
template <int BN, int NSTAGE, bool ROWSTEP, bool PAIR = false>
__global__ void __launch_bounds__(256) conv_wgrad_kernel(ConvWgradArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int A_BYTES = BK * WBM * 2;  // [64 px][128 k], 256-byte rows
  constexpr int B_BYTES = BK * BN * 2;   // [64 px][BN c]
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int ALD = 4;
  constexpr int BCH = BN / 8;            // 16-byte chunks per B row
  constexpr int BLD = BK * BCH / 256;
  constexpr int NLD = ALD + BLD;
  constexpr int NI = BN / 64;
  static_assert(NSTAGE >= 2 && NSTAGE <= 3, "stages");
  static_assert(!PAIR || BN == 128, "tap pairs fill a 128-wide tile");
  constexpr int NTAPG = PAIR ? 5 : 9;     // tap groups per (k, c) tile

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int C = a.C, K = a.K, H = a.H, W = a.W;
  const int ntc = PAIR ? 1 : C / BN, ntk = K / WBM;
  const int ntiles = ntk * NTAPG * ntc;
  const int tile = bid % ntiles, split = bid / ntiles;
  const int tc = tile % ntc, rs = (tile / ntc) % NTAPG, tk = tile / (ntc * NTAPG);
  const int k0 = tk * WBM, c0 = tc * BN;
  int pbeg, pend;
  wgrad_split_range(a, split, &pbeg, &pend);
  const int nsteps = pend > pbeg ? (pend - pbeg + BK - 1) / BK : 0;
  // DMA source addresses as integers (pointer arrays + selects made hipcc
  // spill the array to scratch and index it dynamically)
  const uint64_t zero = reinterpret_cast<uint64_t>(g_conv_zero);

  // A chunks: rows of dy
  uint64_t a_ptr[ALD];
  int a_row[ALD];
#pragma unroll
  for (int i = 0; i < ALD; ++i) {
    const int s = i * 256 + tid;
    const int row = s >> 4, lc = (s & 15) ^ sw_tr256(row);
    a_row[i] = pbeg + row;
    a_ptr[i] = reinterpret_cast<uint64_t>(a.dy + static_cast<size_t>(pbeg + row) * K + k0 + lc * 8);
  }
  // B chunks: rows of x at the tap offset; (h, w) of the row tracked per step
  uint64_t b_ptr[BLD];
  int b_row[BLD], b_h[BLD], b_w[BLD], b_dr[BLD], b_ds[BLD];
  uint32_t b_tok = 0;  // bit j: chunk j belongs to a real tap (PAIR: not the 10th)
#pragma unroll
  for (int j = 0; j < BLD; ++j) {
    const int s = j * 256 + tid;
    int row, lc;
    if constexpr (BN == 128) { row = s >> 4; lc = (s & 15) ^ sw_tr256(row); }
    else { row = s >> 3; lc = (s & 7) ^ sw_tr128(row); }
    int tap = rs, cc = lc;
    if constexpr (PAIR) { tap = 2 * rs + (lc >> 3); cc = lc & 7; }
    b_tok |= (tap < 9 ? 1u : 0u) << j;
    if (tap > 8) tap = 8;
    b_dr[j] = tap / 3 - 1;
    b_ds[j] = tap % 3 - 1;
    const int p = pbeg + row;
    b_row[j] = p;
    const uint32_t q = fdiv(static_cast<uint32_t>(p), a.div_w);
    b_w[j] = p - static_cast<int>(q) * W;
    b_h[j] = static_cast<int>(q - fdiv(q, a.div_h) * H) + b_dr[j];  // tap row of the source
    b_ptr[j] = reinterpret_cast<uint64_t>(a.x + static_cast<int64_t>(p + b_dr[j] * W + b_ds[j]) * C +
                                          c0 + cc * 8);
  }
  // when W | BK a step advances every row by BK/W whole image rows: w is
  // fixed per chunk and h advances incrementally (ROWSTEP); else recompute
  uint32_t b_wok = 0;  // bit j: column of chunk j stays inside the image at its tap
#pragma unroll
  for (int j = 0; j < BLD; ++j)
    b_wok |= (static_cast<unsigned>(b_w[j] + b_ds[j]) < static_cast<unsigned>(W) ? 1u : 0u) << j;
  b_wok &= b_tok;
  const int dh = ROWSTEP ? (BK / W) % H : 0;

  auto issue = [&](int stage, bool full) __attribute__((always_inline)) {
    unsigned char* base = smem + stage * STAGE + wid * 1024;
#pragma unroll
    for (int i = 0; i < ALD; ++i) {
      glds16(reinterpret_cast<const void*>(full || a_row[i] < pend ? a_ptr[i] : zero),
             base + i * 4096);
      a_row[i] += BK;
      a_ptr[i] += static_cast<uint64_t>(BK) * K * 2;
    }
#pragma unroll
    for (int j = 0; j < BLD; ++j) {
      bool ok = static_cast<unsigned>(b_h[j]) < static_cast<unsigned>(H);
      if constexpr (ROWSTEP) ok = ok && ((b_wok >> j) & 1u);
      else ok = ok && ((b_tok >> j) & 1u) && static_cast<unsigned>(b_w[j] + b_ds[j]) < static_cast<unsigned>(W);
      if (!full) ok = ok && b_row[j] < pend;
      glds16(reinterpret_cast<const void*>(ok ? b_ptr[j] : zero), base + A_BYTES + j * 4096);
      b_row[j] += BK;
      b_ptr[j] += static_cast<uint64_t>(BK) * C * 2;
      if constexpr (ROWSTEP) {
        const int nh = b_h[j] + dh;
        b_h[j] = nh - b_dr[j] >= H ? nh - H : nh;
      } else {
        const uint32_t q = fdiv(static_cast<uint32_t>(b_row[j]), a.div_w);
        b_w[j] = b_row[j] - static_cast<int>(q) * W;
        b_h[j] = static_cast<int>(q - fdiv(q, a.div_h) * H) + b_dr[j];
      }
    }
  };

  f32x16_t acc[2][NI];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[mi][ni][e] = 0.f;

  if (nsteps > 0) issue(0, pbeg + BK <= pend);
  if (NSTAGE == 3 && nsteps > 1) issue(1, pbeg + 2 * BK <= pend);
  // this lane's transposed-read offsets at sub-step 0 (the swizzles do not
  // depend on the sub-step: sub-step kk adds kk * 16 rows)
  int toA[2][2], toB[NI][2];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi) tr_offsets<256>(wr * 64 + mi * 32, lane, toA[mi]);
#pragma unroll
  for (int ni = 0; ni < NI; ++ni) tr_offsets<BN * 2>(wc * (BN / 2) + ni * 32, lane, toB[ni]);
  int rd = 0, wrs = NSTAGE - 1;
  for (int st = 0; st < nsteps; ++st) {
    if constexpr (NSTAGE == 3) {
      if (st + 1 < nsteps) wait_vmcnt<NLD>(); else wait_vmcnt<0>();
    } else {
      wait_vmcnt<0>();
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (st + NSTAGE - 1 < nsteps) issue(wrs, pbeg + (st + NSTAGE) * BK <= pend);
    const unsigned char* sA = smem + rd * STAGE;
    const unsigned char* sB = sA + A_BYTES;
    bf16x8_t af[2][2], bfr[2][NI];
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) af[0][mi] = tr_read(sA + toA[mi][0], sA + toA[mi][1]);
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) bfr[0][ni] = tr_read(sB + toB[ni][0], sB + toB[ni][1]);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int cur = kk & 1, nxt = cur ^ 1;
      if (kk + 1 < 4) {
        const int da = (kk + 1) * 16 * 256, db = (kk + 1) * 16 * BN * 2;
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
          af[nxt][mi] = tr_read(sA + toA[mi][0] + da, sA + toA[mi][1] + da);
#pragma unroll
        for (int ni = 0; ni < NI; ++ni)
          bfr[nxt][ni] = tr_read(sB + toB[ni][0] + db, sB + toB[ni][1] + db);
      }
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[cur][mi], bfr[cur][ni], acc[mi][ni], 0, 0, 0);
    }
    rd = rd + 1 == NSTAGE ? 0 : rd + 1;
    wrs = wrs + 1 == NSTAGE ? 0 : wrs + 1;
  }

  // slab[split][k][rs][c] (fp32), lanes 0..31 store 32 consecutive c
  float* slab = a.slab + static_cast<size_t>(split) * K * 9 * C;
  const int hi = lane >> 5, lr = lane & 31;
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int k = k0 + wr * 64 + mi * 32 + (e & 3) + 8 * (e >> 2) + 4 * hi;
        const int n = wc * (BN / 2) + ni * 32 + lr;
        if constexpr (PAIR) {  // column n = (tap 2 rs + n / 64, channel n % 64)
          const int tap = 2 * rs + (n >> 6);
          if (tap < 9) slab[(static_cast<size_t>(k) * 9 + tap) * C + (n & 63)] = acc[mi][ni][e];
        } else {
          slab[(static_cast<size_t>(k) * 9 + rs) * C + c0 + n] = acc[mi][ni][e];
        }
      }
}

// Wide wgrad tile (K >= 256): 256 out channels x 256 columns per block, 8
// waves as 4 (k) x 2 (columns), each wave 64 x 128 (2 x 4 MFMA tiles).  Per
// 64-pixel K-step a wave issues the same 8 LDS-DMA pieces as the 128 x 128
// kernel but runs twice the MFMAs (the DMA issue cost, ~60-180 cycles a
// piece, is what bounds the 128 x 128 tile).  Columns are TPG taps x 256/TPG
// input channels (TPG = 2 for 128-channel inputs: taps 2g, 2g+1; the 10th
// tap of the last group is a zero operand that is never stored).  The
// operand images are pairs of the 128-wide [64 px][128] images of the small
// kernel (same swizzle and transposed reads), one block per CU (128 KB LDS);
// split-K over pixels fills the chip, slabs as in conv_wgrad_kernel.
template <bool ROWSTEP, int TPG, bool IL = true>
__global__ void __launch_bounds__(512) conv_wgrad_wide_kernel(ConvWgradArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int HALF = BK * 128 * 2;           // one [64 px][128] image, 16 KB
  constexpr int A_BYTES = 2 * HALF, STAGE = 4 * HALF;
  constexpr int NTAPG = TPG == 2 ? 5 : 9;
  constexpr int CPT = 256 / TPG;               // input channels per tap in a tile

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int C = a.C, K = a.K, H = a.H, W = a.W;
  const int ntc = C / CPT, ntk = K / 256;
  const int ntiles = ntk * NTAPG * ntc;
  const int tile = bid % ntiles, split = bid / ntiles;
  const int tc = tile % ntc, rs = (tile / ntc) % NTAPG, tk = tile / (ntc * NTAPG);
  const int k0 = tk * 256, c0 = tc * CPT;
  // grouped (channel-stacked) x: pixel row stride and this tile's channel
  // group (kg % 256 == 0: a 256-row tile is one group's output channels)
  const int xs = a.x_stride > 0 ? a.x_stride : C;
  const int cofs = a.kg > 0 ? (k0 / a.kg) * C : 0;
  int pbeg, pend;
  wgrad_split_range(a, split, &pbeg, &pend);
  const int nsteps = pend > pbeg ? (pend - pbeg + BK - 1) / BK : 0;
  const uint64_t zero = reinterpret_cast<uint64_t>(g_conv_zero);

  // piece i (0..3) of thread tid: image half h = i >> 1, chunk s' in the half
  uint64_t a_ptr[4], b_ptr[4];
  int a_row[4], b_row[4], b_h[4], b_w[4], b_dr[4], b_ds[4];
  uint32_t b_ok = 0;  // bit i: piece i belongs to a real tap and its column stays inside the image
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int h = i >> 1, sp = (i & 1) * 512 + tid;
    const int row = sp >> 4, lc = (sp & 15) ^ sw_tr256(row);
    a_row[i] = pbeg + row;
    a_ptr[i] = reinterpret_cast<uint64_t>(a.dy + static_cast<size_t>(pbeg + row) * K + k0 + h * 128 + lc * 8);
    const int n = h * 128 + lc * 8;  // tile column of the piece
    int tap = rs, cc = c0 + n;
    if constexpr (TPG == 2) { tap = 2 * rs + h; cc = c0 + lc * 8; }
    const bool real = tap < 9;
    if (tap > 8) tap = 8;
    b_dr[i] = tap / 3 - 1;
    b_ds[i] = tap % 3 - 1;
    const int p = pbeg + row;
    b_row[i] = p;
    const uint32_t q = fdiv(static_cast<uint32_t>(p), a.div_w);
    b_w[i] = p - static_cast<int>(q) * W;
    b_h[i] = static_cast<int>(q - fdiv(q, a.div_h) * H) + b_dr[i];
    b_ptr[i] = reinterpret_cast<uint64_t>(a.x + static_cast<int64_t>(p + b_dr[i] * W + b_ds[i]) * xs + cofs + cc);
    if (real && static_cast<unsigned>(b_w[i] + b_ds[i]) < static_cast<unsigned>(W)) b_ok |= 1u << i;
    if (!ROWSTEP && real) b_ok |= 16u << i;  // (recomputed per step below)
  }
  const int dh = ROWSTEP ? (BK / W) % H : 0;

  auto issue = [&](int stage, bool full) __attribute__((always_inline)) {
    unsigned char* base = smem + stage * STAGE + wid * 1024;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      glds16(reinterpret_cast<const void*>(full || a_row[i] < pend ? a_ptr[i] : zero),
             base + (i >> 1) * HALF + (i & 1) * 8192);
      a_row[i] += BK;
      a_ptr[i] += static_cast<uint64_t>(BK) * K * 2;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      bool ok = static_cast<unsigned>(b_h[i]) < static_cast<unsigned>(H);
      if constexpr (ROWSTEP) ok = ok && ((b_ok >> i) & 1u);
      else ok = ok && ((b_ok >> (4 + i)) & 1u) && static_cast<unsigned>(b_w[i] + b_ds[i]) < static_cast<unsigned>(W);
      if (!full) ok = ok && b_row[i] < pend;
      glds16(reinterpret_cast<const void*>(ok ? b_ptr[i] : zero),
             base + A_BYTES + (i >> 1) * HALF + (i & 1) * 8192);
      b_row[i] += BK;
      b_ptr[i] += static_cast<uint64_t>(BK) * xs * 2;
      if constexpr (ROWSTEP) {
        const int nh = b_h[i] + dh;
        b_h[i] = nh - b_dr[i] >= H ? nh - H : nh;
      } else {
        const uint32_t q = fdiv(static_cast<uint32_t>(b_row[i]), a.div_w);
        b_w[i] = b_row[i] - static_cast<int>(q) * W;
        b_h[i] = static_cast<int>(q - fdiv(q, a.div_h) * H) + b_dr[i];
      }
    }
  };

  f32x16_t acc[2][4];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[mi][ni][e] = 0.f;

  if (nsteps > 0) issue(0, pbeg + BK <= pend);
  // transposed-read offsets: A rows k = wr*64 + mi*32 live in half wr >> 1;
  // B columns wc*128 + ni*32 in half wc
  int toA[2][2], toB[4][2];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi) {
    tr_offsets<256>((wr & 1) * 64 + mi * 32, lane, toA[mi]);
    toA[mi][0] += (wr >> 1) * HALF;
    toA[mi][1] += (wr >> 1) * HALF;
  }
#pragma unroll
  for (int ni = 0; ni < 4; ++ni) {
    tr_offsets<256>(ni * 32, lane, toB[ni]);
    toB[ni][0] += A_BYTES + wc * HALF;
    toB[ni][1] += A_BYTES + wc * HALF;
  }
  int rd = 0;
  for (int st = 0; st < nsteps; ++st) {
    wait_vmcnt<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (st + 1 < nsteps) issue(rd ^ 1, pbeg + (st + 2) * BK <= pend);
    const unsigned char* sb = smem + rd * STAGE;
    bf16x8_t af[2][2], bfr[2][4];
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) af[0][mi] = tr_read(sb + toA[mi][0], sb + toA[mi][1]);
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) bfr[0][ni] = tr_read(sb + toB[ni][0], sb + toB[ni][1]);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int cur = kk & 1, nxt = cur ^ 1;
      if constexpr (IL) {
        // the 8 MFMAs of kk interleaved with the 12 transposed reads of kk + 1
        // (as the halo wgrad kernel)
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
#pragma unroll
          for (int ni = 0; ni < 4; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[cur][mi], bfr[cur][ni], acc[mi][ni], 0, 0, 0);
        if (kk + 1 < 4) {
          const int dd = (kk + 1) * 16 * 256;
#pragma unroll
          for (int mi = 0; mi < 2; ++mi)
            af[nxt][mi] = tr_read(sb + toA[mi][0] + dd, sb + toA[mi][1] + dd);
#pragma unroll
          for (int ni = 0; ni < 4; ++ni)
            bfr[nxt][ni] = tr_read(sb + toB[ni][0] + dd, sb + toB[ni][1] + dd);
#pragma unroll
          for (int i = 0; i < 6; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
          }
          __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
      } else {
        if (kk + 1 < 4) {
          const int dd = (kk + 1) * 16 * 256;
#pragma unroll
          for (int mi = 0; mi < 2; ++mi)
            af[nxt][mi] = tr_read(sb + toA[mi][0] + dd, sb + toA[mi][1] + dd);
#pragma unroll
          for (int ni = 0; ni < 4; ++ni)
            bfr[nxt][ni] = tr_read(sb + toB[ni][0] + dd, sb + toB[ni][1] + dd);
        }
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
#pragma unroll
          for (int ni = 0; ni < 4; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[cur][mi], bfr[cur][ni], acc[mi][ni], 0, 0, 0);
      }
    }
    rd ^= 1;
  }

  float* slab = a.slab + static_cast<size_t>(split) * K * 9 * C;
  const int hi = lane >> 5, lr = lane & 31;
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const int n = wc * 128 + ni * 32 + lr;
      int tap = rs, c = c0 + n;
      if constexpr (TPG == 2) { tap = 2 * rs + (n >> 7); c = c0 + (n & 127); }
      if (tap > 8) continue;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int k = k0 + wr * 64 + mi * 32 + (e & 3) + 8 * (e >> 2) + 4 * hi;
        slab[(static_cast<size_t>(k) * 9 + tap) * C + c] = acc[mi][ni][e];
      }
    }
}

// Halo wgrad (16 | W, 64 % W == 0, H*W % 64 == 0: ResNet-9 layer 1 / res1 /
// layer 2): one block per (128 out channels, kernel row r, 64 in channels)
// computes the three taps (r, 0..2) at once -- a 128 x 192 tile, 4 waves of
// 64 x 96.  The three taps of one kernel row read the same input rows shifted
// by one column, so the B operand of a 64-pixel K-step is ONE padded window
// (the step's R = 64 / W image rows at row offset r - 1, each with a zero
// column either side: R * (W + 2) rows of 64 channels), and tap s reads it
// shifted by s rows (16 | W: a 16-pixel MFMA sub-step never leaves an image
// row, so its window rows are consecutive).  Per K-step the block stages
// 16 KB of dy + <= 9.2 KB of window for 24 MFMAs per wave, where the
// per-tap kernel stages 32 KB for 16 (the LDS-DMA issue count bounds those
// loops).  Same transposed reads, swizzles and slab layout as
// conv_wgrad_kernel; K-steps never straddle an image (H*W % 64 == 0).
// Window pieces: rounds 0 and 1 (512 pieces, 64 rows) always, round 2 only
// for waves whose pieces start inside the window (wave-uniform), so a stage
// holds 72 window rows and every wave has >= ALD + 2 DMA loads per stage.
constexpr int kHaloWRows = 72;  // window rows staged per K-step (>= R * (W + 2) > 64)
template <int NSTAGE, bool IL = true, bool ROWS = false>
__global__ void __launch_bounds__(256) conv_wgrad_halo_kernel(ConvWgradArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int A_BYTES = BK * WBM * 2;         // [64 px][128 k], 256-byte rows
  constexpr int B_BYTES = kHaloWRows * 128;     // window [rows][64 c], 128-byte rows
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int ALD = 4, BLD = 3, NLD_MIN = ALD + 2;
  static_assert(NSTAGE == 2 || NSTAGE == 3, "stages");
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int C = a.C, K = a.K, H = a.H, W = a.W, HW = H * W;
  const int ntc = C >> 6;
  const int ntiles = (K / WBM) * 3 * ntc;
  const int tile = bid % ntiles, split = bid / ntiles;
  const int tc = tile % ntc, r = (tile / ntc) % 3, tk = tile / (3 * ntc);
  const int k0 = tk * WBM, c0 = tc * 64, dr = r - 1;
  const int R = BK / W, PW = W + 2, NROW = R * PW;
  // grouped (channel-stacked) x: row stride and this tile's channel group
  const int xs = a.x_stride > 0 ? a.x_stride : C;
  const int cofs = a.kg > 0 ? (k0 / a.kg) * C : 0;
  int pbeg, pend;
  wgrad_split_range(a, split, &pbeg, &pend);
  const int nsteps = pend > pbeg ? (pend - pbeg) / BK : 0;  // whole K-steps (host-checked)
  const uint64_t zero = reinterpret_cast<uint64_t>(g_conv_zero);

  // A pieces: rows of dy (every K-step is full)
  uint64_t a_ptr[ALD];
#pragma unroll
  for (int i = 0; i < ALD; ++i) {
    const int sl = i * 256 + tid;
    const int row = sl >> 4, lc = (sl & 15) ^ sw_tr256(row);
    a_ptr[i] = reinterpret_cast<uint64_t>(a.dy + static_cast<size_t>(pbeg + row) * K + k0 + lc * 8);
  }
  // window pieces: window row -> (image row j of the step, column w); the
  // source pixel is p0 + (j + dr) * W + w when 0 <= h0 + j + dr < H, 0 <= w < W
  int b_rel[BLD], b_jj[BLD];
  uint32_t b_ok = 0;
#pragma unroll
  for (int i = 0; i < BLD; ++i) {
    const int sl = i * 256 + tid;
    const int row = sl >> 3, lc = (sl & 7) ^ sw_tr128(row);
    const int j = row / PW, w = row - j * PW - 1;
    b_jj[i] = j + dr;
    b_rel[i] = (j + dr) * W + w;
    if (row < NROW && w >= 0 && w < W) b_ok |= 1u << i;
    b_rel[i] = b_rel[i] * xs + cofs + c0 + lc * 8;  // element offset from pixel p0's row start
  }

  auto issue = [&](int stage, int p0) __attribute__((always_inline)) {
    unsigned char* base = smem + stage * STAGE + wid * 1024;
#pragma unroll
    for (int i = 0; i < ALD; ++i) {
      glds16(reinterpret_cast<const void*>(a_ptr[i]), base + i * 4096);
      a_ptr[i] += static_cast<uint64_t>(BK) * K * 2;
    }
    const int h0 = (p0 % HW) / W;  // first image row of the step (uniform)
    const uint16_t* xrow = a.x + static_cast<size_t>(p0) * xs;
#pragma unroll
    for (int i = 0; i < BLD; ++i) {
      if (i < 2 || i * 256 + wid * 64 < NROW * 8) {
        const bool ok = ((b_ok >> i) & 1u) && static_cast<unsigned>(h0 + b_jj[i]) < static_cast<unsigned>(H);
        glds16(ok ? reinterpret_cast<const void*>(xrow + b_rel[i]) : reinterpret_cast<const void*>(zero),
               base + A_BYTES + i * 4096);
      }
    }
  };

  f32x16_t acc[2][3];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 3; ++ni)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[mi][ni][e] = 0.f;

  if (nsteps > 0) issue(0, pbeg);
  if (NSTAGE == 3 && nsteps > 1) issue(1, pbeg + BK);
  int toA[2][2];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi) tr_offsets<256>(wr * 64 + mi * 32, lane, toA[mi]);
  // B: column n = wc*96 + ni*32 is tap s = n / 64, channels (n % 64)..+31;
  // sub-step kk's pixels 16kk.. sit in image row j = 16kk / W from column
  // w0 = 16kk % W, so tap s reads window rows j*PW + w0 + s + 0..15
  int offB[4][3][2];
  {
    const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
    const int rowr = 8 * (g >> 1) + q, inb = (pp & 1) * 8;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int l0 = 16 * kk, j = l0 / W, w0 = l0 - j * W;
#pragma unroll
      for (int ni = 0; ni < 3; ++ni) {
        const int n = wc * 96 + ni * 32, sft = n >> 6, cb = n & 63;
        const int chk = (cb + 16 * (g & 1) + 4 * pp) >> 3;
        const int base = j * PW + w0 + sft;
        offB[kk][ni][0] = A_BYTES + tr_off<128>(base + rowr, chk) + inb;
        offB[kk][ni][1] = A_BYTES + tr_off<128>(base + rowr + 4, chk) + inb;
      }
    }
  }
  int rd = 0, wrs = NSTAGE - 1;
  for (int st = 0; st < nsteps; ++st) {
    if constexpr (NSTAGE == 3) {
      // the newest stage's loads may stay in flight (every wave has >= NLD_MIN)
      if (st + 1 < nsteps) wait_vmcnt<NLD_MIN>(); else wait_vmcnt<0>();
    } else {
      wait_vmcnt<0>();
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (st + NSTAGE - 1 < nsteps) issue(wrs, pbeg + (st + NSTAGE - 1) * BK);
    const unsigned char* sb = smem + rd * STAGE;
    bf16x8_t af[2][2], bfr[2][3];
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) af[0][mi] = tr_read(sb + toA[mi][0], sb + toA[mi][1]);
#pragma unroll
    for (int ni = 0; ni < 3; ++ni) bfr[0][ni] = tr_read(sb + offB[0][ni][0], sb + offB[0][ni][1]);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int cur = kk & 1, nxt = cur ^ 1;
      // the 6 MFMAs of sub-step kk interleaved with the 10 transposed reads of
      // kk + 1 (two per MFMA gap; the fragments are double-buffered), so the
      // reads are in flight under the MFMAs instead of waited for in front of
      // each (the compiler's own order: disassembly, profiles/r4_experiments.md)
      if constexpr (IL) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < 3; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[cur][mi], bfr[cur][ni], acc[mi][ni], 0, 0, 0);
      if (kk + 1 < 4) {
        const int da = (kk + 1) * 16 * 256;
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
          af[nxt][mi] = tr_read(sb + toA[mi][0] + da, sb + toA[mi][1] + da);
#pragma unroll
        for (int ni = 0; ni < 3; ++ni)
          bfr[nxt][ni] = tr_read(sb + offB[kk + 1][ni][0], sb + offB[kk + 1][ni][1]);
        if constexpr (IL) {
#pragma unroll
          for (int i = 0; i < 5; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
          }
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        }
      }
      if constexpr (IL) __builtin_amdgcn_sched_barrier(0);
    }
    rd = rd + 1 == NSTAGE ? 0 : rd + 1;
    wrs = wrs + 1 == NSTAGE ? 0 : wrs + 1;
  }

  const int hi = lane >> 5, lr = lane & 31;
  if constexpr (ROWS) {
    // the client rows directly (one split): output channel k is row k / kg's
    // channel k % kg; with rows_sub (64-channel clients in pairs) the tile's
    // 128 x 128 block holds two clients, and only the diagonal 64 x 64 blocks
    // (input block tc == the wave's row half wr) are theirs -- wave-uniform.
    // (A template variant of its own: the headline's slab epilogue keeps its
    // register budget, 2 waves / SIMD.)
    const int sb = a.rows_sub, kg = a.kg;
    const int Cl = sb > 0 ? sb : C;
    if (sb > 0 && tc != wr) return;
    const int half = sb > 0 ? wr : 0;
    const int64_t rowb = sb > 0 ? static_cast<int64_t>(k0 / kg) * (kg / sb) + half : -1;
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int ni = 0; ni < 3; ++ni) {
        const int n = wc * 96 + ni * 32 + lr;
        const int tap = 3 * r + (n >> 6), c = c0 + (n & 63) - half * sb;
#pragma unroll
        for (int e0 = 0; e0 < 16; e0 += 4) {
          // (the old values of a batch loaded before its stores: the mirror may
          // alias the rows as far as the compiler knows)
          float old[4];
          int64_t o[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int e = e0 + q;
            const int k = k0 + wr * 64 + mi * 32 + (e & 3) + 8 * (e >> 2) + 4 * hi;
            const int kl = sb > 0 ? k % sb : k % kg;
            const int64_t row = sb > 0 ? rowb : k / kg;
            const int64_t in = (static_cast<int64_t>(kl) * 9 + tap) * Cl + c;
            o[q] = row * a.rows_ld + in;
            old[q] = a.rows_beta != 0.f
                         ? (a.rows_src != nullptr ? a.rows_src[row * a.rows_sld + in] : a.rows[o[q]])
                         : 0.f;
          }
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float v = a.rows_beta * old[q] + a.rows_alpha * acc[mi][ni][e0 + q];
            a.rows[o[q]] = v;
            if (a.rows_mirror != nullptr) a.rows_mirror[o[q]] = static_cast<uint16_t>(pack_bf16(v, 0.f));
          }
        }
      }
    return;
  }
  float* slab = a.slab + static_cast<size_t>(split) * K * 9 * C;
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 3; ++ni) {
      const int n = wc * 96 + ni * 32 + lr;
      const int tap = 3 * r + (n >> 6), c = c0 + (n & 63);
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int k = k0 + wr * 64 + mi * 32 + (e & 3) + 8 * (e >> 2) + 4 * hi;
        slab[(static_cast<size_t>(k) * 9 + tap) * C + c] = acc[mi][ni][e];
      }
    }
}

// dw[k][c][r][s] (fp32, PyTorch layout) = beta*dw + sum_split slab[split][k][rs][c]
// One block per (k, 64 channels).  Thread (c, part) sums the 9 taps of its
// channel over splits part, part+4, ... (9 independent loads per split, read
// along c: coalesced); the 4 partial sums are combined in a fixed order
// (deterministic) and transposed in LDS, so dw is written as one contiguous
// run of 576 floats.
// Grouped (blockIdx.y = group g): sums the group's own splits [g*splits,
// (g+1)*splits) into dw + g * gstride.
// PARTS = 4 (256 threads) or 16 (1024 threads, many splits: the grid has only
// K * C / 64 blocks -- 128 for ResNet-9 layer 1 -- so more loads in flight per block)
template <int PARTS>
__global__ void __launch_bounds__(64 * PARTS) conv_wgrad_reduce_kernel(const float* __restrict__ slab,
                                                                       float* __restrict__ dw, int K, int C,
                                                                       int splits, float beta,
                                                                       int64_t gstride, int kg, int64_t ld,
                                                                       int rsc, int sub, float alpha,
                                                                       uint16_t* __restrict__ mirror,
                                                                       const float* __restrict__ wsrc,
                                                                       int64_t sld) {
  __shared__ float t[PARTS][64 * 9];
  const int ncb = C >> 6;
  const int k = blockIdx.x / ncb, c0 = (blockIdx.x - k * ncb) * 64;
  // sub > 0: each kernel group of kg channels is kg / sub clients whose weights
  // are the diagonal sub x sub blocks of the group's product (two 64-channel
  // clients computed as one 128-channel group); other blocks are not written
  const int half = sub > 0 ? (k % kg) / sub : 0;
  if (sub > 0 && c0 / sub != half) return;  // block-uniform
  slab += static_cast<size_t>(blockIdx.y) * splits * K * 9 * C;
  dw += static_cast<size_t>(blockIdx.y) * gstride;
  float* const dw_base = dw;
  const int cc = threadIdx.x & 63, part = threadIdx.x >> 6;
  const size_t sstride = static_cast<size_t>(K) * 9 * C;
  const float* src = slab + static_cast<size_t>(k) * 9 * C + c0 + cc;
  float acc[9];
#pragma unroll
  for (int rs = 0; rs < 9; ++rs) acc[rs] = 0.f;
#pragma unroll 2
  for (int sp = part; sp < splits; sp += PARTS) {
    const float* p = src + sp * sstride;
#pragma unroll
    for (int rs = 0; rs < 9; ++rs) acc[rs] += p[rs * C];
  }
#pragma unroll
  for (int rs = 0; rs < 9; ++rs) t[part][cc * 9 + rs] = acc[rs];
  __syncthreads();
  // kg > 0: output channel k is row k % kg of group k / kg's weight, groups
  // ld floats apart (the per-client gradient rows of parallel/fedavg_native.py)
  // rsc: the row in (r, s, c) order ([kg][3][3][C], the engine's layout)
  const int Cl = sub > 0 ? sub : C, c0l = c0 - half * sub;
  float* o = sub > 0 ? dw + static_cast<size_t>((k / kg) * (kg / sub) + half) * ld +
                           static_cast<size_t>((k % kg) % sub) * Cl * 9
             : kg > 0 ? dw + static_cast<size_t>(k / kg) * ld + static_cast<size_t>(k % kg) * C * 9
                      : dw + static_cast<size_t>(k) * C * 9;
  // wsrc: the same element of row `row` of the current weights (sld apart; 0:
  // the server row every client starts from -- no broadcast copy into dw)
  const int64_t row = sub > 0 ? static_cast<int64_t>((k / kg) * (kg / sub) + half) : kg > 0 ? k / kg : 0;
  const float* so = wsrc != nullptr ? wsrc + row * sld + (o - (dw + row * ld)) : nullptr;
  for (int e = threadIdx.x; e < 576; e += 64 * PARTS) {
    const int src = rsc ? (e & 63) * 9 + (e >> 6) : e;
    float v = t[0][src];
#pragma unroll
    for (int q = 1; q < PARTS; ++q) v += t[q][src];  // fixed order: deterministic
    float* oe = rsc ? o + (e >> 6) * Cl + c0l + (e & 63) : o + c0l * 9 + e;
    // alpha / beta: the batched FedAvg clients' SGD step applied in place
    // (w = (1 - lr wd) w - lr g), with the bf16 mirror of the new weight
    const float r = beta != 0.f ? beta * (so != nullptr ? so[oe - o] : *oe) + alpha * v : alpha * v;
    *oe = r;
    if (mirror != nullptr) {
      const uint32_t u = __float_as_uint(r);
      mirror[oe - dw_base] = static_cast<uint16_t>((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
    }
  }
}


void launch_wgrad_reduce(const float* slab, float* dw, int K, int C, int splits, float beta,
                         int64_t gstride, int groups, hipStream_t stream, int kg = 0, int64_t ld = 0,
                         bool rsc = false, int sub = 0, float alpha = 1.f, uint16_t* mirror = nullptr,
                         const float* wsrc = nullptr, int64_t sld = 0) {
  const dim3 grid(K * (C / 64), groups);
  if (splits >= 32)
    COMMEFF_LAUNCH(conv_wgrad_reduce_kernel<16>, grid, dim3(1024), 0, stream, slab, dw, K, C, splits,
                       beta, gstride, kg, ld, rsc ? 1 : 0, sub, alpha, mirror, wsrc, sld);
  else
    COMMEFF_LAUNCH(conv_wgrad_reduce_kernel<4>, grid, dim3(256), 0, stream, slab, dw, K, C, splits,
                       beta, gstride, kg, ld, rsc ? 1 : 0, sub, alpha, mirror, wsrc, sld);
}

// w [K][C][3][3] fp32 -> wf [K][3][3][C] bf16 and wt [C][3][3][K] bf16
// (flipped) for up to kPrepMax tensors in one launch.  A block transposes one
// 32(k) x 32(c) x 9 tile through LDS: the fp32 rows w[k][c0:c0+32][:] are
// 1152 contiguous bytes (coalesced reads), and both outputs are written as
// runs of 32 bf16 (64 B) along their fastest axis.
constexpr int kPT = 32;
__global__ void __launch_bounds__(256) conv_weight_prep_kernel(ConvPrepBatch b) {
  __shared__ float s[kPT][kPT * 9 + 1];  // [k][c*9 + rs], +1: odd row stride
  // pick this block's tensor with compile-time indices only (a dynamically
  // indexed by-value argument struct would be copied to scratch)
  ConvPrepItem it = b.t[0];
#pragma unroll
  for (int i = 1; i < kPrepMax; ++i)
    if (i < b.n && static_cast<int>(blockIdx.x) >= b.t[i].block0) it = b.t[i];
  const int tile = blockIdx.x - it.block0;
  const int ntc = (it.C + kPT - 1) / kPT;
  const int k0 = (tile / ntc) * kPT, c0 = (tile % ntc) * kPT;
  const int nk = min(kPT, it.K - k0), nc = min(kPT, it.C - c0);
  const int row = nc * 9;
  // all 36 loads of a thread in flight before the first LDS store
  constexpr int PER = kPT * kPT * 9 / 256;
  float v[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int e = i * 256 + threadIdx.x;
    const int kk = e / (kPT * 9), j = e - kk * (kPT * 9);
    v[i] = (kk < nk && j < row) ? it.w[(static_cast<size_t>(k0 + kk) * it.C + c0) * 9 + j] : 0.f;
  }
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int e = i * 256 + threadIdx.x;
    const int kk = e / (kPT * 9), j = e - kk * (kPT * 9);
    s[kk][j] = v[i];
  }
  __syncthreads();
  if (it.wf != nullptr) {  // wf[k][rs][c]: lanes run along c
    for (int e = threadIdx.x; e < kPT * 9 * kPT; e += 256) {
      const int cc = e % kPT, krs = e / kPT, rs = krs % 9, kk = krs / 9;
      if (kk < nk && cc < nc)
        reinterpret_cast<__bf16*>(it.wf)[(static_cast<size_t>(k0 + kk) * 9 + rs) * it.C + c0 + cc] =
            static_cast<__bf16>(s[kk][cc * 9 + rs]);
    }
  }
  if (it.wt != nullptr) {  // wt[c][rs'][k] = w[k][c][8 - rs']: lanes run along k
    for (int e = threadIdx.x; e < kPT * 9 * kPT; e += 256) {
      const int kk = e % kPT, crs = e / kPT, rs = crs % 9, cc = crs / 9;
      if (kk < nk && cc < nc)
        reinterpret_cast<__bf16*>(it.wt)[(static_cast<size_t>(c0 + cc) * 9 + rs) * it.K + k0 + kk] =
            static_cast<__bf16>(s[kk][cc * 9 + 8 - rs]);
    }
  }
}

// g = gy where y > 0 else 0  (bf16, 8 per thread)
__global__ void __launch_bounds__(256) relu_mask_kernel(const v4u* __restrict__ gy,
                                                        const v4u* __restrict__ y,
                                                        v4u* __restrict__ g, int64_t n8) {
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n8; i += static_cast<int64_t>(gridDim.x) * 256) {
    const v4u av = gy[i], mv = y[i];
    v4u o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      uint32_t r = 0;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uint32_t mb = (mv[j] >> (16 * h)) & 0xffffu;
        if (!(mb & 0x8000u) && mb != 0u) r |= av[j] & (0xffffu << (16 * h));
      }
      o[j] = r;
    }
    g[i] = o;
  }
}

int grid_for(int64_t n, int per_block) {
  int64_t b = (n + per_block - 1) / per_block;
  if (b > 16384) b = 16384;
  return static_cast<int>(b < 1 ? 1 : b);
}

// the wide (256 x 256) wgrad kernel: K a multiple of 256, C = 128 (tap pairs)
// or a multiple of 256
bool wgrad_wide(int K, int C) { return K % 256 == 0 && (C == 128 || C % 256 == 0); }

// the halo wgrad kernel (three taps of a kernel row per block): 16 | W,
// 64 % W == 0 and whole K-steps per image
bool wgrad_halo(int H, int W, int K, int C) {
  return W % 16 == 0 && BK % W == 0 && (H * W) % BK == 0 && K % WBM == 0 && C % 64 == 0 &&
         (BK / W) * (W + 2) <= kHaloWRows;
}


// (k, c) x tap-group tiles of one wgrad: 64-channel inputs pair taps (PAIR)
int wgrad_tiles(int K, int C) {
  if (wgrad_wide(K, C)) return (K / 256) * (C == 128 ? 5 : 9 * (C / 256));
  if (C == 64) return (K / WBM) * 5;
  return (K / WBM) * 9 * (C / (C % 128 == 0 ? 128 : 64));
}

void set_lds(const void* fn, int bytes) {
  (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}

template <int TBM, int BN, int NSTAGE, bool POOL = false>
void launch_fwd(const ConvFwdArgs& a, hipStream_t stream) {
  constexpr int lds_pipe = NSTAGE * (TBM * 128 + BN * 128);
  constexpr int lds_epi = (TBM > 128 ? 128 : TBM) * (BN + 4) * 4;
  constexpr int lds = lds_pipe > lds_epi ? lds_pipe : lds_epi;
  static bool init = false;
  if (!init) {
    set_lds(reinterpret_cast<const void*>(conv_fwd_kernel<TBM, BN, NSTAGE, POOL>), lds);
    init = true;
  }
  const int mt = (a.P + TBM - 1) / TBM;
  COMMEFF_LAUNCH((conv_fwd_kernel<TBM, BN, NSTAGE, POOL>), dim3(mt * (a.K / BN)), dim3(TBM * 2),
                     lds, stream, a);
}

template <int BN, int NSTAGE, bool ROWSTEP, bool PAIR = false>
void launch_wgrad(const ConvWgradArgs& a, hipStream_t stream) {
  constexpr int lds = NSTAGE * (BK * WBM * 2 + BK * BN * 2);
  static bool init = false;
  if (!init) {
    set_lds(reinterpret_cast<const void*>(conv_wgrad_kernel<BN, NSTAGE, ROWSTEP, PAIR>), lds);
    init = true;
  }
  const int tiles = wgrad_tiles(a.K, a.C);
  COMMEFF_LAUNCH((conv_wgrad_kernel<BN, NSTAGE, ROWSTEP, PAIR>), dim3(tiles * a.splits), dim3(256),
                     lds, stream, a);
}

}  // namespace

// channel-stacked grouped wgrad: the halo kernel with its tile's input-channel
// group (output tiles of WBM = 128 rows never straddle a group)
bool conv3x3_wgrad_grouped_supported(int H, int W, int K, int C, int kg) {
  if (kg <= 0 || K % kg != 0 || C % 64 != 0) return false;
  if (wgrad_halo(H, W, K, C)) return kg % WBM == 0;
  // the wide kernel (any image width): its 256-row tiles must not straddle a group
  return kg % 256 == 0 && wgrad_wide(K, C);
}

static int wgrad_slots();


bool conv3x3_supported(int C, int K) { return C % 64 == 0 && K % 64 == 0 && C >= 64 && K >= 64; }

bool conv3x3_pool_supported(int H, int W, int K) {
  return K % 128 == 0 && H % 2 == 0 && W % 2 == 0 && 128 % (2 * W) == 0;
}

// halo-window geometry of a 128-pixel tile (false: not whole image rows, or
// the padded window exceeds 288 rows)
static int wgrad_slots();

bool halo_geom(int H, int W, int K, int TBM, HaloGeom* g, int BN = 128) {
  if (K % BN != 0 || W <= 0 || TBM % W != 0) return false;
  const int R = TBM / W;
  if (R <= H) {
    if (H % R != 0) return false;
    g->G = 1;
    g->Rg = R;
  } else {
    if (R % H != 0) return false;
    g->G = R / H;
    g->Rg = H;
  }
  g->PW = W + 2;
  g->PR = g->G * (g->Rg + 1) + 1;
  g->NPW = g->PR * g->PW;
  // window swizzle per tile width (see sw_halo); other widths: the flat-row
  // swizzle (row >> 1) & 7, which is swa = PW / 2 for an even PW
  g->swa = (g->PW / 2) & 7;
  g->swb = 0;
  if (W == 16) g->swa = 0;
  if (W == 8) g->swa = 4;
  if (W == 4) { g->swa = 2; g->swb = 4; }
  // (ResNet-9 res3, W = 4: 288 padded rows for 128 pixels -- slower alone in
  // scripts/bench_conv.py, but faster inside the round: bench 222-223k with a
  // 256-row cap vs 224-227k with 288, profiles/r1_experiments.md)
  return g->NPW <= (TBM == 256 ? HaloCfg<256>::kMaxRows : HaloCfg<128>::kMaxRows);
}

template <int TBM, bool POOL, bool SPLIT = false, int BN = 128, bool BT = false>
void launch_fwd_halo(const ConvFwdArgs& a, const HaloGeom& hg, hipStream_t stream) {
  constexpr int lds = halo_lds<TBM, BN>() * (SPLIT ? 2 : 1);
  static bool init = false;
  if (!init) {
    set_lds(reinterpret_cast<const void*>(conv_fwd_halo_kernel<TBM, POOL, SPLIT, BN, BT>), lds);
    init = true;
  }
  const int mt = (a.P + TBM - 1) / TBM;
  COMMEFF_LAUNCH((conv_fwd_halo_kernel<TBM, POOL, SPLIT, BN, BT>), dim3(mt * (a.K / BN)),
                 dim3(TBM * 2 * (SPLIT ? 2 : 1)), lds, stream, a, hg);
}

// Grouped conv on channel-stacked images (a.kg, a.x_stride set): the halo
// kernels only, no fused epilogue.  Returns false when the geometry has no
// halo tiling (the caller falls back to a stock grouped convolution).
bool launch_conv3x3_fwd_grouped(ConvFwdArgs a, hipStream_t stream) {
  // (the residual addend epilogue reads [P, K] like the output: the batched
  // FedAvg block's input gradient = dgrad + the identity shortcut's gradient)
  if (a.kg <= 0 || a.pool != 0 || a.relu != 0 || a.mask != nullptr || a.y_pre != nullptr ||
      a.unpool_idx != nullptr || a.dual_mask != nullptr || a.C % 64 != 0 || a.K % a.kg != 0)
    return false;
  a.div_w = make_fastdiv(static_cast<uint32_t>(a.W));
  a.div_h = make_fastdiv(static_cast<uint32_t>(a.H));
  HaloGeom hg;
  if (a.w_bt) {  // input gradient from the conv's own weight rows (transposed B)
    if (a.w_gs == 0) return false;
    if (a.kg % 128 == 0) {
      if (halo_geom(a.H, a.W, a.K, 256, &hg)) { launch_fwd_halo<256, false, false, 128, true>(a, hg, stream); return true; }
      if (halo_geom(a.H, a.W, a.K, 128, &hg)) { launch_fwd_halo<128, false, false, 128, true>(a, hg, stream); return true; }
      return false;
    }
    if (a.kg % 64 == 0 && halo_geom(a.H, a.W, a.K, 256, &hg, 64)) {
      launch_fwd_halo<256, false, false, 64, true>(a, hg, stream);
      return true;
    }
    return false;
  }
  if (a.kg % 128 == 0) {
    if (halo_geom(a.H, a.W, a.K, 256, &hg)) { launch_fwd_halo<256, false>(a, hg, stream); return true; }
    if (halo_geom(a.H, a.W, a.K, 128, &hg)) { launch_fwd_halo<128, false>(a, hg, stream); return true; }
    return false;
  }
  if (a.kg % 64 == 0 && halo_geom(a.H, a.W, a.K, 256, &hg, 64)) {
    launch_fwd_halo<256, false, false, 64>(a, hg, stream);
    return true;
  }
  return false;
}

// cross-block split-K of the 128-pixel halo tiles (KS above): when the grid
// has at most a quarter of the resident slots in tiles, each tile's channel
// blocks are split over S blocks (S a power of two dividing them, tiles x S
// within the slots)
static int fwd_ksplit(const ConvFwdArgs& a) {
  HaloGeom hg;
  if (a.kg != 0 || a.w_bt != 0) return 1;
  if (halo_geom(a.H, a.W, a.K, 256, &hg) &&
      static_cast<int64_t>((a.P + 255) / 256) * (a.K / 128) * 10 >= wgrad_slots() * 9)
    return 1;  // (the 256-pixel path)
  if (!halo_geom(a.H, a.W, a.K, 128, &hg)) return 1;
  const int64_t tiles = static_cast<int64_t>((a.P + 127) / 128) * (a.K / 128);
  const int ncb = a.C / 64;
  if (tiles * 4 > wgrad_slots()) return 1;
  int S = 1;
  while (ncb % (2 * S) == 0 && tiles * 2 * S <= wgrad_slots()) S *= 2;
  return S >= 4 ? S : 1;
}

int64_t conv3x3_fwd_split_floats(const ConvFwdArgs& a) {
  const int S = fwd_ksplit(a);
  if (S <= 1) return 0;
  return static_cast<int64_t>((a.P + 127) / 128) * (a.K / 128) * (S + 1) * 128 * 128;
}

template <bool POOL>
static void launch_fwd_ksplit(const ConvFwdArgs& a, const HaloGeom& hg, hipStream_t stream) {
  constexpr int lds = halo_lds<128, 128>(), epi = 128 * (128 + 4) * 4;
  static bool init = false;
  if (!init) {
    set_lds(reinterpret_cast<const void*>(conv_fwd_halo_kernel<128, POOL, false, 128, false, true>), lds);
    set_lds(reinterpret_cast<const void*>(conv_fwd_combine_kernel<128, POOL, 128>), epi);
    init = true;
  }
  const int tiles = ((a.P + 127) / 128) * (a.K / 128);
  COMMEFF_LAUNCH((conv_fwd_halo_kernel<128, POOL, false, 128, false, true>), dim3(tiles * a.ksplit), dim3(256), lds,
                 stream, a, hg);
  // splits summed chip-wide into the tile buffer behind the partials, then the
  // epilogue from the summed tile
  constexpr int n4 = 128 * 128 / 4;
  ConvFwdArgs b = a;
  b.part = a.part + static_cast<size_t>(tiles) * a.ksplit * 128 * 128;
  b.ksplit = 1;
  COMMEFF_LAUNCH(conv_fwd_psum_kernel, dim3((tiles * n4 + 255) / 256), dim3(256), 0, stream,
                 static_cast<const float*>(a.part), b.part, tiles, a.ksplit, n4);
  COMMEFF_LAUNCH((conv_fwd_combine_kernel<128, POOL, 128>), dim3(tiles), dim3(256), epi, stream, b);
}

void launch_conv3x3_fwd(ConvFwdArgs a, hipStream_t stream) {
  a.div_w = make_fastdiv(static_cast<uint32_t>(a.W));
  a.div_h = make_fastdiv(static_cast<uint32_t>(a.H));
  HaloGeom hg;
  const int ks = fwd_ksplit(a);
  if (ks > 1) {
    if (a.part == nullptr) throw std::runtime_error("conv3x3_fwd: split-K workspace not set");
    a.ksplit = ks;
    (void)halo_geom(a.H, a.W, a.K, 128, &hg);
    if (a.pool == 2) launch_fwd_ksplit<true>(a, hg, stream); else launch_fwd_ksplit<false>(a, hg, stream);
    return;
  }
  // 256-pixel tiles when they still give ~every resident slot (2 per CU) a block
  if (halo_geom(a.H, a.W, a.K, 256, &hg) &&
      static_cast<int64_t>((a.P + 255) / 256) * (a.K / 128) * 10 >= wgrad_slots() * 9) {
    if (a.pool == 2) launch_fwd_halo<256, true>(a, hg, stream); else launch_fwd_halo<256, false>(a, hg, stream);
    return;
  }
  if (halo_geom(a.H, a.W, a.K, 128, &hg)) {
    const int64_t tiles = static_cast<int64_t>((a.P + 127) / 128) * (a.K / 128);
    if ((a.C / 64) % 2 == 0 && tiles * 2 <= wgrad_slots()) {
      if (a.pool == 2) launch_fwd_halo<128, true, true>(a, hg, stream); else launch_fwd_halo<128, false, true>(a, hg, stream);
      return;
    }
    if (a.pool == 2) launch_fwd_halo<128, true>(a, hg, stream); else launch_fwd_halo<128, false>(a, hg, stream);
    return;
  }
  // 64-wide outputs of big layers (ResNet-9 layer-1 dgrad): the halo window
  // replaces 9 staged 256 x 64 A tiles per channel block (the per-tap kernel
  // streams ~3x the L2 bytes per MFMA)
  if (a.pool == 0 && a.K % 128 != 0 &&
      halo_geom(a.H, a.W, a.K, 256, &hg, 64) &&
      static_cast<int64_t>((a.P + 255) / 256) * (a.K / 64) >= 512) {
    launch_fwd_halo<256, false, false, 64>(a, hg, stream);
    return;
  }
  if (a.pool == 2) {  // caller checked conv3x3_pool_supported
    launch_fwd<128, 128, 2, true>(a, stream);
    return;
  }
  const bool wide = a.K % 128 == 0;
  const int bn = wide ? 128 : 64;
  // measured (scripts/bench_conv.py sweep, profiles/r1_conv_tile_sweep.txt):
  // occupancy beats ring depth -- 128-pixel tiles with a 2-stage ring (2
  // blocks/CU) everywhere, except 64-wide outputs of big layers, where 256
  // pixels x 64 (8 waves, 2 stages) amortises the A operand better
  const bool big = static_cast<int64_t>((a.P + 255) / 256) * (a.K / bn) >= 512;
  if (!wide && big) {
    launch_fwd<256, 64, 2>(a, stream);
  } else {
    if (wide) launch_fwd<128, 128, 2>(a, stream); else launch_fwd<128, 64, 2>(a, stream);
  }
}

// resident wgrad blocks per CU (64 KB LDS, 88 VGPRs: 2 blocks) x CUs
static int wgrad_slots() {
  static const int slots = [] {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) {
      hipDeviceProp_t prop;
      if (hipGetDeviceProperties(&prop, dev) == hipSuccess && prop.multiProcessorCount > 0)
        cus = prop.multiProcessorCount;
    }
    return 2 * cus;
  }();
  return slots;
}

template <bool ROWSTEP>
void launch_wgrad_wide(const ConvWgradArgs& a, hipStream_t stream) {
  constexpr int lds = 2 * 4 * BK * 128 * 2;
  const int tiles = wgrad_tiles(a.K, a.C);
  // (the halo wgrad's MFMA / read interleave measured slower here: res3
  // 60.8 -> 65.4 us, layer 3 equal; profiles/r4_experiments.md)
  if (a.C == 128) {
    static bool init = false;
    if (!init) {
      set_lds(reinterpret_cast<const void*>(conv_wgrad_wide_kernel<ROWSTEP, 2, false>), lds);
      init = true;
    }
    COMMEFF_LAUNCH((conv_wgrad_wide_kernel<ROWSTEP, 2, false>), dim3(tiles * a.splits), dim3(512), lds, stream, a);
  } else {
    static bool init = false;
    if (!init) {
      set_lds(reinterpret_cast<const void*>(conv_wgrad_wide_kernel<ROWSTEP, 1, false>), lds);
      init = true;
    }
    COMMEFF_LAUNCH((conv_wgrad_wide_kernel<ROWSTEP, 1, false>), dim3(tiles * a.splits), dim3(512), lds, stream, a);
  }
}

int conv3x3_wgrad_splits(int P, int H, int W, int K, int C) {
  const int steps = (P + BK - 1) / BK;
  if (wgrad_halo(H, W, K, C)) {  // 2 blocks per CU (56 KB LDS), >= 16 K-steps each
    const int tiles = (K / WBM) * 3 * (C / 64);
    int s = wgrad_slots() / tiles;
    if (s > steps / 16) s = steps / 16;
    return s < 1 ? 1 : s;
  }
  const int tiles = wgrad_tiles(K, C);
  if (wgrad_wide(K, C)) {  // one 128 KB block per CU, >= 16 K-steps each
    int s = wgrad_slots() / 2 / tiles;
    if (s > steps / 16) s = steps / 16;
    return s < 1 ? 1 : s;
  }
  // every block resident at once (equal-work blocks: one block past the
  // resident slots costs a whole extra block time), >= 32 K-steps each
  int s = wgrad_slots() / tiles;
  if (s > steps / 32) s = steps / 32;
  return s < 1 ? 1 : s;
}

void launch_conv3x3_wgrad_steps(ConvWgradArgs a, int steps_per_split, hipStream_t stream);



void launch_conv3x3_wgrad(ConvWgradArgs a, float* dw, float beta, hipStream_t stream) {
  const int steps = (a.P + BK - 1) / BK;
  a.group_px = 0;
  launch_conv3x3_wgrad_steps(a, (steps + a.splits - 1) / a.splits, stream);
  launch_wgrad_reduce(a.slab, dw, a.K, a.C, a.splits, beta, int64_t{0}, 1, stream);
}

// channel-stacked grouped wgrad written straight into per-group rows: output
// channel k of group k / kg at dst + (k / kg) * ld + (k % kg) * 9 C
void launch_conv3x3_wgrad_rows(ConvWgradArgs a, float* dst, int kg, int64_t ld, bool rsc, hipStream_t stream,
                               int sub, float beta, float alpha, uint16_t* mirror, const float* wsrc,
                               int64_t sld) {
  const int steps = (a.P + BK - 1) / BK;
  a.group_px = 0;
  if (a.splits == 1 && rsc && wgrad_halo(a.H, a.W, a.K, a.C) && static_cast<int>(a.kg) == kg) {
    // one split: the halo kernel's epilogue updates the rows (no slab, no
    // reduction pass: 8 fewer bytes per weight; FedAvg round 31.46 -> 31.32 ms,
    // same-box A/B)
    a.rows = dst;
    a.rows_ld = ld;
    a.rows_sub = sub;
    a.rows_beta = beta;
    a.rows_alpha = alpha;
    a.rows_mirror = mirror;
    a.rows_src = wsrc;
    a.rows_sld = sld;
    launch_conv3x3_wgrad_steps(a, steps, stream);
    return;
  }
  launch_conv3x3_wgrad_steps(a, (steps + a.splits - 1) / a.splits, stream);
  launch_wgrad_reduce(a.slab, dst, a.K, a.C, a.splits, beta, int64_t{0}, 1, stream, kg, ld, rsc, sub, alpha,
                      mirror, wsrc, sld);
}

// the wgrad GEMM kernels (slabs only) with a given split length
void launch_conv3x3_wgrad_steps(ConvWgradArgs a, int steps_per_split, hipStream_t stream) {
  a.steps_per_split = steps_per_split;
  a.div_w = make_fastdiv(static_cast<uint32_t>(a.W));
  a.div_h = make_fastdiv(static_cast<uint32_t>(a.H));
  const bool rowstep = BK % a.W == 0;
  const bool wide = a.C % 128 == 0;
  if (wgrad_halo(a.H, a.W, a.K, a.C) && (a.group_px == 0 || a.group_px % BK == 0)) {
    // (a 3-stage ring -- 3 x 25 KB still fits 2 blocks/CU -- measured equal to
    // 2 in the ResNet-9 round)
    const int tiles = (a.K / WBM) * 3 * (a.C / 64);
    constexpr int stage_bytes = BK * WBM * 2 + kHaloWRows * 128;
    static bool init = false;
    if (!init) {
      set_lds(reinterpret_cast<const void*>(conv_wgrad_halo_kernel<2>), 2 * stage_bytes);
      set_lds(reinterpret_cast<const void*>(conv_wgrad_halo_kernel<2, true, true>), 2 * stage_bytes);
      init = true;
    }
    if (a.rows != nullptr)  // one split, the rows updated in the epilogue
      COMMEFF_LAUNCH((conv_wgrad_halo_kernel<2, true, true>), dim3(tiles), dim3(256), 2 * stage_bytes, stream, a);
    else
      COMMEFF_LAUNCH((conv_wgrad_halo_kernel<2>), dim3(tiles * a.splits), dim3(256), 2 * stage_bytes, stream, a);
  } else if (wgrad_wide(a.K, a.C)) {
    if (rowstep) launch_wgrad_wide<true>(a, stream); else launch_wgrad_wide<false>(a, stream);
  } else if (a.C == 64) {  // tap pairs: 128-wide tiles (measured 158 -> see profiles/r1_experiments.md)
    if (rowstep) launch_wgrad<128, 2, true, true>(a, stream); else launch_wgrad<128, 2, false, true>(a, stream);
  } else if (rowstep) {
    if (wide) launch_wgrad<128, 2, true>(a, stream); else launch_wgrad<64, 2, true>(a, stream);
  } else {
    if (wide) launch_wgrad<128, 2, false>(a, stream); else launch_wgrad<64, 2, false>(a, stream);
  }
}

void launch_conv3x3_wgrad_grouped(ConvWgradArgs a, int G, float* dw, int64_t gstride, float beta,
                                  hipStream_t stream) {
  // one launch for every group's splits (each split's pixel range inside its
  // group), then one per-group reduction
  a.group_px = a.P / G;
  a.splits_per_group = a.splits / G;
  const int steps = (a.group_px + BK - 1) / BK;
  launch_conv3x3_wgrad_steps(a, (steps + a.splits_per_group - 1) / a.splits_per_group, stream);
  launch_wgrad_reduce(a.slab, dw, a.K, a.C, a.splits_per_group, beta, gstride, G, stream);
}

namespace {
__global__ void __launch_bounds__(256) conv_images_patch_kernel(ConvPatchBatch b, const int64_t* __restrict__ idx,
                                                                int64_t k) {
  const int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (e >= k) return;
  const int64_t i = idx[e];
  // the weight holding coordinate i (compile-time indices only: a dynamically
  // indexed by-value argument array would be copied to scratch)
  int64_t local = -1;
  uint16_t *wf = nullptr, *wt = nullptr;
  int K = 0, C = 0;
#pragma unroll
  for (int j = 0; j < kPrepMax; ++j) {
    if (j < b.n && i >= b.off[j] && i < b.off[j] + b.numel[j]) {
      local = i - b.off[j];
      wf = b.wf[j];
      wt = b.wt[j];
      K = b.K[j];
      C = b.C[j];
    }
  }
  if (local < 0) return;  // not a conv weight with images
  const int rs = static_cast<int>(local % 9);
  const int64_t kc = local / 9;
  const int c = static_cast<int>(kc % C), kk = static_cast<int>(kc / C);
  const __bf16 v = static_cast<__bf16>(b.w_flat[i]);
  reinterpret_cast<__bf16*>(wf)[(static_cast<size_t>(kk) * 9 + rs) * C + c] = v;
  reinterpret_cast<__bf16*>(wt)[(static_cast<size_t>(c) * 9 + 8 - rs) * K + kk] = v;
}
}  // namespace

void launch_conv_images_patch(const ConvPatchBatch& b, const int64_t* idx, int64_t k,
                              hipStream_t stream) {
  if (k <= 0 || b.n <= 0) return;
  COMMEFF_LAUNCH(conv_images_patch_kernel, dim3(static_cast<uint32_t>((k + 255) / 256)), dim3(256), 0,
                     stream, b, idx, k);
}

void launch_conv_weight_prep(ConvPrepBatch b, hipStream_t stream) {
  int blocks = 0;
  for (int i = 0; i < b.n; ++i) {
    b.t[i].block0 = blocks;
    blocks += ((b.t[i].K + kPT - 1) / kPT) * ((b.t[i].C + kPT - 1) / kPT);
  }
  if (blocks == 0) return;
  COMMEFF_LAUNCH(conv_weight_prep_kernel, dim3(blocks), dim3(256), 0, stream, b);
}

void launch_relu_mask(const uint16_t* gy, const uint16_t* y, uint16_t* g, int64_t n,
                      hipStream_t stream) {
  const int64_t n8 = n / 8;
  COMMEFF_LAUNCH(relu_mask_kernel, dim3(grid_for(n8, 256)), dim3(256), 0, stream,
                     reinterpret_cast<const v4u*>(gy), reinterpret_cast<const v4u*>(y),
                     reinterpret_cast<v4u*>(g), n8);
}

}  // namespace commeff
