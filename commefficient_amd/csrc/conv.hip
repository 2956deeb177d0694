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
// Forward/dgrad kernel (`conv_fwd_kernel<BN>`): GEMM M = pixels, N = output
// channels, K = 9*C.  Both operands are K-contiguous (NHWC activation rows,
// [k][r][s][c] weight rows), so a 128 x BN x 64 tile is staged through LDS with
// 16-byte loads (register-staged double buffer, one barrier per K-step) and
// read back with ds_read_b128 in the exact 32x32x16 operand layout.  The
// epilogue goes through an fp32 LDS tile for coalesced 16-byte stores and
// fuses ReLU, a ReLU-mask by another tensor (y = 0 where mask <= 0) and a
// residual addend.
//
// Wgrad kernel (`conv_wgrad_kernel<BN>`): GEMM M = out channels, N = in
// channels (one (r,s) per tile), K = pixels.  The reduction runs over the
// row index of both NHWC images, so the operands are read with the gfx950
// transposing LDS read ds_read_b64_tr_b16 from XOR-swizzled images.  K is
// split over blocks; every split writes an fp32 slab and a second kernel sums
// the slabs in a fixed order (deterministic) into PyTorch's [K][C][3][3].
//
// Tile -> block mapping is XCD-aware: consecutive logical tiles (which share
// activation rows / halos in L2) are placed on the same XCD.
#include <hip/hip_runtime.h>
#include <cstdint>
#include "kernels.h"

namespace commeff {
namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef short s16x8_t __attribute__((ext_vector_type(8)));
typedef uint32_t v4u __attribute__((ext_vector_type(4)));

constexpr int BM = 128;  // fwd: pixels per tile ; wgrad: out channels per tile
constexpr int BK = 64;   // K-step

__device__ __forceinline__ float bf2f(uint32_t h) { return __uint_as_float(h << 16); }
__device__ __forceinline__ uint32_t f2bf(float f) {  // round to nearest even
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u) return (u >> 16) | ((u & 0xffffu) ? 0x40u : 0u);
  u += 0x7fffu + ((u >> 16) & 1u);
  return u >> 16;
}

// bijective XCD remap: blocks dispatched round-robin over 8 XCDs; logical
// tiles l and l+1 land on the same XCD
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// 128-byte rows (64 bf16), 16-byte chunk ch (0..7): conflict-free ds_read_b128
// of 16 consecutive rows at one logical chunk
__device__ __forceinline__ int off128(int row, int ch) {
  return row * 128 + ((ch ^ ((row >> 1) & 7)) << 4);
}

// ------------------------------------------------------------ fwd / dgrad
template <int BN>
__global__ void __launch_bounds__(256, 2) conv_fwd_kernel(ConvFwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int A_BYTES = BM * BK * 2;
  constexpr int B_BYTES = BN * BK * 2;
  constexpr int BUF = A_BYTES + B_BYTES;
  constexpr int NI = BN / 64;      // 32-col MFMA tiles per wave (wave tile 64 x BN/2)
  constexpr int BROWS = BN / 32;   // B rows staged per thread

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int ntn = a.K / BN;
  const int tn = bid % ntn, tm = bid / ntn;
  const int m0 = tm * BM, n0 = tn * BN;
  const int C = a.C, H = a.H, W = a.W;
  const int CB = C >> 6;  // 64-channel blocks per (r, s)
  const int KT = 9 * CB;

  // A rows staged by this thread: (tid >> 3) + 32 i, chunk tid & 7
  const int ch = tid & 7;
  int pix[4], ph[4], pw[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int p = m0 + (tid >> 3) + 32 * i;
    pix[i] = p < a.P ? p : -1;
    const int q = p / W;
    pw[i] = p - q * W;
    ph[i] = q % H;
  }
  const uint16_t* wbase = a.w + static_cast<size_t>(n0) * 9 * C + ch * 8;

  v4u ra[4], rb[BROWS];
  auto gload = [&](int kr, int ks, int cb) __attribute__((always_inline)) {
    const int dr = kr - 1, ds = ks - 1;
    const int coff = cb * 64 + ch * 8;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int hh = ph[i] + dr, ww = pw[i] + ds;
      const bool ok = pix[i] >= 0 && static_cast<unsigned>(hh) < static_cast<unsigned>(H) &&
                      static_cast<unsigned>(ww) < static_cast<unsigned>(W);
      v4u v = {0u, 0u, 0u, 0u};
      if (ok) {
        const int sp = pix[i] + dr * W + ds;
        v = *reinterpret_cast<const v4u*>(a.x + static_cast<size_t>(sp) * C + coff);
      }
      ra[i] = v;
    }
    const int koff = (kr * 3 + ks) * C + cb * 64;
#pragma unroll
    for (int j = 0; j < BROWS; ++j) {
      const int row = (tid >> 3) + 32 * j;
      rb[j] = *reinterpret_cast<const v4u*>(wbase + static_cast<size_t>(row) * 9 * C + koff);
    }
  };
  auto sstore = [&](int buf) __attribute__((always_inline)) {
    unsigned char* sA = smem + buf * BUF;
    unsigned char* sB = sA + A_BYTES;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = (tid >> 3) + 32 * i;
      *reinterpret_cast<v4u*>(sA + off128(row, ch)) = ra[i];
    }
#pragma unroll
    for (int j = 0; j < BROWS; ++j) {
      const int row = (tid >> 3) + 32 * j;
      *reinterpret_cast<v4u*>(sB + off128(row, ch)) = rb[j];
    }
  };

  f32x16_t acc[2][NI];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[mi][ni][e] = 0.f;

  int kr = 0, ks = 0, cb = 0;
  gload(0, 0, 0);
  sstore(0);
  __syncthreads();
  const int hi = lane >> 5, lr = lane & 31;
  for (int kt = 0; kt < KT; ++kt) {
    // next K-step's operands -> registers (in flight during the MFMAs)
    const bool more = kt + 1 < KT;
    if (more) {
      if (++cb == CB) {
        cb = 0;
        if (++ks == 3) { ks = 0; ++kr; }
      }
      gload(kr, ks, cb);
    }
    const unsigned char* sA = smem + (kt & 1) * BUF;
    const unsigned char* sB = sA + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int chk = 2 * kk + hi;
      bf16x8_t af[2], bfr[NI];
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
        af[mi] = *reinterpret_cast<const bf16x8_t*>(sA + off128(wr * 64 + mi * 32 + lr, chk));
#pragma unroll
      for (int ni = 0; ni < NI; ++ni)
        bfr[ni] = *reinterpret_cast<const bf16x8_t*>(sB + off128(wc * (BN / 2) + ni * 32 + lr, chk));
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[mi], bfr[ni], acc[mi][ni], 0, 0, 0);
    }
    if (more) sstore((kt + 1) & 1);
    __syncthreads();
  }

  // ---- epilogue: fp32 tile in LDS -> fused ops -> 16-byte bf16 stores
  constexpr int LD = BN + 4;
  float* ct = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = wr * 64 + mi * 32 + (e & 3) + 8 * (e >> 2) + 4 * hi;
        const int col = wc * (BN / 2) + ni * 32 + lr;
        ct[row * LD + col] = acc[mi][ni][e];
      }
  __syncthreads();
  constexpr int CPR = BN / 8;  // 16-byte chunks per row
  for (int e = tid; e < BM * CPR; e += 256) {
    const int row = e / CPR, cc = e - row * CPR;
    const int p = m0 + row;
    if (p >= a.P) continue;
    const float4 lo = *reinterpret_cast<const float4*>(ct + row * LD + cc * 8);
    const float4 hi4 = *reinterpret_cast<const float4*>(ct + row * LD + cc * 8 + 4);
    float v[8] = {lo.x, lo.y, lo.z, lo.w, hi4.x, hi4.y, hi4.z, hi4.w};
    const size_t o = static_cast<size_t>(p) * a.K + n0 + cc * 8;
    if (a.relu) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = fmaxf(v[j], 0.f);
    }
    if (a.mask != nullptr) {
      const uint4 m = *reinterpret_cast<const uint4*>(a.mask + o);
      const uint32_t mw[4] = {m.x, m.y, m.z, m.w};
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t hb = (mw[j >> 1] >> (16 * (j & 1))) & 0xffffu;
        // bf16 > 0: sign bit clear and not +0
        if ((hb & 0x8000u) || hb == 0u) v[j] = 0.f;
      }
    }
    if (a.addend != nullptr) {
      const uint4 m = *reinterpret_cast<const uint4*>(a.addend + o);
      const uint32_t mw[4] = {m.x, m.y, m.z, m.w};
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += bf2f((mw[j >> 1] >> (16 * (j & 1))) & 0xffffu);
    }
    uint4 out;
    out.x = f2bf(v[0]) | (f2bf(v[1]) << 16);
    out.y = f2bf(v[2]) | (f2bf(v[3]) << 16);
    out.z = f2bf(v[4]) | (f2bf(v[5]) << 16);
    out.w = f2bf(v[6]) | (f2bf(v[7]) << 16);
    *reinterpret_cast<uint4*>(a.y + o) = out;
  }
}

// --------------------------------------------- fwd / dgrad, LDS-DMA pipeline
// 16 zero bytes: the source of every padding / tail row of the im2col operand,
// so each LDS-DMA lane always loads (an exec-masked lane would leave stale LDS)
__device__ __attribute__((aligned(16))) uint32_t g_conv_zero[4] = {0u, 0u, 0u, 0u};

// (a plain device function: referenced from a kernel template, the target
// builtin would make the host-side instantiation fail)
__device__ __forceinline__ void glds16(const void* src, unsigned char* lds) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Tile TBM (pixels) x BN (out channels) x 64, (TBM/64) x 2 waves of 64 x BN/2.
// Operands go global -> LDS with global_load_lds_dwordx4 (no register staging)
// through a 3-stage ring: the loads of step t+2 are in flight while step t
// computes; one raw s_barrier per step (a __syncthreads would drain the
// in-flight DMA with vmcnt(0)).  The LDS image is lane-linear per wave, the
// XOR swizzle of off128 is applied on the SOURCE side (which 16-byte chunk a
// lane fetches).
template <int TBM, int BN>
__global__ void __launch_bounds__(TBM * 2) conv_fwd_glds_kernel(ConvFwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int NT = TBM * 2;
  constexpr int A_BYTES = TBM * 128, B_BYTES = BN * 128, STAGE = A_BYTES + B_BYTES;
  constexpr int NSTAGE = 3;
  constexpr int ALD = TBM * 8 / NT;  // 16-byte A chunks per thread per step (4)
  constexpr int BLD = BN * 8 / NT;   // B chunks per thread per step
  constexpr int NLD = ALD + BLD;
  constexpr int NI = BN / 64;
  static_assert(BLD >= 1, "B tile too small for the block");

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int ntn = a.K / BN;
  const int tn = bid % ntn, tm = bid / ntn;
  const int m0 = tm * TBM, n0 = tn * BN;
  const int C = a.C, H = a.H, W = a.W;
  const int CB = C >> 6;
  const int KT = 9 * CB;

  int a_pix[ALD], a_h[ALD], a_w[ALD], a_col[ALD];
#pragma unroll
  for (int i = 0; i < ALD; ++i) {
    const int s = i * NT + tid;
    const int row = s >> 3, lc = (s & 7) ^ ((row >> 1) & 7);
    const int p = m0 + row;
    a_pix[i] = p < a.P ? p : -1;
    const int q = p / W;
    a_w[i] = p - q * W;
    a_h[i] = q % H;
    a_col[i] = lc * 8;
  }
  const uint16_t* b_src[BLD];
#pragma unroll
  for (int j = 0; j < BLD; ++j) {
    const int s = j * NT + tid;
    const int row = s >> 3, lc = (s & 7) ^ ((row >> 1) & 7);
    b_src[j] = a.w + static_cast<size_t>(n0 + row) * 9 * C + lc * 8;
  }
  const uint16_t* zero = reinterpret_cast<const uint16_t*>(g_conv_zero);
  int kr = 0, ks = 0, cb = 0;  // (r, s, channel block) of the next step to issue
  auto issue = [&](int stage) __attribute__((always_inline)) {
    unsigned char* base = smem + stage * STAGE + wid * 64 * 16;
    const int dr = kr - 1, ds = ks - 1;
#pragma unroll
    for (int i = 0; i < ALD; ++i) {
      const int hh = a_h[i] + dr, ww = a_w[i] + ds;
      const bool ok = a_pix[i] >= 0 && static_cast<unsigned>(hh) < static_cast<unsigned>(H) &&
                      static_cast<unsigned>(ww) < static_cast<unsigned>(W);
      const uint16_t* src =
          ok ? a.x + static_cast<size_t>(a_pix[i] + dr * W + ds) * C + cb * 64 + a_col[i] : zero;
      glds16(src, base + i * NT * 16);
    }
    const int koff = (kr * 3 + ks) * C + cb * 64;
#pragma unroll
    for (int j = 0; j < BLD; ++j)
      glds16(b_src[j] + koff, base + A_BYTES + j * NT * 16);
    if (++cb == CB) {
      cb = 0;
      if (++ks == 3) { ks = 0; ++kr; }
    }
  };

  f32x16_t acc[2][NI];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[mi][ni][e] = 0.f;

  issue(0);
  if (KT > 1) issue(1);
  const int hi = lane >> 5, lr = lane & 31;
  for (int kt = 0; kt < KT; ++kt) {
    if (kt + 1 < KT) wait_vmcnt<NLD>(); else wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    if (kt + 2 < KT) issue((kt + 2) % NSTAGE);
    const unsigned char* sA = smem + (kt % NSTAGE) * STAGE;
    const unsigned char* sB = sA + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int chk = 2 * kk + hi;
      bf16x8_t af[2], bfr[NI];
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
        af[mi] = *reinterpret_cast<const bf16x8_t*>(sA + off128(wr * 64 + mi * 32 + lr, chk));
#pragma unroll
      for (int ni = 0; ni < NI; ++ni)
        bfr[ni] = *reinterpret_cast<const bf16x8_t*>(sB + off128(wc * (BN / 2) + ni * 32 + lr, chk));
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[mi], bfr[ni], acc[mi][ni], 0, 0, 0);
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  // ---- epilogue (as conv_fwd_kernel)
  constexpr int LD = BN + 4;
  float* ct = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = wr * 64 + mi * 32 + (e & 3) + 8 * (e >> 2) + 4 * hi;
        const int col = wc * (BN / 2) + ni * 32 + lr;
        ct[row * LD + col] = acc[mi][ni][e];
      }
  __syncthreads();
  constexpr int CPR = BN / 8;
#pragma unroll 2
  for (int e = tid; e < TBM * CPR; e += NT) {
    const int row = e / CPR, cc = e - row * CPR;
    const int p = m0 + row;
    if (p >= a.P) continue;
    const float4 lo = *reinterpret_cast<const float4*>(ct + row * LD + cc * 8);
    const float4 hi4 = *reinterpret_cast<const float4*>(ct + row * LD + cc * 8 + 4);
    float v[8] = {lo.x, lo.y, lo.z, lo.w, hi4.x, hi4.y, hi4.z, hi4.w};
    const size_t o = static_cast<size_t>(p) * a.K + n0 + cc * 8;
    if (a.relu) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = fmaxf(v[j], 0.f);
    }
    if (a.mask != nullptr) {
      const v4u m = *reinterpret_cast<const v4u*>(a.mask + o);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t hb = (m[j >> 1] >> (16 * (j & 1))) & 0xffffu;
        if ((hb & 0x8000u) || hb == 0u) v[j] = 0.f;
      }
    }
    if (a.addend != nullptr) {
      const v4u m = *reinterpret_cast<const v4u*>(a.addend + o);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += bf2f((m[j >> 1] >> (16 * (j & 1))) & 0xffffu);
    }
    v4u out;
    out[0] = f2bf(v[0]) | (f2bf(v[1]) << 16);
    out[1] = f2bf(v[2]) | (f2bf(v[3]) << 16);
    out[2] = f2bf(v[4]) | (f2bf(v[5]) << 16);
    out[3] = f2bf(v[6]) | (f2bf(v[7]) << 16);
    *reinterpret_cast<v4u*>(a.y + o) = out;
  }
}

// ------------------------------------------------------------------ wgrad
// 256-byte rows (128 bf16), chunk 0..15; swizzle of cdna_hip_programming.md
// T10 (b): conflict-free for the 32x32x16 transposed operand reads
__device__ __forceinline__ int off256(int row, int ch) {
  return row * 256 + ((ch ^ (((row & 3) << 2) | ((row >> 2) & 3))) << 4);
}
// 128-byte rows (64 bf16), chunk 0..7: rows k, k+2 of a 4-row tr block differ in bit 2
__device__ __forceinline__ int off128t(int row, int ch) {
  return row * 128 + ((ch ^ (((row >> 1) & 1) << 2)) << 4);
}

template <int ROWB>
__device__ __forceinline__ int img_off(int row, int ch) {
  if constexpr (ROWB == 256) return off256(row, ch);
  else return off128t(row, ch);
}

// one 32(col) x 16(k) MFMA operand from an image [k rows][cols]: lane holds
// col = cb + (lane & 31), k = kbase + 8 * (lane >> 5) + j
template <int ROWB>
__device__ __forceinline__ bf16x8_t tr_operand(const unsigned char* img, int kbase, int cb, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int col = cb + 16 * (g & 1) + 4 * p;
  const int row = kbase + 8 * (g >> 1) + q;
  const int chk = col >> 3, inb = (p & 1) * 8;
  typedef __attribute__((address_space(3))) s16x4_t lds_s16x4_t;
  const lds_s16x4_t* p0 = reinterpret_cast<const lds_s16x4_t*>(
      reinterpret_cast<uintptr_t>(img + img_off<ROWB>(row, chk) + inb));
  const lds_s16x4_t* p1 = reinterpret_cast<const lds_s16x4_t*>(
      reinterpret_cast<uintptr_t>(img + img_off<ROWB>(row + 4, chk) + inb));
  const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(const_cast<lds_s16x4_t*>(p0));
  const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(const_cast<lds_s16x4_t*>(p1));
  s16x8_t r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return __builtin_bit_cast(bf16x8_t, r);
}

template <int BN>
__global__ void __launch_bounds__(256, 2) conv_wgrad_kernel(ConvWgradArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int A_BYTES = BK * BM * 2;  // [64 px][128 k]
  constexpr int B_BYTES = BK * BN * 2;  // [64 px][BN c]
  constexpr int BUF = A_BYTES + B_BYTES;
  constexpr int NI = BN / 64;
  constexpr int BCH = BN / 8;               // 16-byte chunks per B row
  constexpr int BROWS = (BK * BCH) / 256;   // B chunks per thread

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int C = a.C, K = a.K, H = a.H, W = a.W;
  const int ntc = C / BN, ntk = K / BM;
  const int ntiles = ntk * 9 * ntc;
  const int tile = bid % ntiles, split = bid / ntiles;
  const int tc = tile % ntc, rs = (tile / ntc) % 9, tk = tile / (ntc * 9);
  const int k0 = tk * BM, c0 = tc * BN;
  const int dr = rs / 3 - 1, ds = rs % 3 - 1;
  const int pbeg = split * a.steps_per_split * BK;
  const int pend = min(a.P, pbeg + a.steps_per_split * BK);
  const int nsteps = pend > pbeg ? (pend - pbeg + BK - 1) / BK : 0;

  const int cha = tid & 15;           // A: 16 chunks per 256-byte row
  const int chb = tid % BCH;
  v4u ra[4], rb[BROWS];
  auto gload = [&](int p0) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int p = p0 + (tid >> 4) + 16 * i;
      v4u v = {0u, 0u, 0u, 0u};
      if (p < pend) v = *reinterpret_cast<const v4u*>(a.dy + static_cast<size_t>(p) * K + k0 + cha * 8);
      ra[i] = v;
    }
#pragma unroll
    for (int j = 0; j < BROWS; ++j) {
      const int p = p0 + (tid / BCH) + (256 / BCH) * j;
      const uint32_t q = fdiv(static_cast<uint32_t>(p), a.div_w);
      const int w = p - static_cast<int>(q) * W;
      const int h = static_cast<int>(q - fdiv(q, a.div_h) * H);
      const int hh = h + dr, ww = w + ds;
      v4u v = {0u, 0u, 0u, 0u};
      if (p < pend && static_cast<unsigned>(hh) < static_cast<unsigned>(H) &&
          static_cast<unsigned>(ww) < static_cast<unsigned>(W))
        v = *reinterpret_cast<const v4u*>(a.x + static_cast<size_t>(p + dr * W + ds) * C + c0 + chb * 8);
      rb[j] = v;
    }
  };
  auto sstore = [&](int buf) __attribute__((always_inline)) {
    unsigned char* sA = smem + buf * BUF;
    unsigned char* sB = sA + A_BYTES;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      *reinterpret_cast<v4u*>(sA + off256((tid >> 4) + 16 * i, cha)) = ra[i];
#pragma unroll
    for (int j = 0; j < BROWS; ++j)
      *reinterpret_cast<v4u*>(sB + img_off<BN * 2>((tid / BCH) + (256 / BCH) * j, chb)) = rb[j];
  };

  f32x16_t acc[2][NI];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[mi][ni][e] = 0.f;

  if (nsteps > 0) {
    gload(pbeg);
    sstore(0);
  }
  __syncthreads();
  for (int st = 0; st < nsteps; ++st) {
    const bool more = st + 1 < nsteps;
    if (more) gload(pbeg + (st + 1) * BK);
    const unsigned char* sA = smem + (st & 1) * BUF;
    const unsigned char* sB = sA + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      bf16x8_t af[2], bfr[NI];
#pragma unroll
      for (int mi = 0; mi < 2; ++mi) af[mi] = tr_operand<256>(sA, kk * 16, wr * 64 + mi * 32, lane);
#pragma unroll
      for (int ni = 0; ni < NI; ++ni)
        bfr[ni] = tr_operand<BN * 2>(sB, kk * 16, wc * (BN / 2) + ni * 32, lane);
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[mi], bfr[ni], acc[mi][ni], 0, 0, 0);
    }
    if (more) sstore((st + 1) & 1);
    __syncthreads();
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
        const int c = c0 + wc * (BN / 2) + ni * 32 + lr;
        slab[(static_cast<size_t>(k) * 9 + rs) * C + c] = acc[mi][ni][e];
      }
}

// dw[k][c][r][s] (fp32, PyTorch layout) = sum_split slab[split][k][rs][c]
__global__ void __launch_bounds__(256) conv_wgrad_reduce_kernel(const float* __restrict__ slab,
                                                                 float* __restrict__ dw, int K, int C,
                                                                 int splits, float beta) {
  const size_t n = static_cast<size_t>(K) * 9 * C;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += static_cast<size_t>(gridDim.x) * 256) {
    float s = 0.f;
    for (int t = 0; t < splits; ++t) s += slab[t * n + i];
    const int c = static_cast<int>(i % C);
    const size_t kr = i / C;
    const int rs = static_cast<int>(kr % 9);
    const size_t k = kr / 9;
    const size_t o = (k * C + c) * 9 + rs;
    dw[o] = beta != 0.f ? beta * dw[o] + s : s;
  }
}

// w [K][C][3][3] fp32 -> wf [K][3][3][C] bf16 and wt [C][3][3][K] bf16 (flipped)
__global__ void __launch_bounds__(256) conv_weight_prep_kernel(const float* __restrict__ w,
                                                               uint16_t* __restrict__ wf,
                                                               uint16_t* __restrict__ wt, int K, int C) {
  const int n = K * C * 9;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const int rs = i % 9;
    const int c = (i / 9) % C;
    const int k = i / (9 * C);
    const uint16_t b = static_cast<uint16_t>(f2bf(w[i]));
    if (wf != nullptr) wf[(k * 9 + rs) * C + c] = b;
    if (wt != nullptr) wt[(c * 9 + (8 - rs)) * K + k] = b;
  }
}

// g = gy where y > 0 else 0  (bf16, 8 per thread)
__global__ void __launch_bounds__(256) relu_mask_kernel(const uint4* __restrict__ gy,
                                                        const uint4* __restrict__ y,
                                                        uint4* __restrict__ g, int64_t n8) {
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n8; i += static_cast<int64_t>(gridDim.x) * 256) {
    const uint4 a = gy[i], m = y[i];
    const uint32_t av[4] = {a.x, a.y, a.z, a.w}, mv[4] = {m.x, m.y, m.z, m.w};
    uint32_t o[4];
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
    g[i] = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

int grid_for(int64_t n, int per_block) {
  int64_t b = (n + per_block - 1) / per_block;
  if (b > 16384) b = 16384;
  return static_cast<int>(b < 1 ? 1 : b);
}

template <typename F>
void set_lds(F fn, int bytes) {
  static_assert(sizeof(F) > 0, "");
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(fn),
                            hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}

}  // namespace

bool conv3x3_supported(int C, int K) { return C % 64 == 0 && K % 64 == 0 && C >= 64 && K >= 64; }

template <int TBM, int BN>
void launch_fwd_glds(const ConvFwdArgs& a, hipStream_t stream) {
  constexpr int lds_pipe = 3 * (TBM * 128 + BN * 128);
  constexpr int lds_epi = TBM * (BN + 4) * 4;
  constexpr int lds = lds_pipe > lds_epi ? lds_pipe : lds_epi;
  static bool init = false;
  if (!init) { set_lds(conv_fwd_glds_kernel<TBM, BN>, lds); init = true; }
  const int mt = (a.P + TBM - 1) / TBM;
  hipLaunchKernelGGL((conv_fwd_glds_kernel<TBM, BN>), dim3(mt * (a.K / BN)), dim3(TBM * 2), lds,
                     stream, a);
}

void launch_conv3x3_fwd(const ConvFwdArgs& a, hipStream_t stream) {
  static const int variant = [] {
    const char* e = getenv("COMMEFF_CONV_FWD");
    return e != nullptr && e[0] == 'r' ? 1 : 0;  // "regs": register-staged kernel
  }();
  if (variant == 0) {
    const bool wide = a.K % 128 == 0;
    const int bn = wide ? 128 : 64;
    // 256-pixel tiles when they still give >= 2 blocks per CU, else 128
    const bool big = static_cast<int64_t>((a.P + 255) / 256) * (a.K / bn) >= 512;
    if (big) {
      if (wide) launch_fwd_glds<256, 128>(a, stream); else launch_fwd_glds<256, 64>(a, stream);
    } else {
      if (wide) launch_fwd_glds<128, 128>(a, stream); else launch_fwd_glds<128, 64>(a, stream);
    }
    return;
  }
  const int mt = (a.P + BM - 1) / BM;
  if (a.K % 128 == 0) {
    constexpr int BN = 128;
    const int lds = max(2 * (BM * BK * 2 + BN * BK * 2), BM * (BN + 4) * 4);
    static bool init = false;
    if (!init) { set_lds(conv_fwd_kernel<BN>, lds); init = true; }
    hipLaunchKernelGGL(conv_fwd_kernel<BN>, dim3(mt * (a.K / BN)), dim3(256), lds, stream, a);
  } else {
    constexpr int BN = 64;
    const int lds = max(2 * (BM * BK * 2 + BN * BK * 2), BM * (BN + 4) * 4);
    static bool init = false;
    if (!init) { set_lds(conv_fwd_kernel<BN>, lds); init = true; }
    hipLaunchKernelGGL(conv_fwd_kernel<BN>, dim3(mt * (a.K / BN)), dim3(256), lds, stream, a);
  }
}

int conv3x3_wgrad_splits(int P, int K, int C) {
  const int bn = C % 128 == 0 ? 128 : 64;
  const int tiles = (K / BM) * 9 * (C / bn);
  const int steps = (P + BK - 1) / BK;
  // aim for >= ~1024 blocks (4 per CU) with >= 16 K-steps each
  int s = (1024 + tiles - 1) / tiles;
  if (s > steps / 16) s = steps / 16;
  return s < 1 ? 1 : s;
}

void launch_conv3x3_wgrad(ConvWgradArgs a, float* dw, float beta, hipStream_t stream) {
  const int steps = (a.P + BK - 1) / BK;
  a.steps_per_split = (steps + a.splits - 1) / a.splits;
  a.div_w = make_fastdiv(static_cast<uint32_t>(a.W));
  a.div_h = make_fastdiv(static_cast<uint32_t>(a.H));
  if (a.C % 128 == 0) {
    constexpr int BN = 128;
    const int lds = 2 * (BK * BM * 2 + BK * BN * 2);
    static bool init = false;
    if (!init) { set_lds(conv_wgrad_kernel<BN>, lds); init = true; }
    const int tiles = (a.K / BM) * 9 * (a.C / BN);
    hipLaunchKernelGGL(conv_wgrad_kernel<BN>, dim3(tiles * a.splits), dim3(256), lds, stream, a);
  } else {
    constexpr int BN = 64;
    const int lds = 2 * (BK * BM * 2 + BK * BN * 2);
    static bool init = false;
    if (!init) { set_lds(conv_wgrad_kernel<BN>, lds); init = true; }
    const int tiles = (a.K / BM) * 9 * (a.C / BN);
    hipLaunchKernelGGL(conv_wgrad_kernel<BN>, dim3(tiles * a.splits), dim3(256), lds, stream, a);
  }
  const int64_t n = static_cast<int64_t>(a.K) * 9 * a.C;
  hipLaunchKernelGGL(conv_wgrad_reduce_kernel, dim3(grid_for(n, 256)), dim3(256), 0, stream,
                     a.slab, dw, a.K, a.C, a.splits, beta);
}

void launch_conv_weight_prep(const float* w, uint16_t* wf, uint16_t* wt, int K, int C,
                             hipStream_t stream) {
  hipLaunchKernelGGL(conv_weight_prep_kernel, dim3(grid_for(static_cast<int64_t>(K) * C * 9, 256)),
                     dim3(256), 0, stream, w, wf, wt, K, C);
}

void launch_relu_mask(const uint16_t* gy, const uint16_t* y, uint16_t* g, int64_t n,
                      hipStream_t stream) {
  const int64_t n8 = n / 8;
  hipLaunchKernelGGL(relu_mask_kernel, dim3(grid_for(n8, 256)), dim3(256), 0, stream,
                     reinterpret_cast<const uint4*>(gy), reinterpret_cast<const uint4*>(y),
                     reinterpret_cast<uint4*>(g), n8);
}

}  // namespace commeff
