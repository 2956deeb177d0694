// 3x3 / stride 1 / pad 1 convolution, forward and dgrad, as ONE continuous
// stream of K-steps per workgroup (gfx950, v_mfma_f32_16x16x32_bf16).
//
//   y[p, k] = epilogue( sum_{r,s,c} x[p + (r-1, s-1), c] * w[k, r, s, c] )
//
// (dgrad = the same kernel on dy and the flipped, transposed weights.)  The
// ResNet-9 convolutions this serves (reference model
// /root/reference/CommEfficient/models/resnet9.py:32-130) are short-K GEMMs:
// 256 x 128 output tiles need only 9 * C / 32 K-steps, so a tile's window
// load, its K-steps and its stores are each a large share of its time.  The
// previous kernel (conv.hip, conv_fwd_halo_kernel) ran one tile per workgroup
// with the window reloaded per channel block and the stores at the end: at
// the ResNet-9 batch the whole grid is one wave of tiles, and the chip
// alternated between all-load, all-MFMA and all-store phases (770-1000 TF/s,
// profiles/r5_experiments.md).
//
// Here each workgroup (4 waves, two per CU) walks a static list of tiles as
// one stream of K-steps (K-step = one tap x 32 input channels):
//   * the 32-channel halo WINDOW of a (tile, channel block) period -- the
//     tile's pixels plus a one-pixel frame, 64-byte rows -- serves all 9
//     taps; windows are double-buffered and the window of period q+1 is
//     staged by LDS-DMA (global_load_lds_dwordx4) during period q, one piece
//     per thread per step, so window loads, including the next tile's first,
//     run under the MFMAs;
//   * the weight tile of step g (128 out channels x 32 in channels) goes
//     through a 3-slot ring, issued 3 steps ahead (the DMA of step g+3 is
//     issued right after the barrier that retires slot g % 3);
//   * one raw s_barrier per step, in the MIDDLE of the step: before it every
//     wave waits (counted vmcnt: later DMAs stay in flight) for the weight
//     tile of step g+1 and its own LDS reads; after it the next reads go out
//     under the second half of the step's MFMAs;
//   * the epilogue runs straight from the accumulators (no LDS): the MFMA
//     computes the TRANSPOSED tile (A = weights, B = pixels), so each lane
//     holds 4 consecutive output channels of one pixel -- 8-byte stores, the
//     fused ReLU / mask / residual / 2x2 max-pool / un-pool in registers --
//     and its stores drain while the next tile's K-steps run.
// Wave tile: 64 channels x 128 pixels (16 accumulators of 16 x 16 ... 32 x
// f32x4 = 128 registers); per step 4 weight + 8 pixel fragments
// (ds_read_b128) feed 32 MFMAs.  LDS: 2 x 24 KB windows + 3 x 8 KB ring.
//
// LDS images (64-byte rows, 16-byte chunks c = 0..3, swizzles found by a
// lane-exact model of the ds_read_b128 lane groups, scripts/dev/swz_search.py):
//   window row (pr, pc) [padded row, column]: chunk slot c ^ f(pc),
//     f(pc) = (pc + 2 (pc >> 2)) & 3 (W >= 16) or pc & 3 (W = 8)
//   weight row n: chunk slot c ^ ((n >> 1) & 2)
// The LDS-DMA writes each wave's 1 KB lane-linearly, so the permutation is
// applied on the SOURCE side (the read side applies the same involution).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <type_traits>
#include "kernels.h"
#include "conv_common.h"

namespace commeff {
namespace {

typedef float f32x4_t __attribute__((ext_vector_type(4)));

__device__ __attribute__((aligned(16))) uint32_t g_cs_zero[4] = {0u, 0u, 0u, 0u};

__device__ __forceinline__ void glds(const void* src, unsigned char* lds) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

template <int N>
__device__ __forceinline__ void vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// s_waitcnt vmcnt(n) for a run-time n (the immediate picked by a jump table)
__device__ __forceinline__ void vmcnt_dyn(int n) {
  switch (n < 63 ? n : 63) {
    case 1: vmcnt<1>(); break;
    case 2: vmcnt<2>(); break;
    case 3: vmcnt<3>(); break;
    case 4: vmcnt<4>(); break;
    case 5: vmcnt<5>(); break;
    case 6: vmcnt<6>(); break;
    case 7: vmcnt<7>(); break;
    case 8: vmcnt<8>(); break;
    case 9: vmcnt<9>(); break;
    case 10: vmcnt<10>(); break;
    case 11: vmcnt<11>(); break;
    case 12: vmcnt<12>(); break;
    case 13: vmcnt<13>(); break;
    case 14: vmcnt<14>(); break;
    case 15: vmcnt<15>(); break;
    case 16: vmcnt<16>(); break;
    case 17: vmcnt<17>(); break;
    case 18: vmcnt<18>(); break;
    case 19: vmcnt<19>(); break;
    case 20: vmcnt<20>(); break;
    case 21: vmcnt<21>(); break;
    case 22: vmcnt<22>(); break;
    case 23: vmcnt<23>(); break;
    case 24: vmcnt<24>(); break;
    case 25: vmcnt<25>(); break;
    case 26: vmcnt<26>(); break;
    case 27: vmcnt<27>(); break;
    case 28: vmcnt<28>(); break;
    case 29: vmcnt<29>(); break;
    case 30: vmcnt<30>(); break;
    case 31: vmcnt<31>(); break;
    case 32: vmcnt<32>(); break;
    case 33: vmcnt<33>(); break;
    case 34: vmcnt<34>(); break;
    case 35: vmcnt<35>(); break;
    case 36: vmcnt<36>(); break;
    case 37: vmcnt<37>(); break;
    case 38: vmcnt<38>(); break;
    case 39: vmcnt<39>(); break;
    case 40: vmcnt<40>(); break;
    case 41: vmcnt<41>(); break;
    case 42: vmcnt<42>(); break;
    case 43: vmcnt<43>(); break;
    case 44: vmcnt<44>(); break;
    case 45: vmcnt<45>(); break;
    case 46: vmcnt<46>(); break;
    case 47: vmcnt<47>(); break;
    case 48: vmcnt<48>(); break;
    case 49: vmcnt<49>(); break;
    case 50: vmcnt<50>(); break;
    case 51: vmcnt<51>(); break;
    case 52: vmcnt<52>(); break;
    case 53: vmcnt<53>(); break;
    case 54: vmcnt<54>(); break;
    case 55: vmcnt<55>(); break;
    case 56: vmcnt<56>(); break;
    case 57: vmcnt<57>(); break;
    case 58: vmcnt<58>(); break;
    case 59: vmcnt<59>(); break;
    case 60: vmcnt<60>(); break;
    case 61: vmcnt<61>(); break;
    case 62: vmcnt<62>(); break;
    case 63: vmcnt<63>(); break;
    default: vmcnt<0>(); break;
  }
}

// Tile geometry: TBM = 256 pixels = whole image rows (G images x Rg rows) of
// a square W x W image (W = 32, 16, 8); padded window PR x PW rows.
template <int W>
struct Geo {
  static constexpr int TBM = 256;
  static constexpr int H = W;
  static constexpr int R = TBM / W;                 // image rows per tile
  static constexpr int G = R <= H ? 1 : R / H;      // images per tile
  static constexpr int Rg = R <= H ? R : H;         // rows per image in the tile
  static constexpr int PW = W + 2;
  static constexpr int PR = G * (Rg + 1) + 1;
  static constexpr int NPW = PR * PW;               // window rows (64 B each)
  static constexpr int WINB = ((NPW * 64 + 8191) / 8192) * 8192;  // per buffer, 8 KB granules
  static_assert(TBM % W == 0 && (R <= H ? H % R == 0 : R % H == 0), "tile of whole rows");
  // window row of tile pixel m
  static constexpr int row_of(int m) {
    const int g = m / (Rg * W), rem = m - g * Rg * W, r = rem / W, w = rem - r * W;
    return (g * (Rg + 1) + r + 1) * PW + w + 1;
  }
  __device__ static int swz(int pc) {
    if constexpr (W >= 16) return (pc + 2 * (pc >> 2)) & 3;
    else return pc & 3;
  }
};

struct StreamArgs {
  ConvFwdArgs a;
  int ntiles, ntn;  // tiles (pixel tiles x channel tiles), channel tiles
  // timing experiments only (COMMEFF_STREAM_ABLATE; results are wrong): bit 0
  // no weight DMA after the prologue, 1 no window DMA after it, 2 no mid-step
  // wait / barrier, 3 no epilogue
  int ablate;
};

// FCH: 16-channel fragments per wave, FPX: 16-pixel fragments per wave,
// WCH x WPX = 4 waves; BN = WCH FCH 16 output channels, 256 pixels per tile.
template <int W, int WCH, int WPX, int FCH, int FPX>
__global__ void __launch_bounds__(64 * WCH * WPX, 2 * WCH * WPX / 4)
conv_stream_kernel(StreamArgs sa) {
  using Gm = Geo<W>;
  constexpr int NT = 64 * WCH * WPX;   // threads (two workgroups per CU)
  constexpr int PIECE = NT * 16;       // bytes of one DMA piece per thread
  static_assert(WPX * FPX * 16 == Gm::TBM, "pixel split");
  constexpr int BN = WCH * FCH * 16;
  constexpr int NB = BN * 64 / PIECE;  // weight DMA pieces per thread per step
  constexpr int NW = Gm::WINB / PIECE; // window DMA pieces per thread per window
  static_assert(NB * PIECE == BN * 64 && NW * PIECE == Gm::WINB, "whole DMA pieces");
  constexpr int SLOT = BN * 64;        // weight ring slot bytes
  constexpr int RING0 = 2 * Gm::WINB;  // ring offset in LDS
  constexpr int HP = FPX / 2;          // pixel fragments per half step
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  const ConvFwdArgs& a = sa.a;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wc = wid % WCH, wp = wid / WCH;
  const int C = a.C, K = a.K;
  const int CB = C >> 5;               // 32-channel blocks
  const int S = 9 * CB;                // K-steps per tile
  const int nimg = a.P / (W * W);
  const uint16_t* zero = reinterpret_cast<const uint16_t*>(g_cs_zero);

  // this workgroup's tiles: t_i = i * grid + rb (XCD-aware: neighbouring tiles,
  // which share pixels or weights, run on one XCD)
  const int grid = gridDim.x;
  const int rb = xcd_remap(blockIdx.x, grid);
  const int nt = rb < sa.ntiles ? (sa.ntiles - rb + grid - 1) / grid : 0;
  const int total = nt * S;            // K-steps of this workgroup
  const int nq = nt * CB;              // window periods (9 steps each)
  if (nt == 0) return;

  // ---- per-lane LDS read bases
  const int l16 = lane & 15, lc = lane >> 4;  // fragment row / column, k chunk
  // weight fragment f of step slot s: ring + s SLOT + f 1024 + wbase
  int wbase;
  {
    const int n = wc * FCH * 16 + l16;
    wbase = RING0 + n * 64 + ((lc ^ ((n >> 1) & 2)) << 4);
  }
  // pixel fragment j of tap (dr, dc): buf + pbase[dc + 1] + (row_of(16 j) - row_of(0)
  // + (dr + 1) PW) * 64 -- a compile-time offset: the wave's first pixel is
  // aligned to whole image rows (W >= 16) or images (W = 8); the swizzle
  // depends on the lane only (see header)
  int pbase[3];
  {
    const int m = wp * FPX * 16 + l16;
    const int R0 = Gm::row_of(m);
    const int pc0 = (m % W) + 1;
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      const int pc = pc0 + d - 1;
      // (dr = -1 folded in: every per-fragment / per-tap offset below is a
      // non-negative ds_read immediate)
      pbase[d] = (R0 + d - 1 - Gm::PW) * 64 + ((lc ^ Gm::swz(pc)) << 4);
    }
  }

  // ---- DMA issue helpers
  // weight rows of this thread's pieces (tile independent): row n, chunk
  int boff[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int sl = j * NT + tid, n = sl >> 2, c = (sl & 3) ^ ((n >> 1) & 2);
    boff[j] = n * 9 * C + c * 8;
  }
  auto tile_of = [&](int i, int& m0, int& n0) __attribute__((always_inline)) {
    const int t = i * grid + rb;
    const int tn = t % sa.ntn, tm = t / sa.ntn;
    m0 = tm * Gm::TBM;
    n0 = tn * BN;
  };
  // weight source of period q (tile q / CB, channel block q % CB): the step
  // of tap t reads bsrc(q) + t C
  auto bsrc = [&](int q) __attribute__((always_inline)) {
    const int i = q / CB, cb = q - i * CB;
    int m0, n0;
    tile_of(i, m0, n0);
    return a.w + static_cast<size_t>(n0) * 9 * C + cb * 32;
  };
  auto issue_b = [&](const uint16_t* src, int slot) __attribute__((always_inline)) {
    unsigned char* dst = smem + RING0 + slot * SLOT + wid * 1024;
#pragma unroll
    for (int j = 0; j < NB; ++j) glds(src + boff[j], dst + j * PIECE);
  };
  // window of period q (tile q / CB, channel block q % CB) into buffer q & 1
  // piece k (of NW per thread) of the window of period q (tile q / CB,
  // channel block q % CB) into buffer q & 1; xsrc = x + cb * 32, (img0, h0) =
  // the tile's first image / row
  auto issue_w_piece = [&](int q, int k, const uint16_t* xsrc, int img0, int h0) __attribute__((always_inline)) {
    unsigned char* dst = smem + (q & 1) * Gm::WINB + wid * 1024 + k * PIECE;
    // (an opaque thread index: the per-piece geometry is recomputed per piece
    // instead of being hoisted into registers for the whole stream, where it
    // spilled -- and a spill reload waits for every DMA in flight)
    int tid_o = tid;
    asm volatile("" : "+v"(tid_o));
    const int sl = k * NT + tid_o, row = sl >> 2;
    const uint16_t* src = zero;
    if (row < Gm::NPW) {
      const int pr = row / Gm::PW, pc = row - pr * Gm::PW, w = pc - 1;
      const int c = (sl & 3) ^ Gm::swz(pc);
      int img = img0, h = h0 + pr - 1;
      if constexpr (Gm::G > 1) {
        const int g = pr / (Gm::Rg + 1), rr = pr - g * (Gm::Rg + 1);
        img = img0 + g;
        h = rr - 1;
      }
      if (img < nimg && h >= 0 && h < W && w >= 0 && w < W)
        src = xsrc + (static_cast<size_t>((img * W + h) * W + w)) * C + c * 8;
    }
    glds(src, dst);
  };
  // per-period window source: (x + cb 32, first image, first row)
  struct WinSrc { const uint16_t* x; int img0, h0; };
  auto wsrc = [&](int q) __attribute__((always_inline)) {
    const int i = q / CB, cb = q - i * CB;
    int m0, n0;
    tile_of(i, m0, n0);
    const int img0 = m0 / (W * W), h0 = (m0 - img0 * W * W) / W;
    return WinSrc{a.x + cb * 32, img0, h0};
  };


  // ---- accumulators and fragments
  f32x4_t acc[FCH][FPX];
#pragma unroll
  for (int f = 0; f < FCH; ++f)
#pragma unroll
    for (int j = 0; j < FPX; ++j) acc[f][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  bf16x8_t wf[FCH], pa[HP], pb[HP];

  auto rd = [&](int off) __attribute__((always_inline)) {
    return *reinterpret_cast<const bf16x8_t*>(smem + off);
  };

  // ---- prologue: window 0, weights of steps 0..2, window 1
  const uint16_t* bq0 = bsrc(0);
  {
    const WinSrc w0 = wsrc(0);
#pragma unroll
    for (int k = 0; k < NW; ++k) issue_w_piece(0, k, w0.x, w0.img0, w0.h0);
  }
  issue_b(bq0, 0);
  if (total > 1) issue_b(bq0 + C, 1);
  if (total > 2) issue_b(bq0 + 2 * C, 2);
  // window 1 (and every later one) is staged during the period before it,
  // one piece per thread per step (steps 0 .. NW-1, behind the weights)
  if (total > 2) vmcnt<2 * NB>(); else vmcnt<0>();
  __builtin_amdgcn_s_barrier();
  // step 0's weight fragments and first-half pixel fragments (tap 0: dr = dc = -1)
#pragma unroll
  for (int f = 0; f < FCH; ++f) wf[f] = rd(wbase + f * 1024);
#pragma unroll
  for (int j = 0; j < HP; ++j)
    pa[j] = rd(pbase[0] + (Gm::row_of(16 * j) - Gm::row_of(0)) * 64);

  // VMEM instructions (a lower bound) that the last tile epilogue left in
  // flight: counted by the next two mid-step waits
  int epi_vm = 0;
  // one K-step (tap T of period q), the tap a compile-time constant
  auto step = [&](auto tc, int q, int wb, int wb1, int cbq, const uint16_t* bcur,
                  const uint16_t* bnext, const WinSrc& wn) __attribute__((always_inline)) {
      constexpr int t = decltype(tc)::value;
      const int g = q * 9 + t;
      constexpr int dr = t / 3 - 1, dc = t % 3 - 1;
      // ---- first half: pixel fragments 0..HP-1, read the second half's
      __builtin_amdgcn_sched_barrier(0);
      // opaque per-step bases: keeps the compiler from hoisting base + offset
      // pairs for every (fragment, tap) into registers; the fragment / tap
      // offsets stay ds_read immediates
      int b0 = wb + pbase[dc + 1];
      asm volatile("" : "+v"(b0));
      __builtin_assume(b0 >= 0 && b0 < 0x10000);
#pragma unroll
      for (int jj = 0; jj < HP; ++jj) {
        const int j = HP + jj;
        pb[jj] = rd(b0 +
                    (Gm::row_of(16 * j) - Gm::row_of(0) + (dr + 1) * Gm::PW) * 64);
      }
#pragma unroll
      for (int f = 0; f < FCH; ++f)
#pragma unroll
        for (int j = 0; j < HP; ++j)
          acc[f][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[f], pa[j], acc[f][j], 0, 0, 0);
#pragma unroll
      for (int k = 0; k < HP; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x008, FCH, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
      const bool more = g + 1 < total;
      if (more) {
        // every wave: own reads of slot g % 3 / the window done, weights of
        // step g+1 (and, at the period end, the next window) landed ...
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        // (the DMAs issued after those weights -- and the stores of a tile
        // epilogue in between -- stay in flight: counted vmcnt)
        const bool yb = g + 2 < total;
        // window pieces of period q + 1 issued after those weights (steps t-2, t-1)
        constexpr int npc = (t - 2 >= 0 && t - 2 < NW ? 1 : 0) + (t - 1 >= 0 && t - 1 < NW ? 1 : 0);
        const bool yw = q + 1 < nq;
        if (!(sa.ablate & 4)) {
          vmcnt_dyn((yb ? NB : 0) + (yw ? npc : 0) + (t <= 1 ? epi_vm : 0));
          __builtin_amdgcn_s_barrier();  // ... for every wave; slot g % 3 is free
        }
        if (g + 3 < total && !(sa.ablate & 1)) issue_b((t + 3 < 9 ? bcur : bnext) + ((t + 3) % 9) * C, t % 3);
        if constexpr (t < NW) {
          if (q + 1 < nq && !(sa.ablate & 2)) issue_w_piece(q + 1, t, wn.x, wn.img0, wn.h0);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      // ---- second half: pixel fragments HP..FPX-1; then the next step's reads
      constexpr int tn = (t + 1) % 9, drn = tn / 3 - 1, dcn = tn % 3 - 1;
      int b1 = (t == 8 ? wb1 : wb) + pbase[dcn + 1];
      asm volatile("" : "+v"(b1));
      __builtin_assume(b1 >= 0 && b1 < 0x10000);
      constexpr int slotn = ((t + 1) % 3) * SLOT;
#pragma unroll
      for (int f = 0; f < FCH; ++f) {
#pragma unroll
        for (int j = 0; j < HP; ++j)
          acc[f][HP + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[f], pb[j], acc[f][HP + j], 0, 0, 0);
        // (unconditional: after the last step these read stale, unused bytes)
        wf[f] = rd(wbase + slotn + f * 1024);
        if (f < HP)
          pa[f] = rd(b1 +
                     (Gm::row_of(16 * f) - Gm::row_of(0) + (drn + 1) * Gm::PW) * 64);
      }
#pragma unroll
      for (int f = FCH; f < HP; ++f)
        pa[f] = rd(b1 +
                   (Gm::row_of(16 * f) - Gm::row_of(0) + (drn + 1) * Gm::PW) * 64);
      __builtin_amdgcn_sched_barrier(0);
      // ---- tile end: epilogue straight from the accumulators
      if constexpr (t == 8) if (cbq == CB - 1 && !(sa.ablate & 8)) {
        int m0, n0;
        tile_of(q / CB, m0, n0);
        const int pw0 = m0 + wp * FPX * 16;
        const int ch0 = n0 + wc * FCH * 16 + 4 * lc;
        if (a.pool == 2) {
          // relu + 2x2 max-pool with window codes (csrc/pool.hip semantics):
          // compare the bf16-rounded values, first maximum in window order
          // t = 0 (top-left), 1, 2, 3; code 255 (and 0) where the max <= 0.
          // Two channel fragments per store (v_permlane16_swap, as below).
          const int lofs = (lc & 1) * 16 + (lc >> 1) * 8;
#pragma unroll
          for (int f = 0; f < FCH; f += 2)
#pragma unroll
            for (int j = 0; j < FPX; ++j) {
              constexpr int VJ = W >= 16 ? W / 16 : 0;  // vertical partner fragment offset
              if constexpr (W >= 16) {
                if (((16 * j) / W) % 2 != 0) continue;  // fragment of an odd image row
              }
              uint32_t outp[2][2], codep[2];
#pragma unroll
              for (int h = 0; h < 2; ++h) {
                float cand[4][4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                  const float top = static_cast<float>(static_cast<__bf16>(acc[f + h][j][r]));
                  cand[0][r] = top;
                  cand[1][r] = __shfl_xor(top, 1);
                  if constexpr (W >= 16) {
                    const float bot = static_cast<float>(static_cast<__bf16>(acc[f + h][j + VJ][r]));
                    cand[2][r] = bot;
                    cand[3][r] = __shfl_xor(bot, 1);
                  } else {
                    cand[2][r] = __shfl_xor(top, 8);
                    cand[3][r] = __shfl_xor(top, 9);
                  }
                }
                uint32_t codes = 0, out[2] = {0u, 0u};
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                  float best = cand[0][r];
                  uint32_t arg = 0;
#pragma unroll
                  for (int u = 1; u < 4; ++u)
                    if (cand[u][r] > best) { best = cand[u][r]; arg = u; }
                  const bool pos = best > 0.f;
                  const uint32_t hb = pos ? (__float_as_uint(best) >> 16) : 0u;
                  out[r >> 1] |= hb << (16 * (r & 1));
                  codes |= (pos ? arg : 255u) << (8 * r);
                }
                outp[h][0] = out[0];
                outp[h][1] = out[1];
                codep[h] = codes;
              }
              const auto s0 = __builtin_amdgcn_permlane16_swap(outp[0][0], outp[1][0], false, false);
              const auto s1 = __builtin_amdgcn_permlane16_swap(outp[0][1], outp[1][1], false, false);
              const auto sc = __builtin_amdgcn_permlane16_swap(codep[0], codep[1], false, false);
              const int m = pw0 + 16 * j + l16;  // top-left pixel (even lanes of even rows)
              const bool lead = (l16 & 1) == 0 && (W >= 16 || l16 < 8);
              if (!lead) continue;
              const int n = m / (W * W), rem = m - n * W * W, h = rem / W, w = rem - h * W;
              const size_t qo = (static_cast<size_t>(n * (W / 2) + h / 2) * (W / 2) + w / 2) * K +
                                (ch0 - 4 * lc) + f * 16 + lofs;
              *reinterpret_cast<v4u*>(a.y + qo) = v4u{s0[0], s1[0], s0[1], s1[1]};
              *reinterpret_cast<uint2*>(a.pool_idx + qo) = make_uint2(sc[0], sc[1]);
            }
        } else {
          // two channel fragments per store: v_permlane16_swap gives each lane 8
          // consecutive channels of its pixel (16-byte loads / stores; the
          // epilogue is store-issue bound with 8-byte accesses)
          const bool relu = a.relu != 0;
          const int lofs = (lc & 1) * 16 + (lc >> 1) * 8;  // the lane's channels after the swap
#pragma unroll
          for (int f = 0; f < FCH; f += 2)
#pragma unroll
            for (int j = 0; j < FPX; ++j) {
              const int p = pw0 + 16 * j + l16;
              float v[8];
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[f][j][r]),
                                                                 __float_as_uint(acc[f + 1][j][r]), false, false);
                v[r] = __uint_as_float(sw[0]);
                v[4 + r] = __uint_as_float(sw[1]);
              }
              const size_t o = static_cast<size_t>(p) * K + (ch0 - 4 * lc) + f * 16 + lofs;
              if (relu) {
#pragma unroll
                for (int r = 0; r < 8; ++r) v[r] = fmaxf(v[r], 0.f);
              }
              if (a.mask != nullptr) {
                const v4u mk = *reinterpret_cast<const v4u*>(a.mask + o);
#pragma unroll
                for (int r = 0; r < 8; ++r) {
                  const uint32_t hb = (mk[r >> 1] >> (16 * (r & 1))) & 0xffffu;
                  v[r] = ((hb & 0x8000u) == 0u && hb != 0u) ? v[r] : 0.f;
                }
              }
              if (a.addend != nullptr) {
                if (a.y_pre != nullptr && a.unpool_idx == nullptr) {
                  v4u pre;
#pragma unroll
                  for (int h = 0; h < 4; ++h) pre[h] = pack_bf16(v[2 * h], v[2 * h + 1]);
                  *reinterpret_cast<v4u*>(a.y_pre + o) = pre;
                }
                const v4u ad = *reinterpret_cast<const v4u*>(a.addend + o);
#pragma unroll
                for (int r = 0; r < 8; ++r) v[r] += bf2f((ad[r >> 1] >> (16 * (r & 1))) & 0xffffu);
              }
              v4u out;
#pragma unroll
              for (int h = 0; h < 4; ++h) out[h] = pack_bf16(v[2 * h], v[2 * h + 1]);
              if (a.unpool_idx != nullptr) {
                // relu + max-pool backward: each value to its window position t
                // (code byte per channel, 255 = relu-dead), zeros elsewhere
                const uint64_t codes = *reinterpret_cast<const uint64_t*>(a.unpool_idx + o);
                const int n = p / (W * W), rem = p - n * W * W, oh = rem / W, ow = rem - oh * W;
                const int FW = 2 * W;
                const size_t f0 = (static_cast<size_t>(n * 2 * W + 2 * oh) * FW + 2 * ow) * K + (o - static_cast<size_t>(p) * K);
#pragma unroll
                for (int tt = 0; tt < 4; ++tt) {
                  v4u ot;
#pragma unroll
                  for (int h = 0; h < 4; ++h) {
                    const uint32_t c0 = static_cast<uint32_t>(codes >> (16 * h)) & 0xffu;
                    const uint32_t c1 = static_cast<uint32_t>(codes >> (16 * h + 8)) & 0xffu;
                    ot[h] = (c0 == static_cast<uint32_t>(tt) ? (out[h] & 0xffffu) : 0u) |
                            (c1 == static_cast<uint32_t>(tt) ? (out[h] & 0xffff0000u) : 0u);
                  }
                  *reinterpret_cast<v4u*>(a.y + f0 + static_cast<size_t>((tt >> 1) * FW + (tt & 1)) * K) = ot;
                }
                continue;
              }
              *reinterpret_cast<v4u*>(a.y + o) = out;
              if (a.y_dual != nullptr) {
                const v4u dm = *reinterpret_cast<const v4u*>(a.dual_mask + o);
                v4u od;
#pragma unroll
                for (int h = 0; h < 4; ++h) {
                  const uint32_t lo = dm[h] & 0xffffu, hi = dm[h] >> 16;
                  od[h] = (((lo & 0x8000u) == 0u && lo != 0u) ? (out[h] & 0xffffu) : 0u) |
                          (((hi & 0x8000u) == 0u && hi != 0u) ? (out[h] & 0xffff0000u) : 0u);
                }
                *reinterpret_cast<v4u*>(a.y_dual + o) = od;
              }
            }
        }
#pragma unroll
        for (int f = 0; f < FCH; ++f)
#pragma unroll
          for (int j = 0; j < FPX; ++j) acc[f][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        // stores only (the epilogue's own loads were waited for): pool 2 per
        // even-row fragment; plain / relu / mask 1 per fragment pair; the
        // other variants are not counted (a smaller count only waits longer)
        if (a.pool == 2) epi_vm = FCH * (W >= 16 ? FPX / 2 : FPX);
        else if (a.unpool_idx == nullptr && a.addend == nullptr && a.y_dual == nullptr) epi_vm = FCH / 2 * FPX;
        else epi_vm = 0;
      }
      if constexpr (t == 1) epi_vm = 0;
  };  // step

  const uint16_t* bq = bq0;
  for (int q = 0; q < nq; ++q) {
    const int wb = (q & 1) * Gm::WINB;    // this period's window buffer
    const int wb1 = wb ^ Gm::WINB;        // the next period's
    const int cbq = q % CB;
    const uint16_t* bcur = bq;
    const uint16_t* bnext = q + 1 < nq ? bsrc(q + 1) : bq;
    bq = bnext;
    const WinSrc wn = q + 1 < nq ? wsrc(q + 1) : WinSrc{a.x, 0, 0};
    step(std::integral_constant<int, 0>{}, q, wb, wb1, cbq, bcur, bnext, wn);
    step(std::integral_constant<int, 1>{}, q, wb, wb1, cbq, bcur, bnext, wn);
    step(std::integral_constant<int, 2>{}, q, wb, wb1, cbq, bcur, bnext, wn);
    step(std::integral_constant<int, 3>{}, q, wb, wb1, cbq, bcur, bnext, wn);
    step(std::integral_constant<int, 4>{}, q, wb, wb1, cbq, bcur, bnext, wn);
    step(std::integral_constant<int, 5>{}, q, wb, wb1, cbq, bcur, bnext, wn);
    step(std::integral_constant<int, 6>{}, q, wb, wb1, cbq, bcur, bnext, wn);
    step(std::integral_constant<int, 7>{}, q, wb, wb1, cbq, bcur, bnext, wn);
    step(std::integral_constant<int, 8>{}, q, wb, wb1, cbq, bcur, bnext, wn);
  }
}

template <int W, int WCH, int WPX, int FCH, int FPX>
void launch_stream(const ConvFwdArgs& a, hipStream_t stream) {
  using Gm = Geo<W>;
  constexpr int BN = WCH * FCH * 16;
  constexpr int lds = 2 * Gm::WINB + 3 * BN * 64;
  static bool init = false;
  if (!init) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(conv_stream_kernel<W, WCH, WPX, FCH, FPX>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    init = true;
  }
  StreamArgs sa;
  sa.a = a;
  sa.ablate = 0;
  if (const char* e = getenv("COMMEFF_STREAM_ABLATE")) sa.ablate = atoi(e);
  sa.ntn = a.K / BN;
  sa.ntiles = ((a.P + Gm::TBM - 1) / Gm::TBM) * sa.ntn;
  static const int slots = [] {
    int dev = 0, cus = 256;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess &&
        prop.multiProcessorCount > 0)
      cus = prop.multiProcessorCount;
    return 2 * cus;  // two 4-wave workgroups per CU
  }();
  // enough tiles per workgroup to overlap one tile's stores / next window with
  // another's K-steps, while still filling every slot
  int grid = sa.ntiles < slots ? sa.ntiles : slots;
  if (const char* e = getenv("COMMEFF_STREAM_GRID")) {
    const int v = atoi(e);
    if (v > 0 && v < grid) grid = v;
  }
  COMMEFF_LAUNCH((conv_stream_kernel<W, WCH, WPX, FCH, FPX>), dim3(grid), dim3(64 * WCH * WPX), lds, stream, sa);
}

}  // namespace

// The streamed kernel serves square 32/16/8-pixel layers with 32 | C and
// 64 | K (ungrouped, no ablation); false: use conv.hip.
bool launch_conv3x3_stream(const ConvFwdArgs& a, hipStream_t stream) {
  if (a.kg != 0 || a.x_stride != 0 || a.ablate != 0 || a.H != a.W || a.C % 32 != 0 || a.C < 32)
    return false;
  if (!(a.K % 128 == 0 || a.K == 64)) return false;
  if (a.pool == 2 && a.K % 16 != 0) return false;
  if (a.P % 256 != 0) return false;  // whole tiles only (the epilogue has no pixel bound)
  // epilogue kinds served (COMMEFF_STREAM_EPI bit mask, experiments): 1 plain /
  // relu, 2 pool, 4 mask, 8 addend, 16 un-pool, 32 dual
  static const int epi_mask = [] {
    const char* e = getenv("COMMEFF_STREAM_EPI");
    return e != nullptr ? atoi(e) : 63;
  }();
  int kind = 0;
  if (a.pool == 2) kind |= 2;
  if (a.mask != nullptr) kind |= 4;
  if (a.addend != nullptr) kind |= 8;
  if (a.unpool_idx != nullptr) kind |= 16;
  if (a.y_dual != nullptr) kind |= 32;
  if (kind == 0) kind = 1;
  if ((kind & epi_mask) != kind) return false;
  // 128-channel tiles; 64-channel tiles (twice the tiles, the window read
  // once per channel tile) when the 128-wide grid gives a workgroup fewer than
  // two tiles to stream (COMMEFF_STREAM_NARROW=1/0 forces either)
  bool wide = a.K % 128 == 0;
  if (wide) {
    static const int narrow = [] {
      const char* e = getenv("COMMEFF_STREAM_NARROW");
      return e != nullptr ? atoi(e) : -1;
    }();
    const int64_t tiles128 = static_cast<int64_t>(a.P / 256) * (a.K / 128);
    if (narrow == 1 || (narrow == -1 && tiles128 < 0)) wide = false;  // (measured: narrow tiles lose)
  }
  // COMMEFF_STREAM_WAVES=8: 8-wave workgroups of 64 x 64 wave tiles (4 waves
  // per SIMD, 128 VGPRs) instead of 4-wave ones of 64 x 128 (2 per SIMD)
  static const int waves8 = [] {
    const char* e = getenv("COMMEFF_STREAM_WAVES");
    return e != nullptr && atoi(e) == 8;
  }();
  switch (a.W) {
    case 32:
      if (!wide) launch_stream<32, 1, 4, 4, 4>(a, stream);
      else if (waves8) launch_stream<32, 2, 4, 4, 4>(a, stream);
      else launch_stream<32, 2, 2, 4, 8>(a, stream);
      return true;
    case 16:
      if (!wide) launch_stream<16, 1, 4, 4, 4>(a, stream);
      else if (waves8) launch_stream<16, 2, 4, 4, 4>(a, stream);
      else launch_stream<16, 2, 2, 4, 8>(a, stream);
      return true;
    case 8:
      if (!wide) launch_stream<8, 1, 4, 4, 4>(a, stream);
      else if (waves8) launch_stream<8, 2, 4, 4, 4>(a, stream);
      else launch_stream<8, 2, 2, 4, 8>(a, stream);
      return true;
    default:
      return false;
  }
}

}  // namespace commeff
