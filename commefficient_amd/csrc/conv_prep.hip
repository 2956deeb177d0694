// The ResNet-9 input ("prep") convolution: 3x3 / pad 1, Cin <= 4 -> K = 64,
// fused ReLU, on gfx950 (reference ConvBN(c_in, 64),
// /root/reference/CommEfficient/models/resnet9.py:32-59, 118).
//
// With 3 input channels the layer is pure bandwidth: 27 MACs per output.
// The augmentation kernel stores the input batch with a 4-channel pixel
// stride (8 bytes, channel 3 = 0), so one tap of one pixel is one 8-byte load.
//
// Forward: y^T = W x im2col^T on v_mfma_f32_32x32x16_bf16 with the GEMM K
// index = 4*tap + c (36 used, padded to 48 = 3 K-steps).  The weight operand
// lives in registers for the whole kernel; a lane's B fragment of one K-step
// is two taps of one pixel (two 8-byte loads).  Epilogue: ReLU, 8-byte bf16
// stores (a wave writes 32 whole 128-byte output rows), and a 64-bit ReLU
// mask per pixel (two 32-bit words in accumulator order) for the backward.
//
// Weight gradient: dW[k][c][tap] = sum_p g[p][k] x[p + tap][c] with
// g = gy * mask, as a GEMM over pixels on the same MFMA: per 64-pixel step a
// block stages g [64 px][64 k] (masked while loading) and the im2col tile
// [64 px][16 taps x 4 ch] in LDS, and the waves read both operands with the
// transposing ds_read_b64_tr_b16 (pixels become the reduction index).  Global
// loads of step s+1 are in flight during the MFMAs of step s.  Per-block
// partial [64][64] tiles are summed by a second kernel in a fixed order
// (deterministic).  Reads gy once (bf16) and the 8-byte-per-pixel mask
// instead of the 64-channel activation.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdlib>
#include "kernels.h"
#include "conv_common.h"

namespace commeff {
namespace {

typedef uint32_t v2u __attribute__((ext_vector_type(2)));

constexpr int kPrepK = 64;

struct PrepPix {
  int p, h, w;
  bool valid;
};

__device__ __forceinline__ PrepPix prep_pix(const ConvPrepArgs& a, int p) {
  PrepPix r;
  r.valid = p < a.P;
  r.p = r.valid ? p : 0;
  const uint32_t q = fdiv(static_cast<uint32_t>(r.p), a.div_w);
  r.w = r.p - static_cast<int>(q) * a.W;
  r.h = static_cast<int>(q - fdiv(q, a.div_h) * a.H);
  return r;
}

// the 4 channels of tap `tap` of pixel x (8 bytes; zero outside the image / for
// taps >= 9; channel 3 forced to 0 when Cin == 3 so even a NaN there is inert)
__device__ __forceinline__ v2u prep_tap(const ConvPrepArgs& a, const PrepPix& x, int tap) {
  v2u t = {0u, 0u};
  if (tap < 9) {
    const int dr = tap / 3 - 1, ds = tap % 3 - 1;
    const bool ok = x.valid && static_cast<unsigned>(x.h + dr) < static_cast<unsigned>(a.H) &&
                    static_cast<unsigned>(x.w + ds) < static_cast<unsigned>(a.W);
    if (ok) {
      t = *reinterpret_cast<const v2u*>(a.x + static_cast<size_t>(x.p + dr * a.W + ds) * 4);
      if (a.Cin <= 3) t[1] &= 0xffffu;
    }
  }
  return t;
}

// B fragments of one 32-pixel tile: K-step s, lane half hi -> taps 4s+2hi, 4s+2hi+1
__device__ __forceinline__ void prep_load_b(const ConvPrepArgs& a, int tile, int lr, int hi,
                                            bf16x8_t (&b)[3]) {
  const PrepPix x = prep_pix(a, tile * 32 + lr);
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    const v2u t0 = prep_tap(a, x, 4 * s + 2 * hi), t1 = prep_tap(a, x, 4 * s + 2 * hi + 1);
    const v4u v = {t0[0], t0[1], t1[0], t1[1]};
    b[s] = __builtin_bit_cast(bf16x8_t, v);
  }
}

// The same B fragments as raw loads: every tap loaded unconditionally from a
// clamped in-range pixel, validity kept as bits (bit 2s+h: tap 4s+2hi+h) and
// applied by prep_finish_b just before the MFMAs -- a load under a branch is
// waited for inside it, which had serialised the "in flight" next tile
struct PrepRawB {
  v2u t[3][2];
  uint32_t ok;
};
__device__ __forceinline__ void prep_load_b_raw(const ConvPrepArgs& a, int tile, int lr, int hi, PrepRawB& rb) {
  const PrepPix x = prep_pix(a, tile * 32 + lr);
  rb.ok = 0u;
#pragma unroll
  for (int s = 0; s < 3; ++s)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int tap = 4 * s + 2 * hi + h;
      const int dr = tap / 3 - 1, ds = tap % 3 - 1;
      const bool ok = tap < 9 && x.valid && static_cast<unsigned>(x.h + dr) < static_cast<unsigned>(a.H) &&
                      static_cast<unsigned>(x.w + ds) < static_cast<unsigned>(a.W);
      const int src = ok ? x.p + dr * a.W + ds : x.p;
      rb.t[s][h] = *reinterpret_cast<const v2u*>(a.x + static_cast<size_t>(src) * 4);
      rb.ok |= (ok ? 1u : 0u) << (2 * s + h);
    }
}
__device__ __forceinline__ void prep_finish_b(const ConvPrepArgs& a, const PrepRawB& rb, bf16x8_t (&b)[3]) {
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    v2u t0 = ((rb.ok >> (2 * s)) & 1u) ? rb.t[s][0] : v2u{0u, 0u};
    v2u t1 = ((rb.ok >> (2 * s + 1)) & 1u) ? rb.t[s][1] : v2u{0u, 0u};
    if (a.Cin <= 3) {
      t0[1] &= 0xffffu;
      t1[1] &= 0xffffu;
    }
    const v4u v = {t0[0], t0[1], t1[0], t1[1]};
    b[s] = __builtin_bit_cast(bf16x8_t, v);
  }
}

__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 8))) prep_fwd_kernel(ConvPrepArgs a) {
  // weight fragments (row m = 32 mt + lr, GEMM k = 16 s + 8 hi + j -> tap k/4,
  // channel k%4), built once per block in LDS
  __shared__ bf16x8_t wsm[2][3][64];
  // per-wave output staging: 32 pixel rows of 64 channels, 144-byte row pitch
  // (16-byte aligned, 2-way bank aliasing for the 8-byte fragment writes)
  constexpr int kPitch = 144;
  __shared__ __attribute__((aligned(16))) unsigned char ysm[4][32 * kPitch];
  // all 12 loads of a thread in flight together (unrolled, unconditional at a
  // clamped index): a per-element load-wait loop here was a serial prologue
  // of ~12 memory latencies per block
  float wv[12];
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    const int e = threadIdx.x + 256 * i;
    const int j = e & 7, ln = (e >> 3) & 63, ms = e >> 9;  // ms = mt*3 + s
    const int mt = ms / 3, s = ms - 3 * mt;
    const int kk = 16 * s + 8 * (ln >> 5) + j, tap = kk >> 2, c = kk & 3;
    const int m = 32 * mt + (ln & 31);
    const bool ok = tap < 9 && c < a.Cin;
    wv[i] = a.w[ok ? (m * a.Cin + c) * 9 + tap : 0];
    wv[i] = ok ? wv[i] : 0.f;
  }
#pragma unroll
  for (int i = 0; i < 12; ++i)
    reinterpret_cast<__bf16*>(&wsm[0][0][0])[threadIdx.x + 256 * i] = static_cast<__bf16>(wv[i]);
  __syncthreads();
  const int lane = threadIdx.x & 63, lr = lane & 31, hi = lane >> 5;
  bf16x8_t wa[2][3];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int s = 0; s < 3; ++s) wa[mt][s] = wsm[mt][s][lane];
  const int ntiles = (a.P + 31) >> 5;
  const int nwaves = (gridDim.x * 256) >> 6;
  int tile = (blockIdx.x * 256 + threadIdx.x) >> 6;
  if (tile >= ntiles) return;
  // the next tile's loads in flight during this tile's work (measured: two
  // tiles ahead was no faster); past the end they re-read the current tile
  unsigned char* ys = ysm[threadIdx.x >> 6];
  auto body = [&](PrepRawB& rb, int t) {
    bf16x8_t b[3];
    prep_finish_b(a, rb, b);
    const int ahead = t + nwaves;
    prep_load_b_raw(a, ahead < ntiles ? ahead : t, lr, hi, rb);
    f32x16_t acc[2];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[mt][e] = 0.f;
#pragma unroll
      for (int s = 0; s < 3; ++s)
        acc[mt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[mt][s], b[s], acc[mt], 0, 0, 0);
    }
    const int p = t * 32 + lr;
    // lane (pixel p, hi) holds channels 32 mt + 8 g + 4 hi + (0..3) in
    // acc[mt][4 g ..]: ReLU + bf16 into the wave's LDS rows, then whole
    // 128-byte output rows leave with 16-byte stores (8 rows per instruction)
    uint32_t mbits = 0;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v[j] = fmaxf(acc[mt][4 * g + j], 0.f);
          mbits |= (v[j] > 0.f ? 1u : 0u) << (16 * mt + 4 * g + j);
        }
        const v2u o = {pack_bf16(v[0], v[1]), pack_bf16(v[2], v[3])};
        *reinterpret_cast<v2u*>(ys + lr * kPitch + (32 * mt + 8 * g + 4 * hi) * 2) = o;
      }
    if (p < a.P) a.mask[2 * p + hi] = mbits;
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = q * 64 + lane, row = c >> 3, col = c & 7;
      const v4u o = *reinterpret_cast<const v4u*>(ys + row * kPitch + col * 16);
      if (t * 32 + row < a.P)
        *reinterpret_cast<v4u*>(a.y + static_cast<size_t>(t * 32 + row) * kPrepK + col * 8) = o;
    }
    __builtin_amdgcn_wave_barrier();  // rows read before the next tile overwrites them
  };
  PrepRawB rb;
  prep_load_b_raw(a, tile, lr, hi, rb);
  while (true) {
    body(rb, tile);
    tile += nwaves;
    if (tile >= ntiles) break;
  }
}

// Weight gradient.  LDS images (64 rows of 128 B, sw_tr128 swizzle):
// A = g[px][k] (masked gy), B = im2col[px][4 tap + c] (taps 9..15 zero).
// Raw operands of one 64-pixel step as loaded: every load unconditional (a
// clamped in-range address, validity kept as bits and applied when the step
// is staged in LDS) -- a load under a branch is waited for inside it, which
// had left the "prefetched" step serialised behind the MFMAs
struct PrepWgRaw {
  v4u g[2];   // gy chunks (rows (tid + 256 i) >> 3, chunk (tid + 256 i) & 7)
  v2u mw[2];  // the rows' ReLU-mask words
  v2u t[2][2];  // the two taps of the im2col chunk
  uint32_t ok;  // bit 3i: row valid, 3i+1 / 3i+2: tap 0 / 1 inside the image
};

__device__ __forceinline__ void prep_wg_load_raw(const ConvPrepArgs& a, int step, int tid, PrepWgRaw& st) {
  st.ok = 0u;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int id = tid + 256 * i, row = id >> 3, cc = id & 7;
    const PrepPix x = prep_pix(a, step * 64 + row);  // x.p = 0 when invalid
    st.g[i] = *reinterpret_cast<const v4u*>(a.gy + static_cast<size_t>(x.p) * kPrepK + 8 * cc);
    st.mw[i] = *reinterpret_cast<const v2u*>(a.mask_in + 2 * x.p);
    st.ok |= (x.valid ? 1u : 0u) << (3 * i);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int tap = 2 * cc + h;
      const int dr = tap / 3 - 1, ds = tap % 3 - 1;
      const bool ok = tap < 9 && x.valid && static_cast<unsigned>(x.h + dr) < static_cast<unsigned>(a.H) &&
                      static_cast<unsigned>(x.w + ds) < static_cast<unsigned>(a.W);
      const int src = ok ? x.p + dr * a.W + ds : x.p;
      st.t[i][h] = *reinterpret_cast<const v2u*>(a.x + static_cast<size_t>(src) * 4);
      st.ok |= (ok ? 1u : 0u) << (3 * i + 1 + h);
    }
  }
}

// masked gy chunk / im2col chunk of row i of a raw step
__device__ __forceinline__ void prep_wg_finish(const ConvPrepArgs& a, const PrepWgRaw& st, int i, int cc,
                                               v4u* g, v4u* xb) {
  v4u gg = {0u, 0u, 0u, 0u};
  if ((st.ok >> (3 * i)) & 1u) {
    gg = st.g[i];
    // channels 8cc + j: word j >> 2, bit 16 (cc >> 2) + 4 (cc & 3) + (j & 3)
    const int sh = 16 * (cc >> 2) + 4 * (cc & 3);
    const uint32_t m0 = st.mw[i][0] >> sh, m1 = st.mw[i][1] >> sh;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t bits = q < 2 ? m0 : m1;  // element pair q covers channels 2q, 2q+1
      const int j0 = (2 * q) & 3;
      const uint32_t keep = (((bits >> j0) & 1u) ? 0x0000ffffu : 0u) |
                            (((bits >> (j0 + 1)) & 1u) ? 0xffff0000u : 0u);
      gg[q] &= keep;
    }
  }
  *g = gg;
  v2u t0 = ((st.ok >> (3 * i + 1)) & 1u) ? st.t[i][0] : v2u{0u, 0u};
  v2u t1 = ((st.ok >> (3 * i + 2)) & 1u) ? st.t[i][1] : v2u{0u, 0u};
  if (a.Cin <= 3) {
    t0[1] &= 0xffffu;
    t1[1] &= 0xffffu;
  }
  *xb = v4u{t0[0], t0[1], t1[0], t1[1]};
}

__global__ void __launch_bounds__(256) prep_wgrad_kernel(ConvPrepArgs a, int steps_per_block) {
  __shared__ __attribute__((aligned(16))) unsigned char sm[2 * 64 * 128];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int mi = wid >> 1, ni = wid & 1;
  const int nsteps = (a.P + 63) / 64;
  const int s0 = blockIdx.x * steps_per_block, s1 = min(nsteps, s0 + steps_per_block);
  if (s0 >= s1) return;  // (block-uniform)
  int toA[2], toB[2];
  tr_offsets<128>(mi * 32, lane, toA);
  tr_offsets<128>(ni * 32, lane, toB);
  f32x16_t acc;
#pragma unroll
  for (int e = 0; e < 16; ++e) acc[e] = 0.f;
  // two raw stages: the loads of step s + 2 are in flight during the MFMAs
  // of steps s and s + 1 (step indices past the block clamp to its last step)
  PrepWgRaw sa, sb;
  prep_wg_load_raw(a, s0, tid, sa);
  prep_wg_load_raw(a, min(s0 + 1, s1 - 1), tid, sb);
  auto process = [&](const PrepWgRaw& st) __attribute__((always_inline)) {
    // the previous step's operand reads are done (LDS only: the raw stages
    // ahead stay in flight -- __syncthreads would drain them)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int id = tid + 256 * i, row = id >> 3, cc = id & 7;
      const int off = row * 128 + ((cc ^ sw_tr128(row)) << 4);
      v4u g, xb;
      prep_wg_finish(a, st, i, cc, &g, &xb);
      *reinterpret_cast<v4u*>(sm + off) = g;
      *reinterpret_cast<v4u*>(sm + 8192 + off) = xb;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int d = kk * 16 * 128;
      const bf16x8_t af = tr_read(sm + toA[0] + d, sm + toA[1] + d);
      const bf16x8_t bf = tr_read(sm + 8192 + toB[0] + d, sm + 8192 + toB[1] + d);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bf, acc, 0, 0, 0);
    }
  };
  for (int step = s0; step < s1; step += 2) {
    process(sa);
    prep_wg_load_raw(a, min(step + 2, s1 - 1), tid, sa);
    if (step + 1 < s1) {  // (block-uniform)
      process(sb);
      prep_wg_load_raw(a, min(step + 3, s1 - 1), tid, sb);
    }
  }
  // partial[block][k][n], n = 4 tap + c
  float* out = a.partial + static_cast<size_t>(blockIdx.x) * kPrepK * 64;
  const int hi = lane >> 5, lr = lane & 31;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int m = mi * 32 + (e & 3) + 8 * (e >> 2) + 4 * hi;
    out[m * 64 + ni * 32 + lr] = acc[e];
  }
}

// dw[k][c][tap] (= beta * dw +) sum over blocks of partial[b][k][4 tap + c]:
// 16 threads per output, fixed combination order
__global__ void __launch_bounds__(256) prep_wgrad_reduce_kernel(const float* __restrict__ partial,
                                                                int nblocks, int Cin, float* __restrict__ dw,
                                                                float beta) {
  __shared__ float red[16][17];
  const int o = blockIdx.x * 16 + (threadIdx.x & 15), part = threadIdx.x >> 4;  // o = k*27 + c*9 + tap
  const int k = o / 27, r = o - k * 27, c = r / 9, tap = r - 9 * c;
  const bool live = o < kPrepK * 27 && c < Cin;
  float s = 0.f;
  if (live) {
    const float* src = partial + k * 64 + 4 * tap + c;
#pragma unroll 4
    for (int b = part; b < nblocks; b += 16) s += src[static_cast<size_t>(b) * kPrepK * 64];
  }
  red[part][threadIdx.x & 15] = s;
  __syncthreads();
  if (threadIdx.x < 16 && live) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) t += red[q][threadIdx.x];
    float* d = dw + (k * Cin + c) * 9 + tap;
    *d = beta != 0.f ? beta * *d + t : t;
  }
}

}  // namespace

int conv_prep_wgrad_blocks(int P) {
  constexpr int per = 8;  // pixel steps per block (scripts/bench_prep.py sweep)
  const int steps = (P + 63) / 64;
  int b = (steps + per - 1) / per;
  return b < 1024 ? (b < 1 ? 1 : b) : 1024;
}

void launch_conv_prep_fwd(ConvPrepArgs a, hipStream_t stream) {
  a.div_w = make_fastdiv(static_cast<uint32_t>(a.W));
  a.div_h = make_fastdiv(static_cast<uint32_t>(a.H));
  const int ntiles = (a.P + 31) / 32;
  constexpr int tpw = 4;  // tiles per wave (weights set up once per block; bench_prep.py sweep: 4 best)
  int blocks = (ntiles + 4 * tpw - 1) / (4 * tpw);
  if (blocks > 4096) blocks = 4096;
  COMMEFF_LAUNCH(prep_fwd_kernel, dim3(blocks < 1 ? 1 : blocks), dim3(256), 0, stream, a);
}

void launch_conv_prep_wgrad(ConvPrepArgs a, float* dw, float beta, hipStream_t stream) {
  a.div_w = make_fastdiv(static_cast<uint32_t>(a.W));
  a.div_h = make_fastdiv(static_cast<uint32_t>(a.H));
  const int nb = conv_prep_wgrad_blocks(a.P);
  const int steps = (a.P + 63) / 64;
  const int spb = (steps + nb - 1) / nb;
  COMMEFF_LAUNCH(prep_wgrad_kernel, dim3(nb), dim3(256), 0, stream, a, spb);
  COMMEFF_LAUNCH(prep_wgrad_reduce_kernel, dim3((kPrepK * 27 + 15) / 16), dim3(256), 0, stream,
                     a.partial, nb, a.Cin, dw, beta);
}

}  // namespace commeff
