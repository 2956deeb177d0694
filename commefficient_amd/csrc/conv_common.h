// Device helpers shared by the MFMA convolution kernels (conv.hip,
// conv_prep.hip): bf16 vector types, the XCD-aware block remap, the LDS image
// swizzles and the transposing LDS reads (ds_read_b64_tr_b16, gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace commeff {
namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef short s16x8_t __attribute__((ext_vector_type(8)));
typedef uint32_t v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float bf2f(uint32_t h) { return __uint_as_float(h << 16); }
__device__ __forceinline__ uint32_t pack_bf16(float a, float b) {
  const bf16x2_t t = {static_cast<__bf16>(a), static_cast<__bf16>(b)};
  return __builtin_bit_cast(uint32_t, t);
}

// bijective XCD remap: blocks are dispatched round-robin over 8 XCDs; logical
// tiles l and l+1 land on the same XCD
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// ---- LDS image swizzles (16-byte chunk index XOR a function of the row)
// 128-byte rows, ds_read_b128 of 16 consecutive rows at one chunk: conflict-free
__device__ __forceinline__ int sw_rd128(int row) { return (row >> 1) & 7; }
// 256-byte rows, 32x32x16 transposed reads: T10 (b)
__device__ __forceinline__ int sw_tr256(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }
// 128-byte rows, transposed reads: rows k and k+2 of a 4-row block differ in bit 2
__device__ __forceinline__ int sw_tr128(int row) { return ((row >> 1) & 1) << 2; }

template <int ROWB>
__device__ __forceinline__ int tr_off(int row, int ch) {
  if constexpr (ROWB == 256) return row * 256 + ((ch ^ sw_tr256(row)) << 4);
  else return row * 128 + ((ch ^ sw_tr128(row)) << 4);
}

// one 32(col) x 16(k) MFMA operand from an image [k rows][cols]: lane holds
// col = cb + (lane & 31), k = 8 * (lane >> 5) + j (T10 recipe: lane 4q+p of a
// 16-lane group addresses row q, columns 4p..4p+3 of its 4 x 16 block).
// Sub-step kk reads rows +16 kk: with either swizzle the XOR term is the same.
template <int ROWB>
__device__ __forceinline__ void tr_offsets(int cb, int lane, int (&off)[2]) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int col = cb + 16 * (g & 1) + 4 * p;
  const int row = 8 * (g >> 1) + q;
  const int chk = col >> 3, inb = (p & 1) * 8;
  off[0] = tr_off<ROWB>(row, chk) + inb;
  off[1] = tr_off<ROWB>(row + 4, chk) + inb;
}

__device__ __forceinline__ bf16x8_t tr_read(const unsigned char* a0, const unsigned char* a1) {
  typedef __attribute__((address_space(3))) s16x4_t lds_s16x4_t;
  const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)a0);
  const s16x4_t up = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)a1);
  const s16x8_t r = {lo[0], lo[1], lo[2], lo[3], up[0], up[1], up[2], up[3]};
  return __builtin_bit_cast(bf16x8_t, r);
}

}  // namespace
}  // namespace commeff
