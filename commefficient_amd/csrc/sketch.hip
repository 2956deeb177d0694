// Count-Sketch kernels for gfx950 (MI355X).
//
// Reference semantics: CSVec.accumulateVec / unSketch / zero / l2estimate as
// used at /root/reference/CommEfficient/fed_worker.py:313-320 and
// fed_aggregator.py:584-611.
//
// Design (MI355X-first, not a translation of CSVec's torch code):
//  * hashes are recomputed in registers from 4 u64 coefficients per row that
//    travel in the kernel arguments (SGPRs) -- no r x d index tables;
//  * encode has two forms:
//      - direct: one fp32 global atomic per (coord, row).  Only for sparse
//        inputs: random per-lane atomics run at ~1/17 of the contiguous
//        atomic rate on CDNA4 (MI355X_MICROARCH.md "Global float atomics");
//        a dense 6.5M-coordinate encode measured 1.56 ms;
//      - binned: the hashes are data-independent, so the mapping of every
//        (coordinate, row) entry to its 8192-bucket table tile is fixed.  A
//        one-time layout pass counts entries per (coordinate chunk, tile) and
//        an exclusive scan gives every chunk a private, exactly sized run in
//        every tile's segment of one entry buffer.  Per encode, pass 1 hashes
//        a chunk per workgroup, counting-sorts its (value, bucket) entries by
//        tile in LDS and streams each tile's run out contiguously (no global
//        atomics); pass 2 gives each tile (split over 1-8 workgroups) to
//        workgroups that accumulate its entries with LDS float atomics and
//        fold the tile into the table with coalesced stores / contiguous
//        atomics.  Every global access is a coalesced stream.
//  * query gathers r signed cells per coordinate and takes the lower median
//    (torch.median convention, which CSVec relies on) in registers.
#include <hip/hip_runtime.h>
#include <cstdint>
#include "kernels.h"

namespace commeff {
namespace {

struct HashArgs {
  RowHash row[kMaxRows];
};

constexpr int kTileShift = 13;                 // 8192 buckets per tile
constexpr uint32_t kTile = 1u << kTileShift;   // 32 KiB of LDS in pass 2
constexpr int kStageEntries = 8960;            // pass-1 LDS staging (70 KiB)

struct Entry {
  float v;
  uint32_t gb;  // flat bucket index j*c + bucket
};

__device__ __forceinline__ float load_v(const float* vec, const float* wvec,
                                        float scale, float wscale, uint32_t i) {
  float v = scale * vec[i];
  if (wvec != nullptr) v += wscale * wvec[i];
  return v;
}

// Exclusive prefix of `x` over the 256 threads of a block (4 waves), via
// wave shuffles + one LDS exchange.  `lds4` holds >= 4 u32.
__device__ __forceinline__ uint32_t block_excl_scan256(uint32_t x, uint32_t* lds4) {
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t incl = x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t y = __shfl_up(incl, o);
    if (lane >= static_cast<uint32_t>(o)) incl += y;
  }
  if (lane == 63) lds4[wave] = incl;
  __syncthreads();
  uint32_t base = 0;
  for (uint32_t w = 0; w < wave; ++w) base += lds4[w];
  return base + incl - x;
}

// ------------------------------------------------------------ direct encode
__global__ void __launch_bounds__(256)
cs_encode_direct_kernel(float* __restrict__ table, const float* __restrict__ vec,
                        const float* __restrict__ wvec, float scale, float wscale,
                        HashArgs h, SketchGeom g, const int32_t* __restrict__ blk_off,
                        const float* __restrict__ blk_sign) {
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < g.d; i += stride) {
    float v = load_v(vec, wvec, scale, wscale, i);
    if (v == 0.f) continue;  // sparse inputs: nothing to add
    uint32_t blk, t;
    split_block(i, g, &blk, &t);
    for (uint32_t j = 0; j < g.r; ++j) {
      uint32_t bk;
      float s;
      hash_t(h.row[j], t, blk, g, blk_off + j * g.num_blocks, blk_sign + j * g.num_blocks,
             &bk, &s);
      atomicAdd(table + static_cast<size_t>(j) * g.c + bk, s * v);
    }
  }
}

// --------------------------------------------------------- binned: layout
// counts[chunk][tile] = #entries of the chunk's coordinates (all rows) in tile
__global__ void __launch_bounds__(256)
cs_layout_kernel(HashArgs h, SketchGeom g, const int32_t* __restrict__ blk_off,
                 const float* __restrict__ blk_sign, uint32_t* __restrict__ counts,
                 uint32_t num_tiles, uint32_t chunk) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint32_t* cnt = reinterpret_cast<uint32_t*>(smem);
  for (uint32_t t = threadIdx.x; t < num_tiles; t += blockDim.x) cnt[t] = 0;
  __syncthreads();
  const uint32_t i0 = blockIdx.x * chunk;
  const uint32_t i1 = min(g.d, i0 + chunk);
  for (uint32_t i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
    uint32_t blk, t;
    split_block(i, g, &blk, &t);
    for (uint32_t j = 0; j < g.r; ++j) {
      uint32_t bk;
      float s;
      hash_t(h.row[j], t, blk, g, blk_off + j * g.num_blocks, blk_sign + j * g.num_blocks,
             &bk, &s);
      atomicAdd(cnt + ((j * g.c + bk) >> kTileShift), 1u);
    }
  }
  __syncthreads();
  uint32_t* out = counts + static_cast<size_t>(blockIdx.x) * num_tiles;
  for (uint32_t t = threadIdx.x; t < num_tiles; t += blockDim.x) out[t] = cnt[t];
}

// --------------------------------------------------------- binned: pass 1
// base[chunk][tile] = global entry index where this chunk's run in the
// tile's segment starts (exclusive scan over chunks + segment start).
__global__ void __launch_bounds__(256)
cs_bin_kernel(const float* __restrict__ vec, const float* __restrict__ wvec, float scale,
              float wscale, HashArgs h, SketchGeom g, const int32_t* __restrict__ blk_off,
              const float* __restrict__ blk_sign, const uint32_t* __restrict__ counts,
              const uint32_t* __restrict__ base, Entry* __restrict__ entries,
              uint32_t num_tiles, uint32_t chunk) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  // carve: staging[kStageEntries] | lds4[4] | off | cur | gbase (num_tiles each)
  Entry* stage = reinterpret_cast<Entry*>(smem);
  uint32_t* lds4 = reinterpret_cast<uint32_t*>(stage + kStageEntries);
  uint32_t* off = lds4 + 4;
  uint32_t* cur = off + num_tiles;
  uint32_t* gbase = cur + num_tiles;

  const size_t row0 = static_cast<size_t>(blockIdx.x) * num_tiles;
  // local offsets: exclusive scan of this chunk's per-tile counts
  const uint32_t per = (num_tiles + blockDim.x - 1) / blockDim.x;
  const uint32_t t0 = threadIdx.x * per;
  const uint32_t t1 = min(num_tiles, t0 + per);
  uint32_t acc = 0;
  for (uint32_t t = t0; t < t1; ++t) acc += counts[row0 + t];
  acc = block_excl_scan256(acc, lds4);
  for (uint32_t t = t0; t < t1; ++t) {
    off[t] = acc;
    cur[t] = acc;
    acc += counts[row0 + t];
    gbase[t] = base[row0 + t];
  }
  __syncthreads();

  // counting-sort the chunk's entries into LDS staging
  const uint32_t i0 = blockIdx.x * chunk;
  const uint32_t i1 = min(g.d, i0 + chunk);
  for (uint32_t i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
    const float v = load_v(vec, wvec, scale, wscale, i);
    uint32_t blk, t;
    split_block(i, g, &blk, &t);
    for (uint32_t j = 0; j < g.r; ++j) {
      uint32_t bk;
      float s;
      hash_t(h.row[j], t, blk, g, blk_off + j * g.num_blocks, blk_sign + j * g.num_blocks,
             &bk, &s);
      const uint32_t gb = j * g.c + bk;
      const uint32_t pos = atomicAdd(cur + (gb >> kTileShift), 1u);
      stage[pos] = Entry{s * v, gb};
    }
  }
  __syncthreads();

  // stream out: consecutive threads write consecutive slots of one tile run
  const uint32_t total = (i1 > i0 ? (i1 - i0) : 0u) * g.r;
  for (uint32_t e = threadIdx.x; e < total; e += blockDim.x) {
    const Entry en = stage[e];
    const uint32_t t = en.gb >> kTileShift;
    entries[static_cast<size_t>(gbase[t]) + (e - off[t])] = en;
  }
}

// --------------------------------------------------------- binned: pass 2
// grid = num_tiles * splits.  Block (t, s) accumulates its 1/splits share of
// tile t's segment [seg[t], seg[t+1]) in LDS (ds_add_f32), then folds the
// partial tile into the table: plain read-modify-write when it owns the tile,
// else contiguous global atomics (256 B per wave-instruction: the full-rate
// atomic shape).  Entries are read as 16-byte pairs, 4 pairs in flight per
// thread.
__global__ void __launch_bounds__(1024)
cs_accum_kernel(float* __restrict__ table, const uint32_t* __restrict__ seg,
                const Entry* __restrict__ entries, uint32_t total_buckets, uint32_t splits) {
  __shared__ float tile[kTile];
  const uint32_t t = blockIdx.x / splits;
  const uint32_t s = blockIdx.x - t * splits;
  for (uint32_t b = threadIdx.x; b < kTile; b += blockDim.x) tile[b] = 0.f;
  const uint32_t lo = seg[t], hi = seg[t + 1];
  const uint32_t n = hi - lo;
  // split boundaries on even global indices so every range starts 16-B aligned
  uint32_t e0 = lo + static_cast<uint32_t>(static_cast<uint64_t>(n) * s / splits);
  uint32_t e1 = s + 1 == splits ? hi : lo + static_cast<uint32_t>(static_cast<uint64_t>(n) * (s + 1) / splits);
  e0 = (s == 0) ? lo : (e0 & ~1u);
  if (s + 1 != splits) e1 &= ~1u;
  __syncthreads();
  // scalar head so the pair loop starts 16-B aligned
  uint32_t a0 = e0;
  if ((a0 & 1u) && a0 < e1) {
    if (threadIdx.x == 0) {
      Entry en = entries[a0];
      atomicAdd(tile + (en.gb & (kTile - 1)), en.v);
    }
    ++a0;
  }
  const uint32_t np = (e1 - a0) / 2;
  const uint4* pairs = reinterpret_cast<const uint4*>(entries + a0);
  uint32_t p = threadIdx.x;
  for (; p + 3 * blockDim.x < np; p += 4 * blockDim.x) {
    uint4 q[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) q[u] = pairs[p + u * blockDim.x];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      atomicAdd(tile + (q[u].y & (kTile - 1)), __uint_as_float(q[u].x));
      atomicAdd(tile + (q[u].w & (kTile - 1)), __uint_as_float(q[u].z));
    }
  }
  for (; p < np; p += blockDim.x) {
    uint4 q = pairs[p];
    atomicAdd(tile + (q.y & (kTile - 1)), __uint_as_float(q.x));
    atomicAdd(tile + (q.w & (kTile - 1)), __uint_as_float(q.z));
  }
  if (((e1 - a0) & 1u) && threadIdx.x == 0) {  // scalar tail
    Entry en = entries[e1 - 1];
    atomicAdd(tile + (en.gb & (kTile - 1)), en.v);
  }
  __syncthreads();
  const uint32_t tb = t << kTileShift;
  for (uint32_t b = threadIdx.x; b < kTile; b += blockDim.x) {
    uint32_t gb = tb + b;
    float v = tile[b];
    if (gb < total_buckets && v != 0.f) {
      if (splits == 1) table[gb] += v;
      else atomicAdd(table + gb, v);
    }
  }
}

// -------------------------------------------------------------------- query
// Lower median (torch.median convention, which CSVec relies on) of the first
// r values.  Branch-free odd-even transposition network over a statically
// indexed register array: unused slots are +inf so they sort to the end.
// R > 0 fixes r at compile time (R = 5 -> 10 compare-exchanges).
template <int R>
__device__ __forceinline__ float lower_median(float (&v)[kMaxRows], int r) {
  constexpr int N = R > 0 ? R : kMaxRows;
  if (R == 0) {
#pragma unroll
    for (int q = 0; q < N; ++q)
      if (q >= r) v[q] = __builtin_huge_valf();
  }
#pragma unroll
  for (int pass = 0; pass < N; ++pass) {
#pragma unroll
    for (int q = pass & 1; q + 1 < N; q += 2) {
      float a = v[q], b = v[q + 1];
      v[q] = fminf(a, b);
      v[q + 1] = fmaxf(a, b);
    }
  }
  if (R > 0) return v[(N - 1) / 2];
  const int m = (r - 1) / 2;
  float res = v[0];
#pragma unroll
  for (int q = 0; q < N; ++q)
    if (q == m) res = v[q];
  return res;
}

template <int R>
__global__ void __launch_bounds__(256)
cs_query_kernel(const float* __restrict__ table, float* __restrict__ est, HashArgs h,
                SketchGeom g, const int32_t* __restrict__ blk_off,
                const float* __restrict__ blk_sign) {
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < g.d; i += stride) {
    float v[kMaxRows];
    const int r = R > 0 ? R : static_cast<int>(g.r);
    uint32_t blk, t;
    split_block(i, g, &blk, &t);
#pragma unroll
    for (int j = 0; j < (R > 0 ? R : kMaxRows); ++j) {
      v[j] = 0.f;
      if (j >= r) continue;
      uint32_t bk;
      float s;
      hash_t(h.row[j], t, blk, g, blk_off + j * g.num_blocks, blk_sign + j * g.num_blocks,
             &bk, &s);
      v[j] = s * table[static_cast<size_t>(j) * g.c + bk];
    }
    est[i] = lower_median<R>(v, r);
  }
}

// ------------------------------------------------------- row-wise query
// Two-pass query for large d (no plan needed): pass j gathers row j only,
// vals[j][i] = s_j(i) table[j][h_j(i)] -- one 2 MB table row is re-read by
// every XCD from its own L2 instead of the whole r x c table from the MALL;
// then a streaming pass takes the lower median of the r rows per coordinate.
__global__ void __launch_bounds__(256)
cs_query_row_kernel(const float* __restrict__ trow, float* __restrict__ vrow, HashArgs h,
                    SketchGeom g, const int32_t* __restrict__ blk_off,
                    const float* __restrict__ blk_sign, uint32_t j) {
  const uint32_t stride = gridDim.x * blockDim.x;
  const RowHash hr = h.row[j];
  for (uint32_t i0 = blockIdx.x * blockDim.x + threadIdx.x; i0 < g.d; i0 += 4 * stride) {
    float v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint32_t i = i0 + u * stride;
      v[u] = 0.f;
      if (i < g.d) {
        uint32_t blk, t, bk;
        float sg;
        split_block(i, g, &blk, &t);
        hash_t(hr, t, blk, g, blk_off + j * g.num_blocks, blk_sign + j * g.num_blocks, &bk, &sg);
        v[u] = sg * trow[bk];
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint32_t i = i0 + u * stride;
      if (i < g.d) vrow[i] = v[u];
    }
  }
}

template <int R>
__global__ void __launch_bounds__(256)
cs_median_rows_kernel(const float* __restrict__ vals, float* __restrict__ est, uint32_t d,
                      uint32_t r_rt) {
  const uint32_t stride = gridDim.x * blockDim.x;
  const int r = R > 0 ? R : static_cast<int>(r_rt);
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < d; i += stride) {
    float v[kMaxRows];
#pragma unroll
    for (int j = 0; j < (R > 0 ? R : kMaxRows); ++j) v[j] = j < r ? vals[static_cast<size_t>(j) * d + i] : 0.f;
    est[i] = lower_median<R>(v, r);
  }
}

// ------------------------------------------------------------- zero buckets
__global__ void __launch_bounds__(256)
cs_zero_kernel(float* __restrict__ t1, float* __restrict__ t2,
               const int64_t* __restrict__ idx, const float* __restrict__ vals,
               int64_t k, HashArgs h, SketchGeom g, const int32_t* __restrict__ blk_off,
               const float* __restrict__ blk_sign) {
  int64_t q = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
  if (q >= k) return;
  if (vals != nullptr && vals[q] == 0.f) return;  // S(delta) has no mass here
  uint32_t blk, t;
  split_block(static_cast<uint32_t>(idx[q]), g, &blk, &t);
  for (uint32_t j = 0; j < g.r; ++j) {
    uint32_t bk;
    float s;
    hash_t(h.row[j], t, blk, g, blk_off + j * g.num_blocks, blk_sign + j * g.num_blocks, &bk,
           &s);
    size_t cell = static_cast<size_t>(j) * g.c + bk;
    t1[cell] = 0.f;
    if (t2 != nullptr) t2[cell] = 0.f;
  }
}

// -------------------------------------------------------------- l2estimate
__global__ void __launch_bounds__(256)
row_sqsum_kernel(const float* __restrict__ table, int64_t c, float* __restrict__ partial) {
  // grid (nb, r): partial[row * nb + blk]
  const int row = blockIdx.y;
  const float* t = table + row * c;
  float acc = 0.f;
  for (int64_t i = blockIdx.x * blockDim.x + threadIdx.x; i < c;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    float x = t[i];
    acc += x * x;
  }
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o);
  __shared__ float ws[4];
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) partial[row * gridDim.x + blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

__global__ void l2est_final_kernel(const float* __restrict__ partial, int r, int nb,
                                   float* __restrict__ out) {
  // tiny: one thread per row, then thread 0 takes the lower median
  __shared__ float rows[kMaxRows];
  if (threadIdx.x < r) {
    float acc = 0.f;
    for (int b = 0; b < nb; ++b) acc += partial[threadIdx.x * nb + b];
    rows[threadIdx.x] = acc;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float v[kMaxRows];
#pragma unroll
    for (int j = 0; j < kMaxRows; ++j) v[j] = j < r ? rows[j] : 0.f;
    out[0] = sqrtf(lower_median<0>(v, r));
  }
}

HashArgs to_args(const RowHashes& h, const SketchGeom& g) {
  HashArgs a;
  for (uint32_t j = 0; j < g.r && j < static_cast<uint32_t>(kMaxRows); ++j) a.row[j] = h.row[j];
  return a;
}

int grid_for(int64_t n, int block, int max_blocks) {
  int64_t b = (n + block - 1) / block;
  if (b < 1) b = 1;
  return static_cast<int>(b < max_blocks ? b : max_blocks);
}

size_t bin_lds_bytes(const BinPlan& p) {
  return kStageEntries * sizeof(Entry) + (4 + 3 * p.num_tiles) * sizeof(uint32_t);
}

}  // namespace

void launch_cs_encode(float* table, const float* vec, const float* wvec, float scale,
                      float wscale, const RowHashes& h, const SketchGeom& g,
                      const int32_t* blk_off, const float* blk_sign, hipStream_t stream) {
  if (g.d == 0) return;
  COMMEFF_LAUNCH(cs_encode_direct_kernel, dim3(grid_for(g.d, 256, 8192)), dim3(256), 0,
                     stream, table, vec, wvec, scale, wscale, to_args(h, g), g, blk_off,
                     blk_sign);
}

BinPlan plan_cs_encode_binned(const SketchGeom& g) {
  BinPlan p;
  p.tile = kTile;
  int64_t total = static_cast<int64_t>(g.r) * g.c;
  p.num_tiles = (total + kTile - 1) / kTile;
  int64_t chunk = (kStageEntries / static_cast<int64_t>(g.r)) / 64 * 64;
  if (chunk < 64) chunk = 64;
  p.chunk = chunk;
  p.num_chunks = (static_cast<int64_t>(g.d) + chunk - 1) / chunk;
  p.cap = static_cast<int64_t>(g.d) * g.r;  // entries (exact)
  return p;
}

int64_t cs_encode_binned_scratch_bytes(const BinPlan& p) {
  return p.cap * static_cast<int64_t>(sizeof(Entry));
}

bool cs_binned_supported(const BinPlan& p) {
  return p.num_tiles <= 2048 && bin_lds_bytes(p) <= 160 * 1024 && p.cap < (1ll << 32);
}

void launch_cs_layout(const RowHashes& h, const SketchGeom& g, const int32_t* blk_off,
                      const float* blk_sign, const BinPlan& p, uint32_t* counts,
                      hipStream_t stream) {
  if (g.d == 0) return;
  size_t lds = p.num_tiles * sizeof(uint32_t);
  COMMEFF_LAUNCH(cs_layout_kernel, dim3(static_cast<uint32_t>(p.num_chunks)), dim3(256), lds,
                     stream, to_args(h, g), g, blk_off, blk_sign, counts,
                     static_cast<uint32_t>(p.num_tiles), static_cast<uint32_t>(p.chunk));
}

void launch_cs_encode_binned(float* table, const float* vec, const float* wvec, float scale,
                             float wscale, const RowHashes& h, const SketchGeom& g,
                             const int32_t* blk_off, const float* blk_sign, const BinPlan& p,
                             const uint32_t* counts, const uint32_t* base, const uint32_t* seg,
                             void* entries_buf, hipStream_t stream) {
  if (g.d == 0) return;
  Entry* entries = reinterpret_cast<Entry*>(entries_buf);
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(cs_bin_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  COMMEFF_LAUNCH(cs_bin_kernel, dim3(static_cast<uint32_t>(p.num_chunks)), dim3(256),
                     bin_lds_bytes(p), stream, vec, wvec, scale, wscale, to_args(h, g), g,
                     blk_off, blk_sign, counts, base, entries,
                     static_cast<uint32_t>(p.num_tiles), static_cast<uint32_t>(p.chunk));
  // enough workgroups to cover the 256 CUs ~2x
  uint32_t splits = static_cast<uint32_t>((512 + p.num_tiles - 1) / p.num_tiles);
  if (splits < 1) splits = 1;
  if (splits > 8) splits = 8;
  COMMEFF_LAUNCH(cs_accum_kernel, dim3(static_cast<uint32_t>(p.num_tiles) * splits),
                     dim3(1024), 0, stream, table, seg, entries,
                     static_cast<uint32_t>(static_cast<int64_t>(g.r) * g.c), splits);
}

void launch_cs_query(const float* table, float* est, const RowHashes& h, const SketchGeom& g,
                     const int32_t* blk_off, const float* blk_sign, hipStream_t stream) {
  if (g.d == 0) return;
  dim3 grid(grid_for(g.d, 256, 16384));
  HashArgs a = to_args(h, g);
  switch (g.r) {
    case 1: COMMEFF_LAUNCH(cs_query_kernel<1>, grid, dim3(256), 0, stream, table, est, a, g, blk_off, blk_sign); break;
    case 3: COMMEFF_LAUNCH(cs_query_kernel<3>, grid, dim3(256), 0, stream, table, est, a, g, blk_off, blk_sign); break;
    case 5: COMMEFF_LAUNCH(cs_query_kernel<5>, grid, dim3(256), 0, stream, table, est, a, g, blk_off, blk_sign); break;
    case 7: COMMEFF_LAUNCH(cs_query_kernel<7>, grid, dim3(256), 0, stream, table, est, a, g, blk_off, blk_sign); break;
    default: COMMEFF_LAUNCH(cs_query_kernel<0>, grid, dim3(256), 0, stream, table, est, a, g, blk_off, blk_sign); break;
  }
}

void launch_cs_query_rows(const float* table, float* vals, float* est, const RowHashes& h,
                          const SketchGeom& g, const int32_t* blk_off, const float* blk_sign,
                          hipStream_t stream) {
  if (g.d == 0) return;
  HashArgs a = to_args(h, g);
  const dim3 grid(grid_for(g.d, 1024, 8192));
  for (uint32_t j = 0; j < g.r; ++j)
    COMMEFF_LAUNCH(cs_query_row_kernel, grid, dim3(256), 0, stream, table + static_cast<size_t>(j) * g.c,
                       vals + static_cast<size_t>(j) * g.d, a, g, blk_off, blk_sign, j);
  const dim3 g2(grid_for(g.d, 256, 16384));
  switch (g.r) {
    case 5: COMMEFF_LAUNCH(cs_median_rows_kernel<5>, g2, dim3(256), 0, stream, vals, est, g.d, g.r); break;
    case 3: COMMEFF_LAUNCH(cs_median_rows_kernel<3>, g2, dim3(256), 0, stream, vals, est, g.d, g.r); break;
    case 1: COMMEFF_LAUNCH(cs_median_rows_kernel<1>, g2, dim3(256), 0, stream, vals, est, g.d, g.r); break;
    default: COMMEFF_LAUNCH(cs_median_rows_kernel<0>, g2, dim3(256), 0, stream, vals, est, g.d, g.r); break;
  }
}

void launch_cs_zero_buckets(float* t1, float* t2, const int64_t* idx, const float* vals,
                            int64_t k, const RowHashes& h, const SketchGeom& g,
                            const int32_t* blk_off, const float* blk_sign, hipStream_t stream) {
  if (k <= 0) return;
  COMMEFF_LAUNCH(cs_zero_kernel, dim3((k + 255) / 256), dim3(256), 0, stream, t1, t2, idx,
                     vals, k, to_args(h, g), g, blk_off, blk_sign);
}

void launch_cs_l2estimate(const float* table, int r, int64_t c, float* partial, float* out,
                          hipStream_t stream) {
  const int nb = 256;
  COMMEFF_LAUNCH(row_sqsum_kernel, dim3(nb, r), dim3(256), 0, stream, table, c, partial);
  COMMEFF_LAUNCH(l2est_final_kernel, dim3(1), dim3(64), 0, stream, partial, r, nb, out);
}

}  // namespace commeff
