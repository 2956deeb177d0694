// GPT-2 input embedding for gfx950: e[r] = wte[ids[t]] + wpe[t % L] + wte[tt[t]]
// (t = tok[r], the r-th real token of the padded [N, L] batch) and its
// backward into the fp32 gradient of the (tied) token table and the position
// table.
//
// Reference model: HF GPT2Model.forward (wte(input_ids) + wpe(position_ids) +
// wte(token_type_ids)) of /root/reference/CommEfficient/gpt2_train.py:55-99.
// PyTorch's embedding backward sorts the indices (rocprim radix + merge sort)
// and runs sum_and_scatter + compute_grad_weight per table.  Here the
// backward is order-independent AND deterministic without a sort: every
// gradient element is added in 2^-40 fixed point with 64-bit integer atomics
// (exact: integer addition is associative -- bf16 values of magnitude >= 2^-32
// are represented exactly), into a persistent accumulator of the table's shape;
// the rows touched this call are listed once (first touch), and a flush adds
// them to the fp32 gradient sink and zeroes them for the next call.
// Range: a call adds at most n = (1 or 2) * Mr values into one element, so
// every value below lim = 2^22 / n (a power of two, set by the host) keeps the
// fixed-point sum under 2^62 -- no wrap-around.  Values at or above lim, Inf
// and NaN (which an integer cast would turn into arbitrary finite numbers) go
// to an fp32 spill accumulator instead (float atomics; the key is flagged and
// its flush adds the spill), so a non-finite gradient stays non-finite exactly
// as index_add propagates it and --skip_nonfinite can see it.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdint>
#include "kernels.h"

namespace commeff {
namespace {

typedef uint16_t bf16raw;
constexpr float kFix = 1099511627776.0f;          // 2^40
constexpr double kUnfix = 1.0 / 1099511627776.0;  // 2^-40
constexpr int32_t kSpilled = 1 << 30;             // cnt flag: the key has spill values

__device__ __forceinline__ float bf2f(bf16raw v) { return __uint_as_float(static_cast<uint32_t>(v) << 16); }
__device__ __forceinline__ bf16raw f2bf(float f) {
  const uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return static_cast<bf16raw>((u >> 16) | 0x40u);
  return static_cast<bf16raw>((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

__device__ __forceinline__ int64_t tok_of(const int32_t* tok, int r) { return tok != nullptr ? tok[r] : r; }

// one block (256 threads) per token row, 8 columns per thread and pass
__global__ void __launch_bounds__(256) embed_fwd_kernel(const int64_t* __restrict__ ids,
                                                        const int64_t* __restrict__ tt,
                                                        const int32_t* __restrict__ tok, int L,
                                                        const bf16raw* __restrict__ wte,
                                                        const bf16raw* __restrict__ wpe, bf16raw* __restrict__ out,
                                                        int H) {
  const int r = blockIdx.x;
  const int64_t t = tok_of(tok, r);
  const bf16raw* a = wte + ids[t] * H;
  const bf16raw* p = wpe + (t % L) * H;
  const bf16raw* b = tt != nullptr ? wte + tt[t] * H : nullptr;
  bf16raw* o = out + static_cast<int64_t>(r) * H;
  for (int h = threadIdx.x; h < H; h += 256) {
    float v = bf2f(a[h]) + bf2f(p[h]);
    if (b != nullptr) v += bf2f(b[h]);
    o[h] = f2bf(v);
  }
}

// acc[key][h] += fix(de[r][h]) for the row's key(s); first touch of a key
// appends it to lst (lst[V] = count).  pos != 0: the key is t % L (the
// position table); else ids[t] (and tt[t] when given: the tied token table
// sees both).  A block takes kRB consecutive rows and sums the (exact, integer)
// contributions of equal keys among them first -- the few token-type ids of a
// batch would otherwise serialise thousands of atomics on the same addresses.
constexpr int kRB = 16;

__global__ void __launch_bounds__(256) embed_scatter_kernel(const bf16raw* __restrict__ de,
                                                            const int64_t* __restrict__ ids,
                                                            const int64_t* __restrict__ tt,
                                                            const int32_t* __restrict__ tok, int L, int pos,
                                                            unsigned long long* __restrict__ acc,
                                                            float* __restrict__ spill,
                                                            int32_t* __restrict__ cnt, int32_t* __restrict__ lst,
                                                            int V, int H, int Mr, float lim) {
  __shared__ int64_t skey[2 * kRB];
  __shared__ int sfirst[2 * kRB];
  const int r0 = blockIdx.x * kRB;
  const int nr = min(kRB, Mr - r0);
  const int nq = (!pos && tt != nullptr) ? 2 : 1;
  const int np = nr * nq;  // pairs p = q * nr + row
  if (threadIdx.x < np) {
    const int q = threadIdx.x / nr, i = threadIdx.x - q * nr;
    const int64_t t = tok_of(tok, r0 + i);
    skey[threadIdx.x] = pos ? t % L : (q == 0 ? ids[t] : tt[t]);
  }
  __syncthreads();
  if (threadIdx.x < np) {
    const int64_t k = skey[threadIdx.x];
    int f = threadIdx.x;
    for (int p = 0; p < threadIdx.x; ++p)
      if (skey[p] == k) { f = p; break; }
    sfirst[threadIdx.x] = f;
    // (a spill flag is only ever set after a count increment: old == 0 is the first touch)
    if (f == static_cast<int>(threadIdx.x) && atomicAdd(&cnt[k], 1) == 0)
      lst[atomicAdd(&lst[V], 1)] = static_cast<int32_t>(k);
  }
  __syncthreads();
  for (int h = threadIdx.x; h < H; h += 256) {
    long long v[kRB];
    float fv[kRB];
    uint32_t big = 0;  // rows whose value is out of the fixed-point range (or not finite)
#pragma unroll
    for (int i = 0; i < kRB; ++i) {
      fv[i] = i < nr ? bf2f(de[static_cast<int64_t>(r0 + i) * H + h]) : 0.f;
      const bool ok = fabsf(fv[i]) < lim;  // false for NaN too
      v[i] = ok ? static_cast<long long>(fv[i] * kFix) : 0ll;
      big |= ok ? 0u : (1u << i);
    }
    if (big != 0u) {  // rare path: every (row, key) pair of an out-of-range row
      for (int p = 0; p < np; ++p) {
        const int i2 = p % nr;
        if (!((big >> i2) & 1u)) continue;
        float x = 0.f;
#pragma unroll
        for (int i = 0; i < kRB; ++i)
          if (i == i2) x = fv[i];
        atomicAdd(spill + skey[p] * H + h, x);
        atomicOr(&cnt[skey[p]], kSpilled);
      }
    }
    for (int p = 0; p < np; ++p) {
      if (sfirst[p] != p) continue;
      long long sum = 0;
      for (int p2 = p; p2 < np; ++p2) {
        if (sfirst[p2] != p) continue;
        const int i2 = p2 % nr;
#pragma unroll
        for (int i = 0; i < kRB; ++i)
          if (i == i2) sum += v[i];
      }
      atomicAdd(acc + skey[p] * H + h, static_cast<unsigned long long>(sum));
    }
  }
}

// sink[key][h] += unfix(acc[key][h]) (fp32) and acc / cnt zeroed, for every
// listed key (any order: each row is independent)
__global__ void __launch_bounds__(256) embed_flush_kernel(unsigned long long* __restrict__ acc,
                                                          float* __restrict__ spill,
                                                          int32_t* __restrict__ cnt,
                                                          const int32_t* __restrict__ lst, int V, int H,
                                                          float* __restrict__ sink, int64_t ld) {
  const int n = lst[V];
  for (int j = blockIdx.x; j < n; j += gridDim.x) {
    const int64_t key = lst[j];
    unsigned long long* a = acc + key * H;
    float* sp = spill + key * H;
    float* s = sink + key * ld;
    const bool spilled = (cnt[key] & kSpilled) != 0;
    for (int h = threadIdx.x; h < H; h += 256) {
      const long long v = static_cast<long long>(a[h]);
      double x = static_cast<double>(v) * kUnfix;
      if (spilled) {
        x += static_cast<double>(sp[h]);  // NaN / Inf carry through
        sp[h] = 0.f;
      }
      s[h] += static_cast<float>(x);
      a[h] = 0ull;
    }
    __syncthreads();  // every thread has read the flag
    if (threadIdx.x == 0) cnt[key] = 0;
  }
}

}  // namespace

void launch_embed_fwd(const int64_t* ids, const int64_t* tt, const int32_t* tok, int L, const uint16_t* wte,
                      const uint16_t* wpe, uint16_t* out, int Mr, int H, hipStream_t stream) {
  if (Mr == 0) return;
  COMMEFF_LAUNCH(embed_fwd_kernel, dim3(Mr), dim3(256), 0, stream, ids, tt, tok, L, wte, wpe, out, H);
}

void launch_embed_bwd(const uint16_t* de, const int64_t* ids, const int64_t* tt, const int32_t* tok, int L,
                      int pos, unsigned long long* acc, float* spill, int32_t* cnt, int32_t* lst, int V, int H,
                      float* sink, int64_t ld, int Mr, hipStream_t stream) {
  if (Mr == 0) return;
  // lim = 2^22 / 2^ceil(log2(n)), n = values per element in this call (see top)
  const int n = (!pos && tt != nullptr) ? 2 * Mr : Mr;
  int lg = 0;
  while ((1 << lg) < n) ++lg;
  const float lim = ldexpf(1.f, 22 - lg);
  COMMEFF_LAUNCH(embed_scatter_kernel, dim3((Mr + kRB - 1) / kRB), dim3(256), 0, stream, de, ids, tt, tok, L,
                 pos, acc, spill, cnt, lst, V, H, Mr, lim);
  COMMEFF_LAUNCH(embed_flush_kernel, dim3(1024), dim3(256), 0, stream, acc, spill, cnt, lst, V, H, sink, ld);
  tape_memset(lst + V, 0, sizeof(int32_t), stream);  // the list is empty again
}

}  // namespace commeff
