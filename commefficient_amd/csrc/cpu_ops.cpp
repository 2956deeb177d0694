// Host (CPU) implementations of the codec ops.  Same semantics as the HIP
// kernels; used for `--device cpu` runs (the gloo plumbing configuration of
// BASELINE.json) and as the native CPU backend in the non-GPU test suite.
// Parallelised with at::parallel_for; the sketch encode is parallel over rows
// (each row is owned by one thread), which also makes it deterministic.
#include <ATen/ATen.h>
#include <ATen/Parallel.h>
#include <torch/library.h>

#include <algorithm>
#include <cmath>
#include <vector>

#include "cpu_ops.h"

namespace commeff {
namespace cpu {

namespace {
inline float lower_median(float* v, int r) {
  std::sort(v, v + r);
  return v[(r - 1) / 2];
}

inline uint64_t splitmix(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
}  // namespace

void cs_encode(float* table, const float* vec, const float* wvec, float scale, float wscale,
               const RowHashes& h, const SketchGeom& g, const int32_t* blk_off,
               const float* blk_sign) {
  at::parallel_for(0, g.r, 1, [&](int64_t j0, int64_t j1) {
    for (int64_t j = j0; j < j1; ++j) {
      float* row = table + j * static_cast<int64_t>(g.c);
      const int32_t* bo = blk_off ? blk_off + j * g.num_blocks : nullptr;
      const float* bsg = blk_sign ? blk_sign + j * g.num_blocks : nullptr;
      for (uint32_t i = 0; i < g.d; ++i) {
        float v = scale * vec[i];
        if (wvec) v += wscale * wvec[i];
        if (v == 0.f) continue;
        uint32_t bk;
        float s;
        hash_coord(h.row[j], i, g, bo, bsg, &bk, &s);
        row[bk] += s * v;
      }
    }
  });
}

void cs_query(const float* table, float* est, const RowHashes& h, const SketchGeom& g,
              const int32_t* blk_off, const float* blk_sign) {
  at::parallel_for(0, g.d, 4096, [&](int64_t i0, int64_t i1) {
    float v[kMaxRows];
    for (int64_t i = i0; i < i1; ++i) {
      for (uint32_t j = 0; j < g.r; ++j) {
        uint32_t bk;
        float s;
        hash_coord(h.row[j], static_cast<uint32_t>(i), g,
                   blk_off ? blk_off + j * g.num_blocks : nullptr,
                   blk_sign ? blk_sign + j * g.num_blocks : nullptr, &bk, &s);
        v[j] = s * table[j * static_cast<int64_t>(g.c) + bk];
      }
      est[i] = lower_median(v, static_cast<int>(g.r));
    }
  });
}

void cs_zero_buckets(float* t1, float* t2, const int64_t* idx, const float* vals, int64_t k,
                     const RowHashes& h, const SketchGeom& g, const int32_t* blk_off,
                     const float* blk_sign) {
  for (int64_t q = 0; q < k; ++q) {
    if (vals && vals[q] == 0.f) continue;
    uint32_t i = static_cast<uint32_t>(idx[q]);
    for (uint32_t j = 0; j < g.r; ++j) {
      uint32_t bk;
      float s;
      hash_coord(h.row[j], i, g, blk_off ? blk_off + j * g.num_blocks : nullptr,
                 blk_sign ? blk_sign + j * g.num_blocks : nullptr, &bk, &s);
      int64_t cell = j * static_cast<int64_t>(g.c) + bk;
      t1[cell] = 0.f;
      if (t2) t2[cell] = 0.f;
    }
  }
}

float cs_l2estimate(const float* table, int r, int64_t c) {
  std::vector<float> rows(r);
  for (int j = 0; j < r; ++j) {
    double acc = 0;
    for (int64_t b = 0; b < c; ++b) {
      float x = table[j * c + b];
      acc += static_cast<double>(x) * x;
    }
    rows[j] = static_cast<float>(acc);
  }
  return std::sqrt(lower_median(rows.data(), r));
}

void topk_abs(const float* x, int64_t n, int64_t k, int64_t* idx, float* vals) {
  // same selection rule as the GPU radix select: k largest |x| keys
  // (bits & 0x7fffffff), ties -> lower index, output in ascending index order
  if (k <= 0) return;
  std::vector<uint32_t> keys(n);
  for (int64_t i = 0; i < n; ++i) {
    uint32_t u;
    std::memcpy(&u, x + i, 4);
    keys[i] = u & 0x7fffffffu;
  }
  std::vector<uint32_t> tmp(keys);
  const int64_t kk = std::min(k, n);
  std::nth_element(tmp.begin(), tmp.begin() + (kk - 1), tmp.end(), std::greater<uint32_t>());
  const uint32_t thr = tmp[kk - 1];
  int64_t gt = 0;
  for (int64_t i = 0; i < n; ++i) gt += keys[i] > thr;
  int64_t ties = kk - gt, pos = 0;
  for (int64_t i = 0; i < n && pos < kk; ++i) {
    bool sel = keys[i] > thr;
    if (!sel && keys[i] == thr && ties > 0) {
      sel = true;
      --ties;
    }
    if (sel) {
      idx[pos] = i;
      vals[pos] = x[i];
      ++pos;
    }
  }
}

void momentum_ef(float* V, float* E, const float* G, int64_t n, float rho, float gscale,
                 int mode) {
  at::parallel_for(0, n, 1 << 14, [&](int64_t a, int64_t b) {
    for (int64_t i = a; i < b; ++i) {
      float v = rho * V[i] + gscale * G[i];
      V[i] = v;
      if (mode == 1) E[i] += v;
      else if (mode == 2) E[i] = v;
    }
  });
}

void sparse_apply(float* w, const int64_t* idx, const float* vals, int64_t k, float lr,
                  const float* lr_vec, int32_t* last_mod, int32_t round, int32_t* hist) {
  for (int64_t q = 0; q < k; ++q) {
    int64_t i = idx[q];
    float l = lr_vec ? lr_vec[i] : lr;
    float old = w[i], nw = old - l * vals[q];
    w[i] = nw;
    if (last_mod && nw != old) {
      const int32_t from = last_mod[i];
      last_mod[i] = round;
      if (hist && from != round) {
        --hist[from + 1];
        ++hist[round + 1];
      }
    }
  }
}

void dense_apply(float* w, const float* delta, int64_t n, float lr, const float* lr_vec,
                 int32_t* last_mod, int32_t round, int32_t* hist) {
  // serial when the change histogram is maintained (shared counters)
  const int64_t grain = hist ? n + 1 : (1 << 14);
  at::parallel_for(0, n, grain, [&](int64_t a, int64_t b) {
    for (int64_t i = a; i < b; ++i) {
      float l = lr_vec ? lr_vec[i] : lr;
      float old = w[i], nw = old - l * delta[i];
      w[i] = nw;
      if (last_mod && nw != old) {
        const int32_t from = last_mod[i];
        last_mod[i] = round;
        if (hist && from != round) {
          --hist[from + 1];
          ++hist[round + 1];
        }
      }
    }
  });
}

void account_hist(const int32_t* hist, int nbins, const int64_t* meta, int W, double* client_dl,
                  double* client_ul, double upc, double* dl) {
  std::vector<int64_t> suffix(nbins + 1, 0);
  for (int b = nbins - 1; b >= 0; --b) suffix[b] = suffix[b + 1] + hist[b];
  for (int j = 0; j < W; ++j) {
    int64_t b0 = meta[j] + 1;
    if (b0 < 0) b0 = 0;
    const double v = 4.0 * static_cast<double>(b0 < nbins ? suffix[b0] : 0);
    const int64_t c = meta[W + j];
    dl[j] = v;
    client_dl[c] += v;
    client_ul[c] += upc;
  }
}

void count_ge(const int32_t* last_mod, int64_t n, const int32_t* thr, int T, int64_t* out) {
  std::vector<int64_t> bins(T + 1, 0);
  for (int64_t i = 0; i < n; ++i) {
    int64_t lo = std::upper_bound(thr, thr + T, last_mod[i]) - thr;
    bins[lo]++;
  }
  int64_t run = 0;
  for (int b = T; b >= 1; --b) {
    run += bins[b];
    out[b - 1] = run;
  }
}

void axpby(float* out, const float* a, float alpha, const float* b, float beta, int64_t n) {
  at::parallel_for(0, n, 1 << 14, [&](int64_t s, int64_t e) {
    for (int64_t i = s; i < e; ++i) out[i] = alpha * a[i] + (b ? beta * b[i] : 0.f);
  });
}

float l2norm(const float* x, int64_t n) {
  double acc = 0;
  for (int64_t i = 0; i < n; ++i) acc += static_cast<double>(x[i]) * x[i];
  return static_cast<float>(std::sqrt(acc));
}

void clip_noise(float* x, int64_t n, const float* norm, float clip, float noise_std,
                uint64_t seed, uint64_t offset) {
  float scale = 1.f;
  if (clip > 0.f && norm && norm[0] > clip) scale = clip / norm[0];
  for (int64_t i = 0; i < n; ++i) {
    float v = x[i] * scale;
    if (noise_std != 0.f) {
      uint64_t r = splitmix(seed ^ splitmix(offset + static_cast<uint64_t>(i)));
      float u1 = ((r >> 40) + 0.5f) / 16777216.f;
      float u2 = (((r >> 16) & 0xffffff) + 0.5f) / 16777216.f;
      v += noise_std * std::sqrt(-2.f * std::log(u1)) * std::cos(6.28318530718f * u2);
    }
    x[i] = v;
  }
}

void client_state(const float* g, float* u, float* e, int64_t n, float rho) {
  at::parallel_for(0, n, 1 << 14, [&](int64_t s, int64_t t) {
    for (int64_t i = s; i < t; ++i) {
      float v = g[i];
      if (u) {
        v = rho * u[i] + v;
        u[i] = v;
      }
      if (e) e[i] += v;
    }
  });
}

void augment_u8_nhwc(const uint8_t* data, const int64_t* idx, int64_t B, int H, int W, int C,
                     int pad, int flip, const float* mean, const float* inv_std, uint64_t seed,
                     const int64_t* keys, float* out) {
  // same random stream as the GPU kernel (splitmix-style finaliser of
  // seed*golden + slot)
  auto mix32 = [](uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return static_cast<uint32_t>(x);
  };
  auto reflect = [](int p, int n) {
    if (p < 0) p = -p;
    if (p >= n) p = 2 * n - 2 - p;
    return p;
  };
  at::parallel_for(0, B, 1, [&](int64_t b0, int64_t b1) {
    for (int64_t b = b0; b < b1; ++b) {
      const uint64_t key = keys ? static_cast<uint64_t>(keys[b]) : static_cast<uint64_t>(b);
      uint32_t rnd = mix32(seed * 0x9E3779B97F4A7C15ull + key);
      int dy = 0, dx = 0;
      if (pad > 0) {
        dy = static_cast<int>(rnd % (2 * pad + 1));
        dx = static_cast<int>((rnd >> 8) % (2 * pad + 1));
      }
      bool fl = flip && ((rnd >> 16) & 1u);
      for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
          int xx = fl ? (W - 1 - x) : x;
          int sy = reflect(y + dy - pad, H), sx = reflect(xx + dx - pad, W);
          const uint8_t* src = data + ((idx[b] * H + sy) * W + sx) * C;
          float* dst = out + ((b * H + y) * W + x) * C;
          for (int ch = 0; ch < C; ++ch)
            dst[ch] = (src[ch] * (1.f / 255.f) - mean[ch]) * inv_std[ch];
        }
    }
  });
}

}  // namespace cpu
}  // namespace commeff
