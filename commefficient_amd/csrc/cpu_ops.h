#pragma once
#include <cstdint>
#include <cstring>
#include "sketch_hash.h"

namespace commeff {
namespace cpu {
void cs_encode(float* table, const float* vec, const float* wvec, float scale, float wscale,
               const RowHashes& h, const SketchGeom& g, const int32_t* blk_off,
               const float* blk_sign);
void cs_query(const float* table, float* est, const RowHashes& h, const SketchGeom& g,
              const int32_t* blk_off, const float* blk_sign);
void cs_zero_buckets(float* t1, float* t2, const int64_t* idx, const float* vals, int64_t k,
                     const RowHashes& h, const SketchGeom& g, const int32_t* blk_off,
                     const float* blk_sign);
float cs_l2estimate(const float* table, int r, int64_t c);
void topk_abs(const float* x, int64_t n, int64_t k, int64_t* idx, float* vals);
void momentum_ef(float* V, float* E, const float* G, int64_t n, float rho, float gscale,
                 int mode);
void sparse_apply(float* w, const int64_t* idx, const float* vals, int64_t k, float lr,
                  const float* lr_vec, int32_t* last_mod, int32_t round, int32_t* hist);
void dense_apply(float* w, const float* delta, int64_t n, float lr, const float* lr_vec,
                 int32_t* last_mod, int32_t round, int32_t* hist);
void account_hist(const int32_t* hist, int nbins, const int64_t* meta, int W, double* client_dl,
                  double* client_ul, double upc, double* dl);
void count_ge(const int32_t* last_mod, int64_t n, const int32_t* thr, int T, int64_t* out);
void axpby(float* out, const float* a, float alpha, const float* b, float beta, int64_t n);
float l2norm(const float* x, int64_t n);
void clip_noise(float* x, int64_t n, const float* norm, float clip, float noise_std,
                uint64_t seed, uint64_t offset);
void client_state(const float* g, float* u, float* e, int64_t n, float rho);
void augment_u8_nhwc(const uint8_t* data, const int64_t* idx, int64_t B, int H, int W, int C,
                     int pad, int flip, const float* mean, const float* inv_std, uint64_t seed,
                     const int64_t* keys, float* out);
}  // namespace cpu
}  // namespace commeff
