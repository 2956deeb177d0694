// Launcher declarations for the gfx950 HIP kernels of the codec engine.
// The kernels (*.hip) are compiled by hipcc without any torch headers; the
// torch-op bindings (bindings.cpp) call these launchers with raw device
// pointers and the current HIP stream.
#pragma once
#include <hip/hip_runtime_api.h>
#include <cstdint>
#include "sketch_hash.h"
#include "launch.h"

namespace commeff {

// ---------------------------------------------------------------- sketch --
// table[j, b_j(i)] += s_j(i) * (scale*vec[i] + wscale*wvec[i])   (wvec optional)
void launch_cs_encode(float* table, const float* vec, const float* wvec,
                      float scale, float wscale, const RowHashes& h,
                      const SketchGeom& g, const int32_t* blk_off,
                      const float* blk_sign, hipStream_t stream);
// Binned (LDS-privatised) encode for dense vectors, see sketch.hip.  The
// per-(chunk, tile) layout depends only on the hashes: build it once with
// launch_cs_layout (counts), then base = exclusive scan over chunks + segment
// start, seg = tile segment starts [num_tiles + 1].
struct BinPlan {
  int64_t tile;        // buckets per LDS tile (flat over rows)
  int64_t num_tiles;
  int64_t chunk;       // coordinates per pass-1 block
  int64_t num_chunks;
  int64_t cap;         // total entries = d * r
};
BinPlan plan_cs_encode_binned(const SketchGeom& g);
int64_t cs_encode_binned_scratch_bytes(const BinPlan& p);
bool cs_binned_supported(const BinPlan& p);
void launch_cs_layout(const RowHashes& h, const SketchGeom& g, const int32_t* blk_off,
                      const float* blk_sign, const BinPlan& p, uint32_t* counts,
                      hipStream_t stream);
void launch_cs_encode_binned(float* table, const float* vec, const float* wvec,
                             float scale, float wscale, const RowHashes& h,
                             const SketchGeom& g, const int32_t* blk_off,
                             const float* blk_sign, const BinPlan& plan,
                             const uint32_t* counts, const uint32_t* base,
                             const uint32_t* seg, void* entries, hipStream_t stream);
// Planned (precomputed-permutation, atomic-free) encode / query, see
// sketch_planned.hip and ops/sketch_plan.py.
constexpr int64_t kPlanSegCap = 32767;    // max entries of one tile segment (LDS, 15-bit ids)
constexpr int64_t kPlanStageCap = 65535;  // max entries of one coordinate chunk (16-bit slots)
struct PlanGeom {
  int64_t tile;        // buckets per tile (power of 2, 512..4096; 8192 when dense)
  int64_t num_tiles;   // ceil(r*c / tile)
  int64_t chunk;       // coordinates per chunk
  int64_t num_chunks;
  bool dense = false;  // many entries per bucket (GPT-2): encode P2 accumulates
                       // with LDS atomics, plan slot 2 holds chunk-major
                       // in-tile bucket | sign instead of the bucket-order perm
  int64_t p2_splits = 1;  // dense: blocks per tile of encode P2 (chunk-range shares)
};
// false when the geometry does not fit (too many entries per bucket)
bool planned_geometry(int64_t d, int64_t r, int64_t c, PlanGeom* out);
// the dense variant (any entries per bucket; false only for d*r >= 2^31)
bool planned_geometry_dense(int64_t d, int64_t r, int64_t c, PlanGeom* out);
struct PlannedArgs {
  const uint16_t* src_info;  // [d*r]  slot of (i,j) in its chunk's stage
  const uint16_t* ent_info;  // [d*r]  entry order: in-tile bucket | sign << 15
  const uint16_t* perm;      // [d*r]  bucket order: segment-local entry | sign << 15
  const int32_t* csr;        // [num_tiles*tile + 1] bucket starts in perm
  const int32_t* base;       // [num_chunks, num_tiles] global run starts
  const int32_t* off;        // [num_chunks, num_tiles + 1] in-chunk run starts
  const int32_t* seg;        // [num_tiles + 1] tile segment starts
  float* vals;               // [d*r] scratch
  const int32_t* p2_src;     // [num_tiles, num_chunks] run start in chunk-major vals
  const int32_t* p2_pos;     // [num_tiles, num_chunks + 1] run start in the segment
  // dense plans, fixed-point encode P2 (plan slot 10; nullptr: fp32 LDS atomics)
  int64_t* fx = nullptr;     // [p2_splits, num_tiles*tile] per-split tile partials (int64)
  float* bmax = nullptr;     // [num_chunks] max |v| of each P1 chunk
  float* gmax = nullptr;     // [1] max |v| of the vector
};
void launch_cs_hash_all(const RowHashes& h, const SketchGeom& g, const int32_t* blk_off,
                        const float* blk_sign, int32_t* out, hipStream_t stream);
// overwrite: table = S(v) (every bucket written, no prior zeroing) instead of +=
void launch_cs_encode_planned(float* table, const float* vec, const float* wvec, float scale,
                              float wscale, int64_t d, int r, int64_t c, const PlanGeom& p,
                              const PlannedArgs& a, bool overwrite, hipStream_t stream);
// est[i] for the coordinates of plan chunks [c0, c1) only (c1 < 0: all)
void launch_cs_query_planned(const float* table, float* est, int64_t d, int r, int64_t c,
                             const PlanGeom& p, const PlannedArgs& a, hipStream_t stream,
                             int64_t c0 = 0, int64_t c1 = -1);
// est[i] = lower-median_j( s_j(i) * table[j, b_j(i)] )
void launch_cs_query(const float* table, float* est, const RowHashes& h,
                     const SketchGeom& g, const int32_t* blk_off,
                     const float* blk_sign, hipStream_t stream);
// the same estimate in r gather passes (one table row each, L2-resident) into
// vals [r, d] and a median pass
void launch_cs_query_rows(const float* table, float* vals, float* est, const RowHashes& h,
                          const SketchGeom& g, const int32_t* blk_off, const float* blk_sign,
                          hipStream_t stream);
// For every selected coordinate idx[t] with vals[t] != 0 zero the r cells
// (j, b_j(idx[t])) of t1 and (optionally) t2.
void launch_cs_zero_buckets(float* t1, float* t2, const int64_t* idx,
                            const float* vals, int64_t k, const RowHashes& h,
                            const SketchGeom& g, const int32_t* blk_off,
                            const float* blk_sign, hipStream_t stream);
// Region sketch (sketch_region.hip, ops/sketch_region.py): perm [r, m] u32 =
// P_j(o) | S_j(o) << 31; cinfo [r, nch] u32 = region | shift << 24 | sigma << 31;
// lists [nch] chunks grouped (group-major, batches of W), goffs [G + 1].
bool region_geometry_supported(int64_t r, int64_t m, int64_t g, int64_t W);
// Table layout of a region sketch: cell (group grp, row j, bucket t of the
// group) at (grp - g0) * gs + j * rs + t for grp in [g0, g1).  Row-major
// [r][c]: {g*m, c, 0, G}; group-major [G'][r][g*m] (sharded server): {r*g*m,
// g*m, g0, g1} with the tensor starting at group g0.
struct RegionLayout {
  uint32_t gs, rs, g0, g1;
};
// c: buckets per row (row-major: the unused tail past G*g*m is zeroed on overwrite)
void launch_cs_region_encode(float* table, const float* vec, const float* wvec, float scale,
                             float wscale, int64_t d, int r, int64_t c, int64_t m, int64_t g, int64_t G,
                             int64_t W, int64_t nch, const uint32_t* perm, const uint32_t* cinfo,
                             const int32_t* lists, const int32_t* goffs, bool overwrite, RegionLayout L,
                             hipStream_t stream, float* zero_vec = nullptr);  // zero_vec: vec, cleared
// est[i] for the coordinates of chunks [q0, q1) whose group is in [L.g0, L.g1)
// (one block per such group; the others are left unset); hist0 != nullptr:
// also the top-k's first histogram of est (see topk_prepare)
// mom_mode 1 / 2: the server momentum on the table first (1: V = rho V +
// gscale G, table = E += V; 2: table = V = rho V + gscale G), see
// sketch_region.hip RegionMom (V, G in the table's layout)
void launch_cs_region_query(float* table, float* est, int64_t d, int r, int64_t m, int64_t g,
                            int64_t W, int64_t nch, const uint32_t* perm, const uint32_t* cinfo,
                            const int32_t* lists, const int32_t* goffs, int64_t q0, int64_t q1,
                            RegionLayout L, hipStream_t stream, const uint32_t* hint = nullptr,
                            uint32_t* hist0 = nullptr, float* momV = nullptr, const float* momG = nullptr,
                            float rho = 0.f, float gscale = 0.f, int mom_mode = 0,
                            uint64_t* ballots = nullptr, uint32_t* segtot = nullptr,
                            const int32_t* cpos = nullptr);  // cpos: est / ballots at compact chunk slots
// zero the cells of idx (vals != 0) whose group is in [L.g0, L.g1)
void launch_cs_region_zero(float* t1, float* t2, const int64_t* idx, const float* vals, int64_t k,
                           int64_t d, int r, int64_t g, int64_t m, int64_t nch, const uint32_t* perm,
                           const uint32_t* cinfo, RegionLayout L, hipStream_t stream);
// sharded-server k-list helpers (shard.hip)
bool merge_packed_supported(int nl);
// cmap (optional): idx are compact shard positions, global = cmap[idx / m] * m + idx % m
void launch_topk_pack(const int64_t* idx, const float* vals, int64_t k, const int32_t* cmap, int64_t m,
                      int64_t* out, hipStream_t stream);
void launch_merge_packed(const int64_t* allp, int nl, int64_t k, float* vals, int64_t* idx, hipStream_t stream);
void launch_gather_i64(const int64_t* src, const int64_t* pos, int64_t n, int64_t* out, hipStream_t stream);
// dst (device) = n bytes read by a kernel from pinned host memory (its device mapping)
void launch_host_read_copy(const void* host_src, void* dst, int64_t n, hipStream_t stream);
// one-block kernel launched with ``lds_bytes`` of dynamic LDS (writes 64 to
// out[0]): exercises the launch status check (launch.h)
void launch_probe(int32_t* out, uint32_t lds_bytes, hipStream_t stream);
// out[0] = sqrt(lower-median_j sum_c table[j,c]^2); partial: >= r*256 floats
void launch_cs_l2estimate(const float* table, int r, int64_t c, float* partial,
                          float* out, hipStream_t stream);

// ------------------------------------------------------------------ topk --
struct TopkWorkspace {
  // all device pointers; sizes given by topk_workspace_bytes
  void* base;
};
int64_t topk_workspace_bytes(int64_t n);
// Deterministic magnitude top-k: selects the k largest |x| (ties -> lower
// index), writes idx (ascending) and vals = x[idx].  No host sync.
void launch_topk_abs(const float* x, int64_t n, int64_t k, int64_t* idx,
                     float* vals, void* workspace, hipStream_t stream,
                     uint32_t* hint = nullptr);
// the same selection split at the first histogram: topk_prepare zeroes the
// histograms, a producer builds hist[0] (uint32 [2048] at the workspace
// start: keys = bits & 0x7fffffff >= hint[0], bin key >> 20), then the rest
void topk_prepare(void* workspace, hipStream_t stream);
void launch_topk_abs_rest(const float* x, int64_t n, int64_t k, int64_t* idx, float* vals,
                          void* workspace, hipStream_t stream, uint32_t* hint);
// candidate-list variant (csrc/topk.hip cand_compact_kernel): the producer of
// hist[0] also writes the per-64-element-chunk masks of keys >= hint and the
// per-segment popcounts (topk_cand_ptrs); topk_cand_prepare zeroes the
// histograms and segment totals.  Same result as launch_topk_abs_rest.
bool topk_cand_supported(int64_t n);
int64_t topk_cand_workspace_bytes(int64_t n);
void topk_cand_prepare(void* workspace, hipStream_t stream);
void topk_cand_ptrs(void* workspace, int64_t n, uint64_t** ballots, uint32_t** seg);
// persistent: the workspace is reused across calls (zeroed once by the
// caller): the last pass re-zeroes the histograms / segment totals, so no
// topk_cand_prepare is needed before the next call
void launch_topk_cand_rest(const float* x, int64_t n, int64_t k, int64_t* idx, float* vals, void* workspace,
                           hipStream_t stream, uint32_t* hint, bool persistent = false);

// ----------------------------------------------------------- elementwise --
// V = rho*V + gscale*G ; mode 1: E += V ; mode 2: E = V
void launch_momentum_ef(float* V, float* E, const float* G, int64_t n,
                        float rho, float gscale, int mode, hipStream_t stream);
// w[idx] -= lr(idx) * vals ; last_mod[idx] = round where w changed
void launch_sparse_apply(float* w, const int64_t* idx, const float* vals,
                         int64_t k, float lr, const float* lr_vec,
                         int32_t* last_mod, int32_t round, const int32_t* step,
                         int32_t* hist, hipStream_t stream);
// the same plus the region sketch's heavy-hitter zeroing of the list (cells of
// coordinates with nonzero vals in t1 and t2; cs_region_zero semantics)
void launch_sparse_apply_region_zero(float* w, const int64_t* idx, const float* vals, int64_t k, float lr,
                                     const float* lr_vec, int32_t* last_mod, int32_t round, const int32_t* step,
                                     int32_t* hist, float* t1, float* t2, const uint32_t* perm,
                                     const uint32_t* cinfo, int r, int64_t g, int64_t m, int64_t nch, int64_t d,
                                     RegionLayout L, hipStream_t stream);
// w -= lr(i) * delta ; last_mod[i] = round where w changed
// (step != nullptr: lr = bits of step[0], round = step[1], read on the device
// so a captured HIP graph replays with the current round's values)
// hist (optional): change histogram, hist[r+1] = #{i : last_mod[i] == r},
// maintained incrementally as stamps move
void launch_dense_apply(float* w, const float* delta, int64_t n, float lr,
                        const float* lr_vec, int32_t* last_mod, int32_t round,
                        const int32_t* step, int32_t* hist, hipStream_t stream);
// per-client download bytes from the change histogram (meta = int64
// [last_seen (W) | clients (W)])
void launch_account_hist(const int32_t* hist, int nbins, const int64_t* meta, int W,
                         double* client_dl, double* client_ul, double upc, double* dl,
                         hipStream_t stream);
// counts[t] = #{i : last_mod[i] >= thr[t]}  (thr sorted ascending, T <= 1024)
void launch_count_ge(const int32_t* last_mod, int64_t n, const int32_t* thr,
                     int T, int64_t* counts, hipStream_t stream);
// one round of byte accounting: meta = [thr (T, ascending) | inv (W) | clients (W)]
// (int64); dl[j] = 4 * #{i : last_mod[i] >= thr[inv[j]]}; client_dl[clients[j]] +=
// dl[j]; client_ul[clients[j]] += upc.  partial: account_round_blocks(n) * (T+1) u32.
int account_round_blocks(int64_t n);
void launch_account_round(const int32_t* last_mod, int64_t n, const int64_t* meta, int T, int W,
                          uint32_t* partial, double* client_dl, double* client_ul, double upc,
                          double* dl, hipStream_t stream);
// out = alpha*a + beta*b   (b optional -> out = alpha*a)
void launch_axpby(float* out, const float* a, float alpha, const float* b,
                  float beta, int64_t n, hipStream_t stream);
// partial sums of squares -> out[0] = sqrt(sum) ; partial >= 1024 floats
void launch_l2norm(const float* x, int64_t n, float* partial, float* out,
                   hipStream_t stream);
// x = x * min(1, clip/norm[0]) (clip <= 0: no clipping) + std * N(0,1)
// (Philox-4x32-10 keyed by seed, counter = offset + i)
void launch_clip_noise(float* x, int64_t n, const float* norm, float clip,
                       float noise_std, uint64_t seed, uint64_t offset,
                       hipStream_t stream);
// u = rho*u + g (if u) ; e += (u ? u : g) (if e)
// fused client transmit tail: t = scale (g + wd w); u = rho u + t (t = u); e += t;
// g = t when u and e are both null.  n % 4 == 0, 16-byte aligned.
void launch_client_tail(float* g, const float* w, float wd, float scale, float* u, float* e, float rho,
                        int64_t n, hipStream_t stream);
void launch_client_state(const float* g, float* u, float* e, int64_t n,
                         float rho, hipStream_t stream);
// x[idx[t]] = 0 for t < k  (up to 3 arrays)
void launch_zero_at(float* a, float* b, float* c, const int64_t* idx,
                    int64_t k, hipStream_t stream);
// out[:] = 0 ; out[idx] = vals
void launch_scatter_dense(float* out, int64_t n, const int64_t* idx,
                          const float* vals, int64_t k, hipStream_t stream);

// ----------------------------------------------------------------- conv --
// 3x3 / stride 1 / pad 1 NHWC bf16 convolution on MFMA (conv.hip).
struct ConvFwdArgs {
  const uint16_t* x;       // [P, C]  (P = N*H*W pixels, NHWC)
  const uint16_t* w;       // [K, 3, 3, C]
  uint16_t* y;             // [P, K]
  const uint16_t* mask;    // optional [P, K]: y = 0 where mask <= 0
  const uint16_t* addend;  // optional [P, K]: y += addend (after relu / mask)
  uint16_t* y_pre;         // optional [P, K]: the value before the addend (with addend only)
  uint8_t* pool_idx;       // pool == 2: y = maxpool2(relu(conv)) [P/4, K], codes [P/4, K]
  int P, H, W, C, K;
  int relu;
  int pool;                // 0, or 2: fused relu + 2x2 max-pool epilogue (128 % (2W) == 0)
  FastDivU32 div_w, div_h;  // set by the launcher
  // optional [P, K] 2x2 max-pool window codes (csrc/pool.hip) of the layer whose
  // pooled output is this conv's OUTPUT grid: y is then the [N, 2H, 2W, K]
  // un-pooled tensor, each value routed to its code's window position (zeros
  // elsewhere) -- the relu + max-pool backward fused into the dgrad epilogue
  const uint8_t* unpool_idx = nullptr;
  // optional [P, K]: also write y_dual = y where dual_mask > 0 else 0 (the
  // relu backward of the layer that produced this conv's input, for the
  // consumer of that layer's other input gradient -- ops/nn.py _MaskLink)
  const uint16_t* dual_mask = nullptr;
  uint16_t* y_dual = nullptr;
  // grouped conv on channel-stacked images (batched FedAvg, ops/nn.py
  // _GConv3x3): x rows hold x_stride channels, output channels come in groups
  // of kg that read only input channels [g C, (g+1) C) (C = a.C, per group) and
  // weight rows g kg .. (g+1) kg of a [G kg][3][3][C] image.  0 = ungrouped.
  int x_stride = 0;
  int kg = 0;
  // grouped weights: 0 = one contiguous [G kg][3][3][C] image; > 0 = group g's
  // kg rows start at w + g * w_gs (per-client bf16 weight rows,
  // parallel/fedavg_native.py); < 0 = every group reads the same kg rows
  int64_t w_gs = 0;
  // grouped input gradient (with w_gs != 0): w holds the CONV's weight rows
  // [C][3][3][kg] per group, read flipped and transposed (conv_fwd_halo_kernel BT)
  int w_bt = 0;
  // split-K across blocks for grids of few tiles (conv3x3_fwd_split_floats > 0):
  // fp32 partial tiles, summed by a combine kernel that runs the epilogue
  float* part = nullptr;
  int ksplit = 0;
};
struct ConvWgradArgs {
  const uint16_t* dy;  // [P, K]
  const uint16_t* x;   // [P, C]
  // grouped (channel-stacked) wgrad: x rows of x_stride channels, dy rows of
  // K (= G kg) channels; output channel k reads input channels [g C, (g+1) C)
  // of its group g = k / kg (C = per-group channels).  0 = ungrouped.
  int x_stride = 0;
  int kg = 0;
  float* slab;         // [splits, K, 9, C] scratch
  int P, H, W, C, K;
  int splits;
  int steps_per_split;  // set by the launcher
  FastDivU32 div_w, div_h;
  // grouped (per-client) weight gradients, ops/grouped.py: the P pixels are
  // G groups of group_px; the splits are G x splits_per_group, each split
  // inside one group (0: ungrouped)
  int group_px = 0;
  int splits_per_group = 0;
  // one split on the halo kernel (launch_conv3x3_wgrad_rows): the epilogue
  // updates the client rows itself -- rows = beta src + alpha dW in (r, s, c)
  // order, + the bf16 mirror -- instead of writing a slab for the reduction
  // (rows_sub: the 64-channel clients' pairs, see conv_wgrad_reduce_kernel)
  float* rows = nullptr;
  int64_t rows_ld = 0;
  int rows_sub = 0;
  float rows_beta = 0.f, rows_alpha = 1.f;
  uint16_t* rows_mirror = nullptr;
  const float* rows_src = nullptr;
  int64_t rows_sld = 0;
};
bool conv3x3_supported(int C, int K);
bool conv3x3_pool_supported(int H, int W, int K);
void launch_conv3x3_fwd(ConvFwdArgs a, hipStream_t stream);
// fp32 workspace (floats) the launch of a needs for its cross-block split-K
// (0: none; the caller sets a.part to that many floats before launching)
int64_t conv3x3_fwd_split_floats(const ConvFwdArgs& a);
int conv3x3_wgrad_splits(int P, int H, int W, int K, int C);
// dw [K][C][3][3] fp32 = beta * dw + sum_p dy x  (beta 0: overwrite)
void launch_conv3x3_wgrad(ConvWgradArgs a, float* dw, float beta, hipStream_t stream);
// grouped (a.kg, a.x_stride set) wgrad into per-group fp32 rows ld apart
// (rsc: rows in (r, s, c) order instead of PyTorch's (c, r, s))
// (sub > 0: every kernel group of kg channels is kg / sub clients -- the
// diagonal sub x sub blocks are written, each to its client's row)
// (beta / alpha: dst = beta dst + alpha dW -- an SGD step in place -- and the
// bf16 mirror of the result at the same offsets from `mirror`; wsrc: beta
// scales wsrc's rows (sld apart, 0: one shared row) instead of dst's)
void launch_conv3x3_wgrad_rows(ConvWgradArgs a, float* dst, int kg, int64_t ld, bool rsc, hipStream_t stream,
                               int sub = 0, float beta = 0.f, float alpha = 1.f, uint16_t* mirror = nullptr,
                               const float* wsrc = nullptr, int64_t sld = 0);
// grouped convs on channel-stacked images (a.kg / a.x_stride set): false when
// the geometry has no halo tiling (the caller falls back)
bool launch_conv3x3_fwd_grouped(ConvFwdArgs a, hipStream_t stream);
bool conv3x3_wgrad_grouped_supported(int H, int W, int K, int C, int kg);
// per-group dw_g [K][C][3][3] (+)= the wgrad of group g's pixels, dw_g at
// dw + g * gstride floats (a.splits = G x splits_per_group, set by the caller)
void launch_conv3x3_wgrad_grouped(ConvWgradArgs a, int G, float* dw, int64_t gstride, float beta,
                                  hipStream_t stream);
// w [K][C][3][3] fp32 -> wf [K][3][3][C] bf16 (either output optional) and
// wt [C][3][3][K] bf16 spatially flipped (the dgrad weight), for up to
// kPrepMax weights in one launch
constexpr int kPrepMax = 16;
struct ConvPrepItem {
  const float* w;
  uint16_t* wf;  // bf16
  uint16_t* wt;
  int K, C;
  int block0;  // set by the launcher
};
struct ConvPrepBatch {
  ConvPrepItem t[kPrepMax];
  int n;
};
void launch_conv_weight_prep(ConvPrepBatch b, hipStream_t stream);
// re-convert the coordinates idx of the flat fp32 weight vector w_flat into
// the bf16 GEMM images of the conv weights laid out at off[j] (the images of
// conv_weight_prep): a sparse server update touches only these
struct ConvPatchBatch {
  const float* w_flat;
  int64_t off[kPrepMax];
  int64_t numel[kPrepMax];
  uint16_t* wf[kPrepMax];
  uint16_t* wt[kPrepMax];
  int K[kPrepMax], C[kPrepMax];
  int n;
};
void launch_conv_images_patch(const ConvPatchBatch& b, const int64_t* idx, int64_t k,
                              hipStream_t stream);
// g = gy where y > 0 else 0 (bf16, n % 8 == 0)
void launch_relu_mask(const uint16_t* gy, const uint16_t* y, uint16_t* g, int64_t n,
                      hipStream_t stream);

// ResNet-9 input conv (conv_prep.hip): 3x3 pad 1, Cin <= 4 -> 64 channels,
// ReLU.  x: bf16 pixels with a 4-channel stride; y: [P, 64] bf16; mask: two
// 32-bit ReLU-mask words per pixel.
struct ConvPrepArgs {
  const uint16_t* x;        // [P, 4]
  const float* w;           // [64, Cin, 3, 3]
  uint16_t* y;              // [P, 64]
  uint32_t* mask;           // [P, 2] (forward output)
  const uint16_t* gy;       // [P, 64] (backward)
  const uint32_t* mask_in;  // [P, 2] (backward)
  float* partial;           // [conv_prep_wgrad_blocks(P), 64, 64] scratch (backward)
  int P, H, W, Cin;
  FastDivU32 div_w, div_h;  // set by the launchers
};
int conv_prep_wgrad_blocks(int P);
void launch_conv_prep_fwd(ConvPrepArgs a, hipStream_t stream);
// dw [64][Cin][3][3] fp32 = beta * dw + sum_p (gy * mask) x
void launch_conv_prep_wgrad(ConvPrepArgs a, float* dw, float beta, hipStream_t stream);

// ----------------------------------------------------------------- loss --
// per-example cross-entropy of logits [B, C] (bf16 or f32): loss, top-1
// correctness and the unit gradient softmax - onehot (logits dtype)
// ResNet-9 head (head.hip): maxpool(HxW) -> scale * linear (no bias) -> CE
bool head_supported(int C, int NCLS);
void launch_head_fwd(const uint16_t* x, const float* w, const int64_t* tgt, int B, int C, int NPIX, int NCLS,
                     float scale, float* loss, float* correct, float* gunit, uint16_t* pooled, uint8_t* codes,
                     hipStream_t stream);
void launch_head_bwd(const float* gl, const float* gunit, const float* w, const uint16_t* pooled,
                     const uint8_t* codes, int B, int C, int NPIX, int NCLS, float scale, uint16_t* dx,
                     float* dw, float beta, hipStream_t stream, const uint16_t* ymask = nullptr,
                     uint16_t* dxm = nullptr);
// ghost batch norm (bn.hip): x NHWC bf16, G groups of M pixels, C % 8 == 0,
// C <= 2048; part = bn_scratch_floats(G, M, C) floats, stat = ab = 2GC, coef = 3GC
int bn_slabs(int G, int M);
int64_t bn_scratch_floats(int G, int M, int C);
// relu: y = max(BN(x), 0); its backward passes y_relu (the saved output)
void launch_bn_fwd(const uint16_t* x, const float* w, const float* b, int G, int M, int C, float eps,
                   float momentum, float* run_mean, float* run_var, float* part, float* stat, float* ab,
                   bool relu, int64_t* nbt, uint16_t* y, hipStream_t stream,
                   const uint16_t* addend = nullptr, uint8_t* relu_bits = nullptr,
                   const float* tile_stats = nullptr);
// rows per tile of the GEMM-epilogue batch-norm moments (GemmArgs::stats)
constexpr int kBnStatTile = 128;
// y_relu: the forward's 1-bit ReLU mask (one byte per 8 channels of a pixel)
// channel-stacked clients (C = G * cg channels, one pixel group of M rows):
// per-channel statistics, affine parameters from per-client fp32 rows
// (prm[(c / cg) * ld + off + c % cg]), fused ReLU (bits), weight / bias
// gradients into the per-client gradient rows (grad[(c / cg) * gld + off + c % cg])
int64_t bn_cs_scratch_floats(int M, int C);
void launch_bn_cs_fwd(const uint16_t* x, const float* prm, int64_t ld, int64_t woff, int64_t boff, int cg,
                      int M, int C, float eps, float momentum, float* run_mean, float* run_var,
                      int64_t* nbt, float* part, float* stat, float* ab, uint16_t* y, uint8_t* relu_bits,
                      const uint16_t* post_add, hipStream_t stream);
void launch_bn_cs_bwd(const uint16_t* x, const uint16_t* dy, const uint8_t* y_relu, const float* stat,
                      const float* prm, int64_t ld, int64_t woff, int cg, int M, int C, float* part,
                      float* coef, float* grad, int64_t gld, int64_t gwoff, int64_t gboff, uint16_t* dx,
                      hipStream_t stream, float beta = 0.f, float alpha = 1.f, const float* wsrc = nullptr,
                      int64_t sld = 0);
void launch_bn_bwd(const uint16_t* x, const uint16_t* dy, const uint8_t* y_relu, const float* stat,
                   const float* w, int G, int M, int C, float* part, float* coef, float* dw, float* db,
                   float beta, uint16_t* dx, hipStream_t stream, float* gdw = nullptr,
                   float* gdb = nullptr, int64_t gstride = 0, uint16_t* dadd = nullptr);

constexpr int kClientMeanRows = 4;
struct ClientMeanRows {
  const float* p[kClientMeanRows];
  int m;
};
void launch_client_means(const ClientMeanRows& rows, const int64_t* slot, int n, const void* counts,
                         bool counts_f32, int W, float* out, hipStream_t stream);
void launch_scale_rows(void* g, bool bf16, const float* s, int64_t B, int C, int64_t ldg, hipStream_t stream);
void launch_ce_fwd(const void* x, bool bf16, const int64_t* tgt, int64_t B, int C, int64_t ldx, float* loss,
                   float* correct, void* grad, hipStream_t stream);

// ----------------------------------------------------------------- pool --
// y = maxpool_k(relu(x)) on NHWC bf16 (C % 8 == 0, H, W % k == 0), k in {2, 4};
// idx = window position of the max (255: max <= 0, gradient 0)
void launch_relu_maxpool_fwd(const uint16_t* x, uint16_t* y, uint8_t* idx, int N, int H,
                             int W, int C, int k, hipStream_t stream);
void launch_relu_maxpool_bwd(const uint16_t* gy, const uint8_t* idx, uint16_t* gx, int N,
                             int H, int W, int C, int k, hipStream_t stream);

// --------------------------------------------------------------- im2col --
// explicit-GEMM convolutions (csrc/im2col.hip): col [N*OH*OW][Kc] bf16,
// column (r*S + s)*C + c, zero outside the image and for columns >= R*S*C
struct Im2colArgs {
  const uint16_t* x;  // NHWC bf16, channel stride 1, strides sN / sH / sW
  uint16_t* col;
  int N, H, W, C, OH, OW, R, S, stride, pad, Kc;
  int64_t sN, sH, sW;
  bool vec;  // C % 8 == 0 and 16-byte aligned pixels: 16-byte moves
  // grouped column images (batched FedAvg, parallel/fedavg_native.py): G
  // groups of C channels, group g's input at x + g * sG, col [P][G][Kc]; the
  // col2im gather then writes gx [N][H][W][G*C].  0 / 0 = one group.
  int G;
  int64_t sG;
};
void launch_im2col(const Im2colArgs& a, hipStream_t stream);
// gx NHWC [N][H][W][C] (C % 8 == 0) = the dgrad gather of gcol [N*OH*OW][Kc]
void launch_col2im(const Im2colArgs& a, const uint16_t* gcol, uint16_t* gx, hipStream_t stream);
// w fp32 [K][C][R*S] -> bf16 [K][Kc] in the column order above
void launch_weight_rsc(const float* w, uint16_t* out, int K, int C, int RS, int Kc,
                       hipStream_t stream);
// dst[g][k][c][t] (+)= sum over the `splits` partial products src[g*splits+u][k][t*C+c]
void launch_wgrad_rsc_add(float* dst, int64_t dst_ld, const float* src, int G, int splits,
                          int K, int C, int RS, int Kc, bool accumulate, hipStream_t stream);
// k x k / stride s / padding p max-pool on NHWC bf16 (C % 8 == 0), 1-byte codes
void launch_maxpool_fwd(const uint16_t* x, uint16_t* y, uint8_t* codes, int N, int H, int W,
                        int C, int k, int s, int p, hipStream_t stream);
void launch_maxpool_bwd(const uint16_t* gy, const uint8_t* codes, uint16_t* gx, int N, int H,
                        int W, int C, int k, int s, int p, hipStream_t stream);

// -------------------------------------------------------------- augment --
// CIFAR-style augmentation of uint8 NHWC images into a bf16 NHWC
// (channels_last) batch: reflect-pad `pad`, random crop, random h-flip,
// normalise.  Randomness: counter hash of (seed, keys[b] or b).  Pixels are
// written out_cstride (>= C) channels apart, the extra channels zeroed.
void launch_augment_u8_nhwc(const uint8_t* data, const int64_t* idx,
                            int64_t B, int H, int W, int C, int pad,
                            int flip, const float* mean, const float* inv_std,
                            uint64_t seed, const int64_t* keys, uint16_t* out_bf16,
                            int out_cstride, hipStream_t stream,
                            const int64_t* targets = nullptr, int64_t* yout = nullptr);

// ---------------------------------------------------------- transformer --
// GPT-2 block junctions on bf16 [M, H] rows (transformer.hip, ops/transformer.py).
// h = x + drop(p + bias) (p null: h = drop(x)); y = LN(h)*gamma + beta
bool resid_ln_supported(int64_t H);  // H = 256*V, V in 1..6
void launch_resid_ln_fwd(const void* x, const void* p, const void* bias, const void* gamma,
                         const void* beta, void* h_out, void* y_out, float* mean, float* rstd,
                         int64_t M, int64_t H, float p_drop, uint32_t seed, float eps,
                         hipStream_t stream);
// dh = LN'(gy) + gh; dp = drop'(dh); part [blocks][3][H] = column partials of
// (gy*xhat, gy, dp)
int resid_ln_bwd_blocks(int64_t M);
void launch_resid_ln_bwd(const void* gy, const void* gh, const void* h, const float* mean,
                         const float* rstd, const void* gamma, void* dh_out, void* dp_out,
                         float* part, int64_t M, int64_t H, float p_drop, uint32_t seed,
                         hipStream_t stream);
// f = gelu_tanh(u + b), N % 8 == 0
void launch_bias_gelu_fwd(const void* u, const void* b, void* f, int64_t M, int64_t N,
                          hipStream_t stream);
// du = gf * gelu_tanh'(u + b) (gelu) or gf; part [blocks][N] = column partials of du
int bias_act_bwd_blocks(int64_t M);
void launch_bias_act_bwd(const void* gf, const void* u, const void* b, void* du, float* part,
                         int64_t M, int64_t N, bool gelu, hipStream_t stream);
struct ColsumOut {
  void* p[3];   // [N] outputs per partial quantity (nullptr: skip)
  int mode[3];  // 0: store bf16, 1: store fp32, 2: fp32 += (a flat fp32 gradient view)
};
// token rows [Mr, P*H] <-> padded per-head tensors [N, nh, L, hd] (bf16, hd % 8 == 0)
struct HeadSrcs {
  const void* p[3];
  int64_t stride[3][3];  // element strides of (n, h, t) per source, multiples of 8; d contiguous
};
// out[pos] = src[inv[pos]] (row of K bf16) or 0 where inv[pos] < 0 (inv null: identity)
void launch_pad_rows(const void* src, int64_t src_ld, int64_t K, const int32_t* inv, int64_t rows,
                     void* out, hipStream_t stream);
void launch_heads_to_rows(const HeadSrcs& src, int P, int64_t H, int64_t hd, int64_t L,
                          const int32_t* tok, int64_t Mr, void* out, hipStream_t stream);
// fused causal attention over unpadded token rows (attention.hip): sequence n
// = rows [start[n], start[n] + len[n]), len <= lse_ld <= 1024, head dim 64;
// lse_ld == 128: the all-in-LDS short kernels, else (a multiple of 128) the
// flash-style long kernels
struct AttnArgs {
  const uint16_t* qkv;  // [M, 3H] bf16 (q | k | v)
  uint16_t* o;          // [M, H] bf16 (forward output, backward input)
  float* lse;           // [N * nh * lse_ld] fp32
  float* dbuf;          // [N * nh * lse_ld] fp32 (long backward: dO . O per row)
  int lse_ld;
  const uint16_t* dout; // [M, H] bf16 (backward)
  uint16_t* dqkv;       // [M, 3H] bf16 (backward)
  const int32_t* start;
  const int32_t* len;
  int nh;
  float scale;
  uint32_t thresh;  // set by the launchers from p_drop
  float dscale;
  uint32_t seed;
};
void launch_attn_fwd(AttnArgs a, int64_t nseq, float p_drop, hipStream_t stream);
void launch_attn_bwd(AttnArgs a, int64_t nseq, float p_drop, hipStream_t stream);
// C[M][N] (fp32, row stride ldc) += A^T B, A [T][lda] and B [T][ldb] bf16
// (gemm_tn.hip; M, N multiples of 256, lda / ldb multiples of 8); split-K
// over T with fp32 slabs [splits][M][N] summed into C in a fixed order
// C[M][N] = act(A[M][K] . op(B) + bias) (+ beta C); NT: B [N][K], NN: B [K][N]
// (gemm.hip).  bf16 operands / output (f32: fp32 output), act 1: tanh-GELU with
// the pre-activation written to C2.  N % 64 == 0, K % 64 == 0.
struct GemmArgs {
  const uint16_t* A;
  int64_t lda;
  const uint16_t* B;
  int64_t ldb;
  void* C;
  int64_t ldc;
  void* C2;
  const float* bias;
  const uint16_t* bias16 = nullptr;  // bf16 bias (instead of the fp32 one)
  int M, N, K;
  float beta;
  // batch-norm statistics of the (bf16-rounded) output, per 128-row tile and
  // group slot: stats[tile][slot][mean | M2][N], rows split at multiples of
  // stats_mg (>= 128: a tile spans at most two groups; slot 0 = the group of
  // the tile's first row).  bf16 output without activation only.
  float* stats = nullptr;
  int stats_mg = 0;
  // G independent products (the batched FedAvg clients' channel-stacked
  // operands): group g reads A + g sa, B + g sb and writes C + g sc
  int G = 1;
  int64_t sa = 0, sb = 0, sc = 0;
  // imp_C > 0 (NT only): A is the IMPLICIT column image of the channels-last x
  // (a.A; pixel rows lda apart, group offset sa) of imp_H x imp_W images, an
  // imp_R x imp_R conv with stride imp_s / pad imp_pad onto imp_OH x imp_OW:
  // column k = tap * imp_C + c (imp_C % 64 == 0: a K-step stays in one tap)
  int imp_C = 0, imp_H = 0, imp_W = 0, imp_OH = 0, imp_OW = 0, imp_R = 3, imp_s = 1, imp_pad = 1;
};
// batched FedAvg per-client classifier + cross-entropy + SGD (fedavg.hip)
constexpr int kFaMaxN = 32;             // examples per client
constexpr int kFaMaxLds = 96 * 1024;    // n F (and n C) fp32
constexpr int kFaCls = 16;              // classes per logits block
struct FaLinearArgs {
  const void* feat;       // (client g, example i, feature f) at g * fsg + i * fsn + f
  int64_t fsg, fsn;
  const float* W;         // weight rows: client g's [C][F] at g * wld + woff, bias at + boff (< 0: none)
  int64_t wld, woff, boff;
  const int64_t* y;       // [G n] targets in [0, C)
  int n, C, F;
  float scale;
  float* loss;            // [G n]
  float* correct;         // [G n]
  void* dfeat;            // like feat: g * dsg + i * dsn + f (+ s * dss: the slab of class chunk s)
  int64_t dsg, dsn, dss;
  int ccs;                // classes per chunk (<= 0: all; > 0: ceil(C / ccs) partial dfeat slabs)
  float* dst;             // updated rows: g * dld + woff / boff
  int64_t dld;
  float beta, alpha;
  const float* src;       // beta's rows (nullptr: dst's own), g * sld
  int64_t sld;
  uint16_t* mirror;       // bf16 copy of the updated rows (nullptr: none), g * mld
  int64_t mld;
};
int64_t fa_linear_lds_bytes(int n, int C, int F);
void launch_fa_linear_ce(FaLinearArgs a, int G, bool feat_bf16, bool dfeat_bf16, float* logits, hipStream_t stream);
// batched FedAvg per-client scalar affine maps of the Fixup models (fedavg.hip)
struct FaAffine {
  const uint16_t* x;      // bf16 activations
  const uint16_t* add;    // + residual (nullptr: none)
  uint16_t* y;
  const float* S;         // scale of group g at S[g * ld] (nullptr: none)
  const float* B;         // bias of group g at B[g * ld] (nullptr: none)
  const float* P;         // post bias after the relu, P[g * ld] (nullptr: none)
  int64_t ld;
  int64_t per;            // elements per client
  int64_t GC;             // channel-stacked: G C channels a pixel (0 with C = 0: client-major)
  int G, C, relu;
};
struct FaAffineBwd {
  const uint16_t* dy;
  const uint16_t* yrelu;  // the forward output (relu mask), nullptr: no relu
  const uint16_t* xs;     // the scale's input (its gradient sum dpre x), nullptr: sum dy (unmasked) instead
  int mask_x;             // relu mask recomputed from xs (x s + b > 0, no add), second sum = dy unmasked
  const uint16_t* add2;   // + this to out1 (nullptr: none)
  uint16_t* out1;         // dpre * s (+ add2), nullptr: not written
  uint16_t* out2;         // dpre, nullptr: not written
  float* part;            // [chunks][G][2] sums of dpre, dpre x
  int64_t chunk;          // elements per block
};
void launch_fa_affine(const FaAffine& a, hipStream_t stream);
void launch_fa_affine_bwd(const FaAffine& a, const FaAffineBwd& b, int chunks, hipStream_t stream);
void launch_fx_part_sum(const float* part, int chunks, float* out, hipStream_t stream);
void launch_fa_scalar_sgd(const float* part, int chunks, int G, float* dst, int64_t ld, int64_t boff, int64_t soff,
                          float beta, float alpha, const float* src, int64_t sld, hipStream_t stream);
bool gemm_supported(int M, int N, int K, bool nn);
bool gemm_supported_nedge(int M, int N, int K);
void launch_gemm(const GemmArgs& a, bool nn, int act, bool f32, hipStream_t stream);
void launch_splitk_tail(const float* part, int S, int M, int N, const uint16_t* A, int64_t lda, const uint16_t* B,
                        int64_t ldb, int k0, int k1, uint16_t* out, int64_t ldo, hipStream_t stream);
struct GemmTnArgs {
  const uint16_t* A;
  int64_t lda;
  const uint16_t* B;
  int64_t ldb;
  float* C;
  int64_t ldc;
  float* slab;
  int M, N, T;  // T: rows of each group
  int splits;
  int steps_per_split;  // set by the launcher
  int G = 1;            // groups: A / B rows [g T, (g + 1) T) -> C + g cg
  int64_t cg = 0;
  int slab_only = 0;    // write every split's product to the slabs, no reduction into C
  int64_t sa = -1, sb = -1;       // group strides of A / B in elements (< 0: T lda / T ldb)
  float beta = 1.f, alpha = 1.f;  // C = beta C + alpha A^T B
  uint16_t* mirror = nullptr;     // + bf16(C) at the same [m][n] (ldc), group stride mcg
  int64_t mcg = 0;
  int small = -1;                 // tile: -1 by shape, 0: 256 x 256, 1: 128 x 128
  // imp_C > 0: B is the IMPLICIT 3x3 / stride-1 / pad-1 column image of the
  // channel-stacked x (a.B; pixel rows ldb apart, group g at + g sb) of
  // imp_H x imp_W images: column j = tap * imp_C + c reads pixel p shifted by
  // the tap (zero outside the image) -- no column image in memory
  int imp_C = 0, imp_H = 0, imp_W = 0;
  // (output grid / conv geometry of the implicit image; 0: same as the input,
  // 3x3, stride 1, pad 1)
  int imp_OH = 0, imp_OW = 0, imp_R = 3, imp_s = 1, imp_pad = 1;
  const float* src = nullptr;     // beta scales src (group stride scg, 0: shared) instead of C
  int64_t scg = 0;
  int nt = 0;                     // (staged epilogue) nontemporal stores
  int stage = 0;                  // 128 x 128, one split: C updated through LDS, 16 bytes a lane
                                  // (ldc, cg, mcg multiples of 4; C, mirror 16 / 8-byte aligned)
};
int gemm_tn_splits(int M, int N, int T, int cus, int small = -1);
void launch_gemm_tn_acc(GemmTnArgs a, hipStream_t stream);
// out_q[c] = sum over b < G of part[b*stride + q*N + c], q < Q (fixed order)
void launch_colsum_final(const float* part, int G, int Q, int64_t N, int64_t stride,
                         const ColsumOut& out, hipStream_t stream);

}  // namespace commeff
