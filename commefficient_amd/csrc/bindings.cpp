// torch.ops.commeff.* registrations: one schema per op, a CPU kernel (native
// C++, cpu_ops.cpp) and a CUDA-dispatch-key kernel (HIP launchers for gfx950).
// On ROCm builds of PyTorch HIP tensors dispatch under the CUDA key and report
// DeviceType::CUDA, so the device guard / current stream come from the
// "MasqueradingAsCUDA" HIP classes.
#include <ATen/ATen.h>
#include <ATen/Parallel.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <torch/library.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "cpu_ops.h"
#include "kernels.h"

namespace commeff {
namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

void check_f32(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.scalar_type() == at::kFloat, name, " must be float32");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

const int64_t* key_ptr(const c10::optional<at::Tensor>& k, int64_t n) {
  if (!k.has_value() || !k->defined()) return nullptr;
  TORCH_CHECK(k->scalar_type() == at::kLong && k->is_contiguous() && k->numel() == n,
              "keys must be contiguous int64 [B]");
  return k->data_ptr<int64_t>();
}

float* fptr(const c10::optional<at::Tensor>& t) {
  return t.has_value() && t->defined() ? t->data_ptr<float>() : nullptr;
}

struct HashCtx {
  RowHashes rows;
  SketchGeom geom;
  const int32_t* blk_off = nullptr;
  const float* blk_sign = nullptr;
};

HashCtx make_ctx(const at::Tensor& hashes, const at::Tensor& blk_off, const at::Tensor& blk_sign,
                 int64_t num_blocks, int64_t d, int64_t c, bool on_device) {
  TORCH_CHECK(hashes.device().is_cpu() && hashes.scalar_type() == at::kLong &&
                  hashes.dim() == 2 && hashes.size(1) == kHashParams,
              "hashes must be a CPU int64 tensor [r, 4]");
  const int64_t r = hashes.size(0);
  TORCH_CHECK(r >= 1 && r <= kMaxRows, "num_rows must be in [1, 16]");
  TORCH_CHECK(d >= 0 && d < (1ll << 31), "sketched vector length must be < 2^31");
  TORCH_CHECK(c >= 1 && r * c < (1ll << 32), "r*c must be < 2^32");
  HashCtx ctx;
  auto hc = hashes.contiguous();
  const int64_t* hp = hc.data_ptr<int64_t>();
  for (int64_t j = 0; j < r; ++j) {
    RowHash& rh = ctx.rows.row[j];
    rh.a = static_cast<uint64_t>(hp[j * kHashParams + 0]) | 1ull;
    rh.b = static_cast<uint64_t>(hp[j * kHashParams + 1]);
    rh.a2 = static_cast<uint64_t>(hp[j * kHashParams + 2]) | 1ull;
    rh.b2 = static_cast<uint64_t>(hp[j * kHashParams + 3]);
  }
  ctx.geom = make_geom(static_cast<uint32_t>(d), static_cast<uint32_t>(r),
                       static_cast<uint32_t>(c), static_cast<uint32_t>(num_blocks));
  if (ctx.geom.num_blocks > 1) {
    TORCH_CHECK(blk_off.numel() == r * ctx.geom.num_blocks && blk_sign.numel() == r * ctx.geom.num_blocks,
                "blk_off/blk_sign must be [r, num_blocks]");
    TORCH_CHECK(blk_off.scalar_type() == at::kInt && blk_sign.scalar_type() == at::kFloat,
                "blk_off int32, blk_sign float32");
    TORCH_CHECK(blk_off.is_cuda() == on_device && blk_sign.is_cuda() == on_device,
                "blk_off/blk_sign must live on the op's device");
    ctx.blk_off = blk_off.data_ptr<int32_t>();
    ctx.blk_sign = blk_sign.data_ptr<float>();
  }
  return ctx;
}

// ============================================================ CPU kernels

void cs_encode_cpu(at::Tensor table, const at::Tensor& vec, const at::Tensor& hashes,
                   const at::Tensor& blk_off, const at::Tensor& blk_sign, int64_t num_blocks,
                   double scale, const c10::optional<at::Tensor>& wvec, double wscale,
                   at::TensorList layout) {
  (void)layout;  // the CPU encode is row-parallel and needs no binning
  check_f32(table, "table");
  check_f32(vec, "vec");
  auto ctx = make_ctx(hashes, blk_off, blk_sign, num_blocks, vec.numel(), table.size(-1), false);
  TORCH_CHECK(table.numel() == static_cast<int64_t>(ctx.geom.r) * ctx.geom.c, "table shape");
  cpu::cs_encode(table.data_ptr<float>(), vec.data_ptr<float>(), fptr(wvec),
                 static_cast<float>(scale), static_cast<float>(wscale), ctx.rows, ctx.geom,
                 ctx.blk_off, ctx.blk_sign);
}

at::Tensor cs_query_cpu(const at::Tensor& table, const at::Tensor& hashes,
                        const at::Tensor& blk_off, const at::Tensor& blk_sign,
                        int64_t num_blocks, int64_t d) {
  check_f32(table, "table");
  auto ctx = make_ctx(hashes, blk_off, blk_sign, num_blocks, d, table.size(-1), false);
  auto est = at::empty({d}, table.options());
  cpu::cs_query(table.data_ptr<float>(), est.data_ptr<float>(), ctx.rows, ctx.geom, ctx.blk_off,
                ctx.blk_sign);
  return est;
}

void cs_zero_buckets_cpu(at::Tensor t1, const c10::optional<at::Tensor>& t2,
                         const at::Tensor& idx, const c10::optional<at::Tensor>& vals,
                         const at::Tensor& hashes, const at::Tensor& blk_off,
                         const at::Tensor& blk_sign, int64_t num_blocks, int64_t d) {
  check_f32(t1, "t1");
  auto ctx = make_ctx(hashes, blk_off, blk_sign, num_blocks, d, t1.size(-1), false);
  cpu::cs_zero_buckets(t1.data_ptr<float>(), fptr(t2), idx.data_ptr<int64_t>(), fptr(vals),
                       idx.numel(), ctx.rows, ctx.geom, ctx.blk_off, ctx.blk_sign);
}

at::Tensor cs_l2estimate_cpu(const at::Tensor& table) {
  check_f32(table, "table");
  auto out = at::empty({}, table.options());
  out.fill_(cpu::cs_l2estimate(table.data_ptr<float>(), static_cast<int>(table.size(0)),
                               table.size(1)));
  return out;
}

std::tuple<at::Tensor, at::Tensor> topk_abs_cpu(const at::Tensor& x, int64_t k,
                                                const c10::optional<at::Tensor>& /*hint: GPU only*/) {
  check_f32(x, "x");
  const int64_t n = x.numel();
  const int64_t kk = std::max<int64_t>(0, std::min(k, n));
  auto idx = at::empty({kk}, x.options().dtype(at::kLong));
  auto vals = at::empty({kk}, x.options());
  cpu::topk_abs(x.data_ptr<float>(), n, kk, idx.data_ptr<int64_t>(), vals.data_ptr<float>());
  return {idx, vals};
}

void momentum_ef_cpu(at::Tensor V, const c10::optional<at::Tensor>& E, const at::Tensor& G,
                     double rho, double gscale, int64_t mode) {
  check_f32(V, "V");
  check_f32(G, "G");
  TORCH_CHECK(mode == 0 || (E.has_value() && E->numel() == V.numel()), "E required for mode>0");
  cpu::momentum_ef(V.data_ptr<float>(), fptr(E), G.data_ptr<float>(), V.numel(),
                   static_cast<float>(rho), static_cast<float>(gscale), static_cast<int>(mode));
}

// step: optional int32 [2] = (bits of lr, round) overriding lr / round
static void read_step(const c10::optional<at::Tensor>& step, double& lr, int64_t& round) {
  if (!step.has_value() || !step->defined()) return;
  auto s = step->to(at::kCPU).contiguous();
  TORCH_CHECK(s.scalar_type() == at::kInt && s.numel() == 2, "step must be int32 [2]");
  const int32_t* p = s.data_ptr<int32_t>();
  float f;
  std::memcpy(&f, p, sizeof(float));
  lr = f;
  round = p[1];
}

static const int32_t* step_ptr(const c10::optional<at::Tensor>& step) {
  if (!step.has_value() || !step->defined()) return nullptr;
  TORCH_CHECK(step->scalar_type() == at::kInt && step->numel() == 2 && step->is_contiguous(),
              "step must be a contiguous int32 [2]");
  return step->data_ptr<int32_t>();
}

static int32_t* hist_ptr(const c10::optional<at::Tensor>& hist) {
  if (!hist.has_value() || !hist->defined()) return nullptr;
  TORCH_CHECK(hist->scalar_type() == at::kInt && hist->is_contiguous(), "hist must be contiguous int32");
  return hist->data_ptr<int32_t>();
}

void sparse_apply_cpu(at::Tensor w, const at::Tensor& idx, const at::Tensor& vals, double lr,
                      const c10::optional<at::Tensor>& lr_vec,
                      const c10::optional<at::Tensor>& last_mod, int64_t round,
                      const c10::optional<at::Tensor>& step,
                      const c10::optional<at::Tensor>& hist) {
  read_step(step, lr, round);
  check_f32(w, "w");
  int32_t* lm = last_mod.has_value() && last_mod->defined() ? last_mod->data_ptr<int32_t>() : nullptr;
  cpu::sparse_apply(w.data_ptr<float>(), idx.data_ptr<int64_t>(), vals.data_ptr<float>(),
                    idx.numel(), static_cast<float>(lr), fptr(lr_vec), lm,
                    static_cast<int32_t>(round), hist_ptr(hist));
}

void dense_apply_cpu(at::Tensor w, const at::Tensor& delta, double lr,
                     const c10::optional<at::Tensor>& lr_vec,
                     const c10::optional<at::Tensor>& last_mod, int64_t round,
                     const c10::optional<at::Tensor>& step,
                     const c10::optional<at::Tensor>& hist) {
  read_step(step, lr, round);
  check_f32(w, "w");
  check_f32(delta, "delta");
  int32_t* lm = last_mod.has_value() && last_mod->defined() ? last_mod->data_ptr<int32_t>() : nullptr;
  cpu::dense_apply(w.data_ptr<float>(), delta.data_ptr<float>(), w.numel(),
                   static_cast<float>(lr), fptr(lr_vec), lm, static_cast<int32_t>(round),
                   hist_ptr(hist));
}

at::Tensor count_ge_cpu(const at::Tensor& last_mod, const at::Tensor& thr) {
  auto thr_c = thr.to(at::kInt).contiguous();
  const int T = static_cast<int>(thr_c.numel());
  auto out = at::zeros({T}, last_mod.options().dtype(at::kLong));
  if (T > 0)
    cpu::count_ge(last_mod.data_ptr<int32_t>(), last_mod.numel(), thr_c.data_ptr<int32_t>(), T,
                  out.data_ptr<int64_t>());
  return out;
}

void axpby_cpu(at::Tensor out, const at::Tensor& a, double alpha,
               const c10::optional<at::Tensor>& b, double beta) {
  check_f32(out, "out");
  check_f32(a, "a");
  cpu::axpby(out.data_ptr<float>(), a.data_ptr<float>(), static_cast<float>(alpha), fptr(b),
             static_cast<float>(beta), out.numel());
}

at::Tensor l2norm_cpu(const at::Tensor& x) {
  check_f32(x, "x");
  auto out = at::empty({}, x.options());
  out.fill_(cpu::l2norm(x.data_ptr<float>(), x.numel()));
  return out;
}

void clip_noise_cpu(at::Tensor x, const c10::optional<at::Tensor>& norm, double clip,
                    double noise_std, int64_t seed, int64_t offset) {
  check_f32(x, "x");
  cpu::clip_noise(x.data_ptr<float>(), x.numel(), fptr(norm), static_cast<float>(clip),
                  static_cast<float>(noise_std), static_cast<uint64_t>(seed),
                  static_cast<uint64_t>(offset));
}

void client_state_cpu(const at::Tensor& g, const c10::optional<at::Tensor>& u,
                      const c10::optional<at::Tensor>& e, double rho) {
  check_f32(g, "g");
  cpu::client_state(g.data_ptr<float>(), fptr(u), fptr(e), g.numel(), static_cast<float>(rho));
}

void client_tail_check(const at::Tensor& g, const c10::optional<at::Tensor>& w,
                       const c10::optional<at::Tensor>& u, const c10::optional<at::Tensor>& e) {
  check_f32(g, "g");
  for (const auto* t : {&w, &u, &e})
    if (t->has_value() && (*t)->defined())
      TORCH_CHECK((*t)->scalar_type() == at::kFloat && (*t)->is_contiguous() && (*t)->numel() == g.numel() &&
                      (*t)->device() == g.device(),
                  "client_tail: contiguous fp32 operands of g's size and device");
}

void client_tail_cpu(at::Tensor g, const c10::optional<at::Tensor>& w, double wd, double scale,
                     const c10::optional<at::Tensor>& u, const c10::optional<at::Tensor>& e, double rho) {
  client_tail_check(g, w, u, e);
  float* gp = g.data_ptr<float>();
  const float* wp = fptr(w);
  float *up = fptr(u), *ep = fptr(e);
  const float fwd = static_cast<float>(wd), fs = static_cast<float>(scale), fr = static_cast<float>(rho);
  for (int64_t i = 0; i < g.numel(); ++i) {
    float t = gp[i];
    if (wp) t += fwd * wp[i];
    t *= fs;
    if (up) {
      t = fr * up[i] + t;
      up[i] = t;
    }
    if (ep) ep[i] += t;
    if (!up && !ep) gp[i] = t;
  }
}

void zero_at_cpu(const c10::optional<at::Tensor>& a, const c10::optional<at::Tensor>& b,
                 const c10::optional<at::Tensor>& c, const at::Tensor& idx) {
  const int64_t* ip = idx.data_ptr<int64_t>();
  for (float* p : {fptr(a), fptr(b), fptr(c)})
    if (p)
      for (int64_t q = 0; q < idx.numel(); ++q) p[ip[q]] = 0.f;
}

at::Tensor scatter_dense_cpu(const at::Tensor& idx, const at::Tensor& vals, int64_t n) {
  auto out = at::zeros({n}, vals.options());
  float* o = out.data_ptr<float>();
  const int64_t* ip = idx.data_ptr<int64_t>();
  const float* vp = vals.data_ptr<float>();
  for (int64_t q = 0; q < idx.numel(); ++q) o[ip[q]] = vp[q];
  return out;
}

at::Tensor augment_cpu(const at::Tensor& data, const at::Tensor& idx, int64_t pad, bool flip,
                       const at::Tensor& mean, const at::Tensor& inv_std, int64_t seed,
                       bool out_bf16, const c10::optional<at::Tensor>& keys) {
  TORCH_CHECK(data.scalar_type() == at::kByte && data.dim() == 4 && data.is_contiguous(),
              "data must be uint8 [N,H,W,C] contiguous");
  const int64_t B = idx.numel(), H = data.size(1), W = data.size(2), C = data.size(3);
  auto out = at::empty({B, H, W, C}, data.options().dtype(at::kFloat));
  auto mc = mean.to(at::kFloat).contiguous(), sc = inv_std.to(at::kFloat).contiguous();
  cpu::augment_u8_nhwc(data.data_ptr<uint8_t>(), idx.contiguous().data_ptr<int64_t>(), B,
                       static_cast<int>(H), static_cast<int>(W), static_cast<int>(C),
                       static_cast<int>(pad), flip ? 1 : 0, mc.data_ptr<float>(),
                       sc.data_ptr<float>(), static_cast<uint64_t>(seed), key_ptr(keys, B),
                       out.data_ptr<float>());
  auto o = out.permute({0, 3, 1, 2});  // logical NCHW, physical NHWC
  return out_bf16 ? o.to(at::kBFloat16) : o;
}

// ============================================================ HIP kernels

void cs_encode_hip(at::Tensor table, const at::Tensor& vec, const at::Tensor& hashes,
                   const at::Tensor& blk_off, const at::Tensor& blk_sign, int64_t num_blocks,
                   double scale, const c10::optional<at::Tensor>& wvec, double wscale,
                   at::TensorList layout) {
  check_f32(table, "table");
  check_f32(vec, "vec");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(table.device());
  auto ctx = make_ctx(hashes, blk_off, blk_sign, num_blocks, vec.numel(), table.size(-1), true);
  TORCH_CHECK(table.numel() == static_cast<int64_t>(ctx.geom.r) * ctx.geom.c, "table shape");
  if (wvec.has_value() && wvec->defined()) check_f32(*wvec, "wvec");
  if (!layout.empty()) {
    // layout = [counts, base, seg, entries] from cs_layout for this geometry
    TORCH_CHECK(layout.size() == 4, "layout must be [counts, base, seg, entries]");
    BinPlan plan = plan_cs_encode_binned(ctx.geom);
    TORCH_CHECK(layout[0].numel() == plan.num_chunks * plan.num_tiles &&
                    layout[1].numel() == plan.num_chunks * plan.num_tiles &&
                    layout[2].numel() == plan.num_tiles + 1,
                "layout does not match this sketch geometry");
    TORCH_CHECK(layout[3].nbytes() >= static_cast<size_t>(cs_encode_binned_scratch_bytes(plan)),
                "entry buffer too small for binned encode");
    launch_cs_encode_binned(table.data_ptr<float>(), vec.data_ptr<float>(), fptr(wvec),
                            static_cast<float>(scale), static_cast<float>(wscale), ctx.rows,
                            ctx.geom, ctx.blk_off, ctx.blk_sign, plan,
                            reinterpret_cast<const uint32_t*>(layout[0].data_ptr<int32_t>()),
                            reinterpret_cast<const uint32_t*>(layout[1].data_ptr<int32_t>()),
                            reinterpret_cast<const uint32_t*>(layout[2].data_ptr<int32_t>()),
                            layout[3].data_ptr(), cur_stream());
  } else {
    launch_cs_encode(table.data_ptr<float>(), vec.data_ptr<float>(), fptr(wvec),
                     static_cast<float>(scale), static_cast<float>(wscale), ctx.rows, ctx.geom,
                     ctx.blk_off, ctx.blk_sign, cur_stream());
  }
}

at::Tensor cs_query_hip(const at::Tensor& table, const at::Tensor& hashes,
                        const at::Tensor& blk_off, const at::Tensor& blk_sign,
                        int64_t num_blocks, int64_t d) {
  check_f32(table, "table");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(table.device());
  auto ctx = make_ctx(hashes, blk_off, blk_sign, num_blocks, d, table.size(-1), true);
  auto est = at::empty({d}, table.options());
  launch_cs_query(table.data_ptr<float>(), est.data_ptr<float>(), ctx.rows, ctx.geom, ctx.blk_off,
                  ctx.blk_sign, cur_stream());
  return est;
}

// two-pass row-wise query (large d without a plan): r x d fp32 scratch
at::Tensor cs_query_rows_hip(const at::Tensor& table, const at::Tensor& hashes,
                             const at::Tensor& blk_off, const at::Tensor& blk_sign,
                             int64_t num_blocks, int64_t d) {
  check_f32(table, "table");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(table.device());
  auto ctx = make_ctx(hashes, blk_off, blk_sign, num_blocks, d, table.size(-1), true);
  auto est = at::empty({d}, table.options());
  auto vals = at::empty({static_cast<int64_t>(ctx.geom.r) * d}, table.options());
  launch_cs_query_rows(table.data_ptr<float>(), vals.data_ptr<float>(), est.data_ptr<float>(), ctx.rows,
                       ctx.geom, ctx.blk_off, ctx.blk_sign, cur_stream());
  return est;
}

void cs_zero_buckets_hip(at::Tensor t1, const c10::optional<at::Tensor>& t2,
                         const at::Tensor& idx, const c10::optional<at::Tensor>& vals,
                         const at::Tensor& hashes, const at::Tensor& blk_off,
                         const at::Tensor& blk_sign, int64_t num_blocks, int64_t d) {
  check_f32(t1, "t1");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(t1.device());
  auto ctx = make_ctx(hashes, blk_off, blk_sign, num_blocks, d, t1.size(-1), true);
  launch_cs_zero_buckets(t1.data_ptr<float>(), fptr(t2), idx.data_ptr<int64_t>(), fptr(vals),
                         idx.numel(), ctx.rows, ctx.geom, ctx.blk_off, ctx.blk_sign,
                         cur_stream());
}

// ---- region sketch (sketch_region.hip)
struct RegionParams {
  int64_t r, c, m, g, G, W, nch;
  RegionLayout L;
};

// The table's shape gives its layout (kernels.h RegionLayout):
//   [r, c]          row-major, every group (g0 must be 0);
//   [Gs, r, g*m]    group-major, groups [g0, g0 + Gs) (the sharded server's
//                   per-rank state, or the padded payload with g0 = 0).
RegionParams check_region(const at::Tensor& table, int64_t d, int64_t m, int64_t g, int64_t W,
                          const at::Tensor& perm, const at::Tensor& cinfo, const at::Tensor* lists,
                          const at::Tensor* goffs, int64_t g0 = 0) {
  check_f32(table, "table");
  RegionParams p;
  p.m = m;
  p.g = g;
  p.W = W;
  p.nch = (d + m - 1) / m;
  const int64_t gm = g * m;
  if (table.dim() == 3) {
    TORCH_CHECK(table.size(2) == gm && g0 >= 0, "region sketch: group-major table must be [groups, r, g*m]");
    p.r = table.size(1);
    p.c = 0;
    p.G = goffs != nullptr ? goffs->numel() - 1 : g0 + table.size(0);
    const int64_t g1 = std::min(p.G, g0 + table.size(0));
    p.L = RegionLayout{static_cast<uint32_t>(p.r * gm), static_cast<uint32_t>(gm), static_cast<uint32_t>(g0),
                       static_cast<uint32_t>(std::max(g0, g1))};
  } else {
    TORCH_CHECK(g0 == 0, "region sketch: a row-major table holds every group (g0 = 0)");
    p.c = table.size(-1);
    p.r = table.numel() / p.c;
    p.G = p.c / gm;
    p.L = RegionLayout{static_cast<uint32_t>(gm), static_cast<uint32_t>(p.c), 0u, static_cast<uint32_t>(p.G)};
  }
  TORCH_CHECK(region_geometry_supported(p.r, m, g, W) && p.G >= 1 && d >= 1 && d < (int64_t(1) << 32) &&
                  p.G * g < (int64_t(1) << 24),
              "region sketch: unsupported geometry (r <= 16, m <= 64, W <= min(16, g), r*g*m floats in LDS)");
  auto i32 = [&](const at::Tensor& t, int64_t n, const char* what) {
    TORCH_CHECK(t.scalar_type() == at::kInt && t.is_contiguous() && t.numel() == n && t.device() == table.device(),
                "region sketch: ", what, " must be int32 with ", n, " elements on the table's device");
  };
  i32(perm, p.r * m, "perm [r, m]");
  i32(cinfo, p.r * p.nch, "cinfo [r, nch] / [nch, r]");
  if (lists != nullptr) i32(*lists, p.nch, "lists [nch]");
  if (goffs != nullptr && table.dim() != 3) i32(*goffs, p.G + 1, "goffs [G + 1]");
  return p;
}

void cs_region_encode_hip(at::Tensor table, const at::Tensor& vec, double scale,
                          const c10::optional<at::Tensor>& wvec, double wscale, int64_t m, int64_t g, int64_t W,
                          const at::Tensor& perm, const at::Tensor& cinfo, const at::Tensor& lists,
                          const at::Tensor& goffs, bool overwrite, bool zero_vec) {
  check_f32(vec, "vec");
  const int64_t d = vec.numel();
  const RegionParams p = check_region(table, d, m, g, W, perm, cinfo, &lists, &goffs);
  TORCH_CHECK(table.dim() != 3 || table.size(0) >= p.G, "cs_region_encode: a group-major table needs every group");
  if (wvec.has_value() && wvec->defined()) {
    check_f32(*wvec, "wvec");
    TORCH_CHECK(wvec->numel() == d && wvec->device() == vec.device(), "wvec must match vec");
  }
  TORCH_CHECK(vec.device() == table.device(), "region sketch: vec on another device");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(table.device());
  launch_cs_region_encode(table.data_ptr<float>(), vec.data_ptr<float>(), fptr(wvec),
                          static_cast<float>(scale), static_cast<float>(wscale), d, static_cast<int>(p.r), p.c,
                          m, g, p.G, W, p.nch, reinterpret_cast<const uint32_t*>(perm.data_ptr<int32_t>()),
                          reinterpret_cast<const uint32_t*>(cinfo.data_ptr<int32_t>()), lists.data_ptr<int32_t>(),
                          goffs.data_ptr<int32_t>(), overwrite, p.L, cur_stream(),
                          zero_vec ? const_cast<float*>(vec.data_ptr<float>()) : nullptr);
}

// est [d]; with q0 < q1 only the coordinates of chunks [q0, q1) are computed
// (a rank's shard of the unsketch; the rest of est is left unset)
at::Tensor cs_region_query_hip(const at::Tensor& table, int64_t d, int64_t m, int64_t g, int64_t W,
                               const at::Tensor& perm, const at::Tensor& cinfo, const at::Tensor& lists,
                               const at::Tensor& goffs, int64_t q0, int64_t q1, int64_t g0) {
  const RegionParams p = check_region(table, d, m, g, W, perm, cinfo, &lists, &goffs, g0);
  if (q1 < 0) q1 = p.nch;
  TORCH_CHECK(q0 >= 0 && q0 <= q1 && q1 <= p.nch, "cs_region_query: chunk range out of bounds");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(table.device());
  auto est = at::empty({d}, table.options());
  launch_cs_region_query(const_cast<float*>(table.data_ptr<float>()), est.data_ptr<float>(), d, static_cast<int>(p.r),
                         m, g, W, p.nch, reinterpret_cast<const uint32_t*>(perm.data_ptr<int32_t>()),
                         reinterpret_cast<const uint32_t*>(cinfo.data_ptr<int32_t>()), lists.data_ptr<int32_t>(),
                         goffs.data_ptr<int32_t>(), q0, q1, p.L, cur_stream());
  return est;
}

// the unsketch of a chunk range in one go: median query fused with the top-k's
// first histogram, then the remaining top-k passes over est[q0*m, q1*m);
// returns (idx relative to q0*m, vals)
// mom_mode 1 / 2 (momV, momG given): the server momentum fused into the
// query's staging of the table (1: table = E, V = rho V + gscale G, E += V;
// 2: table = V = rho V + gscale G)
std::tuple<at::Tensor, at::Tensor> cs_region_topk_hip(at::Tensor table, int64_t d, int64_t m, int64_t g,
                                                      int64_t W, const at::Tensor& perm, const at::Tensor& cinfo,
                                                      const at::Tensor& lists, const at::Tensor& goffs, int64_t k,
                                                      const c10::optional<at::Tensor>& hint, int64_t q0,
                                                      int64_t q1, const c10::optional<at::Tensor>& momV,
                                                      const c10::optional<at::Tensor>& momG, double rho,
                                                      double gscale, int64_t mom_mode,
                                                      const c10::optional<at::Tensor>& ws_keep, int64_t g0,
                                                      const c10::optional<at::Tensor>& cpos, int64_t ncoord) {
  const RegionParams p = check_region(table, d, m, g, W, perm, cinfo, &lists, &goffs, g0);
  const int32_t* cp = nullptr;
  if (cpos.has_value() && cpos->defined()) {
    // a group-major shard's query: est holds the shard's ncoord coordinates
    // at compact positions (chunks ascending), idx are compact positions
    TORCH_CHECK(cpos->scalar_type() == at::kInt && cpos->is_contiguous() && cpos->numel() == p.nch &&
                    cpos->device() == table.device() && ncoord >= 1 && ncoord <= d && q0 == 0,
                "cs_region_topk: cpos must be int32 [nch] with 1 <= ncoord <= d");
    cp = cpos->data_ptr<int32_t>();
  }
  float* mv = nullptr;
  const float* mg = nullptr;
  if (mom_mode != 0) {
    TORCH_CHECK((mom_mode == 1 || mom_mode == 2) && momG.has_value() && momG->defined(),
                "cs_region_topk: mom_mode 1 / 2 needs momG (and momV for 1)");
    TORCH_CHECK(momG->sizes() == table.sizes() && momG->scalar_type() == at::kFloat && momG->is_contiguous() &&
                    momG->device() == table.device(), "cs_region_topk: momG must match the table");
    mg = momG->data_ptr<float>();
    if (mom_mode == 1) {
      TORCH_CHECK(momV.has_value() && momV->defined() && momV->sizes() == table.sizes() &&
                      momV->scalar_type() == at::kFloat && momV->is_contiguous() && momV->device() == table.device(),
                  "cs_region_topk: momV must match the table");
      mv = momV->data_ptr<float>();
    }
  }
  if (q1 < 0) q1 = p.nch;
  TORCH_CHECK(q0 >= 0 && q0 < q1 && q1 <= p.nch, "cs_region_topk: chunk range out of bounds");
  const int64_t lo = cp != nullptr ? 0 : q0 * m, hi = cp != nullptr ? ncoord : std::min(d, q1 * m), n = hi - lo;
  TORCH_CHECK(k >= 1 && k < n, "cs_region_topk: need 1 <= k < shard size");
  uint32_t* hp = nullptr;
  if (hint.has_value() && hint->defined()) {
    TORCH_CHECK(hint->scalar_type() == at::kInt && hint->numel() >= 1 && hint->device() == table.device(),
                "cs_region_topk: hint must be an int32 device tensor");
    hp = reinterpret_cast<uint32_t*>(hint->data_ptr<int32_t>());
  }
  c10::hip::HIPGuardMasqueradingAsCUDA guard(table.device());
  // candidate-list top-k (else the full-vector passes)
  const bool cand = m == 64 && topk_cand_supported(n);
  auto est = at::empty({d}, table.options());
  // a caller-kept workspace (zeroed once, see cs_region_topk_ws_bytes) is
  // left zeroed by the passes: no memset per call
  const bool keep = cand && ws_keep.has_value() && ws_keep->defined();
  if (keep)
    TORCH_CHECK(ws_keep->scalar_type() == at::kByte && ws_keep->is_contiguous() &&
                    ws_keep->device() == table.device() && ws_keep->numel() >= topk_cand_workspace_bytes(n),
                "cs_region_topk: ws must be a contiguous uint8 tensor of cs_region_topk_ws_bytes bytes");
  auto ws = keep ? *ws_keep
                 : at::empty({cand ? topk_cand_workspace_bytes(n) : topk_workspace_bytes(n)},
                             table.options().dtype(at::kByte));
  auto idx = at::empty({k}, table.options().dtype(at::kLong));
  auto vals = at::empty({k}, table.options());
  uint64_t* ballots = nullptr;
  uint32_t* seg = nullptr;
  if (cand) {
    if (!keep) topk_cand_prepare(ws.data_ptr(), cur_stream());
    topk_cand_ptrs(ws.data_ptr(), n, &ballots, &seg);
  } else {
    topk_prepare(ws.data_ptr(), cur_stream());
  }
  launch_cs_region_query(table.data_ptr<float>(), est.data_ptr<float>(), d, static_cast<int>(p.r), m, g,
                         W, p.nch, reinterpret_cast<const uint32_t*>(perm.data_ptr<int32_t>()),
                         reinterpret_cast<const uint32_t*>(cinfo.data_ptr<int32_t>()), lists.data_ptr<int32_t>(),
                         goffs.data_ptr<int32_t>(), q0, q1, p.L, cur_stream(), hp,
                         reinterpret_cast<uint32_t*>(ws.data_ptr()), mv, mg, static_cast<float>(rho),
                         static_cast<float>(gscale), static_cast<int>(mom_mode), ballots, seg, cp);
  if (cand) {
    launch_topk_cand_rest(est.data_ptr<float>() + lo, n, k, idx.data_ptr<int64_t>(), vals.data_ptr<float>(),
                          ws.data_ptr(), cur_stream(), hp, keep);
  }
  else
    launch_topk_abs_rest(est.data_ptr<float>() + lo, n, k, idx.data_ptr<int64_t>(), vals.data_ptr<float>(),
                         ws.data_ptr(), cur_stream(), hp);
  return {idx, vals};
}

// bytes of a kept cs_region_topk workspace for the chunk range [q0, q1)
// (0: the call sizes its own -- candidate lists unsupported or disabled)
int64_t cs_region_topk_ws_bytes(int64_t d, int64_t m, int64_t q0, int64_t q1) {
  const int64_t lo = q0 * m, hi = std::min(d, q1 * m), n = hi - lo;
  if (m != 64 || !topk_cand_supported(n)) return 0;
  return topk_cand_workspace_bytes(n);
}

void cs_region_zero_hip(at::Tensor t1, const c10::optional<at::Tensor>& t2, const at::Tensor& idx,
                        const c10::optional<at::Tensor>& vals, int64_t d, int64_t m, int64_t g,
                        const at::Tensor& perm, const at::Tensor& cinfo, int64_t g0) {
  const RegionParams p = check_region(t1, d, m, g, 1, perm, cinfo, nullptr, nullptr, g0);
  TORCH_CHECK(idx.scalar_type() == at::kLong && idx.is_contiguous() && idx.device() == t1.device(),
              "cs_region_zero: idx must be int64 on the table's device");
  if (t2.has_value() && t2->defined())
    TORCH_CHECK(t2->sizes() == t1.sizes() && t2->scalar_type() == at::kFloat && t2->is_contiguous(),
                "cs_region_zero: t2 must match t1");
  if (vals.has_value() && vals->defined())
    TORCH_CHECK(vals->numel() == idx.numel() && vals->scalar_type() == at::kFloat && vals->is_contiguous(),
                "cs_region_zero: vals must be f32 like idx");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(t1.device());
  launch_cs_region_zero(t1.data_ptr<float>(), fptr(t2), idx.data_ptr<int64_t>(), fptr(vals), idx.numel(), d,
                        static_cast<int>(p.r), g, m, p.nch, reinterpret_cast<const uint32_t*>(perm.data_ptr<int32_t>()),
                        reinterpret_cast<const uint32_t*>(cinfo.data_ptr<int32_t>()), p.L, cur_stream());
}

at::Tensor cs_l2estimate_hip(const at::Tensor& table) {
  check_f32(table, "table");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(table.device());
  const int r = static_cast<int>(table.size(0));
  TORCH_CHECK(r <= kMaxRows, "rows");
  auto partial = at::empty({r * 256}, table.options());
  auto out = at::empty({}, table.options());
  launch_cs_l2estimate(table.data_ptr<float>(), r, table.size(1), partial.data_ptr<float>(),
                       out.data_ptr<float>(), cur_stream());
  return out;
}

// hint: optional int32 [1] device tensor carried between calls of one
// selection site (previous threshold / 2; 0 = no bound) -- see topk.hip
std::tuple<at::Tensor, at::Tensor> topk_abs_hip(const at::Tensor& x, int64_t k,
                                                const c10::optional<at::Tensor>& hint) {
  check_f32(x, "x");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  const int64_t n = x.numel();
  const int64_t kk = std::max<int64_t>(0, std::min(k, n));
  auto idx = at::empty({kk}, x.options().dtype(at::kLong));
  auto vals = at::empty({kk}, x.options());
  if (kk == 0) return {idx, vals};
  if (kk == n) {  // everything selected, in index order
    idx.copy_(at::arange(n, idx.options()));
    vals.copy_(x.reshape({-1}));
    return {idx, vals};
  }
  auto ws = at::empty({topk_workspace_bytes(n)}, x.options().dtype(at::kByte));
  uint32_t* hp = nullptr;
  if (hint.has_value() && hint->defined()) {
    TORCH_CHECK(hint->scalar_type() == at::kInt && hint->numel() >= 1 && hint->device() == x.device(),
                "topk_abs: hint must be an int32 device tensor");
    hp = reinterpret_cast<uint32_t*>(hint->data_ptr<int32_t>());
  }
  launch_topk_abs(x.data_ptr<float>(), n, kk, idx.data_ptr<int64_t>(), vals.data_ptr<float>(),
                  ws.data_ptr(), cur_stream(), hp);
  return {idx, vals};
}

void momentum_ef_hip(at::Tensor V, const c10::optional<at::Tensor>& E, const at::Tensor& G,
                     double rho, double gscale, int64_t mode) {
  check_f32(V, "V");
  check_f32(G, "G");
  TORCH_CHECK(mode == 0 || (E.has_value() && E->numel() == V.numel()), "E required for mode>0");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(V.device());
  launch_momentum_ef(V.data_ptr<float>(), fptr(E), G.data_ptr<float>(), V.numel(),
                     static_cast<float>(rho), static_cast<float>(gscale), static_cast<int>(mode),
                     cur_stream());
}

void sparse_apply_hip(at::Tensor w, const at::Tensor& idx, const at::Tensor& vals, double lr,
                      const c10::optional<at::Tensor>& lr_vec,
                      const c10::optional<at::Tensor>& last_mod, int64_t round,
                      const c10::optional<at::Tensor>& step,
                      const c10::optional<at::Tensor>& hist) {
  check_f32(w, "w");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(w.device());
  int32_t* lm = last_mod.has_value() && last_mod->defined() ? last_mod->data_ptr<int32_t>() : nullptr;
  launch_sparse_apply(w.data_ptr<float>(), idx.data_ptr<int64_t>(), vals.data_ptr<float>(),
                      idx.numel(), static_cast<float>(lr), fptr(lr_vec), lm,
                      static_cast<int32_t>(round), step_ptr(step), hist_ptr(hist), cur_stream());
}

// sparse_apply + cs_region_zero of the same (idx, vals) in one kernel
void cs_region_zero_apply_hip(at::Tensor t1, const c10::optional<at::Tensor>& t2, const at::Tensor& idx,
                              const at::Tensor& vals, int64_t d, int64_t m, int64_t g, const at::Tensor& perm,
                              const at::Tensor& cinfo, at::Tensor w, double lr,
                              const c10::optional<at::Tensor>& lr_vec, const c10::optional<at::Tensor>& last_mod,
                              int64_t round, const c10::optional<at::Tensor>& hist,
                              const c10::optional<at::Tensor>& step, int64_t g0) {
  const RegionParams p = check_region(t1, d, m, g, 1, perm, cinfo, nullptr, nullptr, g0);
  check_f32(w, "w");
  TORCH_CHECK(idx.scalar_type() == at::kLong && idx.is_contiguous() && idx.device() == t1.device(),
              "cs_region_zero_apply: idx must be int64 on the table's device");
  TORCH_CHECK(vals.numel() == idx.numel() && vals.scalar_type() == at::kFloat && vals.is_contiguous(),
              "cs_region_zero_apply: vals must match idx");
  TORCH_CHECK(w.device() == t1.device() && w.numel() == d, "cs_region_zero_apply: w must hold the d weights");
  TORCH_CHECK(p.r >= 1 && p.r <= 8, "cs_region_zero_apply: at most 8 rows (rh::kZeroRows)");
  float* t2p = nullptr;
  if (t2.has_value() && t2->defined()) {
    TORCH_CHECK(t2->sizes() == t1.sizes() && t2->scalar_type() == at::kFloat && t2->is_contiguous(),
                "cs_region_zero_apply: t2 must match t1");
    t2p = t2->data_ptr<float>();
  }
  c10::hip::HIPGuardMasqueradingAsCUDA guard(w.device());
  int32_t* lm = last_mod.has_value() && last_mod->defined() ? last_mod->data_ptr<int32_t>() : nullptr;
  launch_sparse_apply_region_zero(w.data_ptr<float>(), idx.data_ptr<int64_t>(), vals.data_ptr<float>(),
                                  idx.numel(), static_cast<float>(lr), fptr(lr_vec), lm,
                                  static_cast<int32_t>(round), step_ptr(step), hist_ptr(hist), t1.data_ptr<float>(), t2p,
                                  reinterpret_cast<const uint32_t*>(perm.data_ptr<int32_t>()),
                                  reinterpret_cast<const uint32_t*>(cinfo.data_ptr<int32_t>()),
                                  static_cast<int>(p.r), g, m, p.nch, d, p.L, cur_stream());
}

void dense_apply_hip(at::Tensor w, const at::Tensor& delta, double lr,
                     const c10::optional<at::Tensor>& lr_vec,
                     const c10::optional<at::Tensor>& last_mod, int64_t round,
                     const c10::optional<at::Tensor>& step,
                     const c10::optional<at::Tensor>& hist) {
  check_f32(w, "w");
  check_f32(delta, "delta");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(w.device());
  int32_t* lm = last_mod.has_value() && last_mod->defined() ? last_mod->data_ptr<int32_t>() : nullptr;
  launch_dense_apply(w.data_ptr<float>(), delta.data_ptr<float>(), w.numel(),
                     static_cast<float>(lr), fptr(lr_vec), lm, static_cast<int32_t>(round),
                     step_ptr(step), hist_ptr(hist), cur_stream());
}

at::Tensor count_ge_hip(const at::Tensor& last_mod, const at::Tensor& thr) {
  c10::hip::HIPGuardMasqueradingAsCUDA guard(last_mod.device());
  auto thr_c = thr.to(last_mod.device(), at::kInt).contiguous();
  const int T = static_cast<int>(thr_c.numel());
  TORCH_CHECK(T <= 1024, "count_ge supports at most 1024 thresholds per call");
  auto buf = at::zeros({2 * (T + 1)}, last_mod.options().dtype(at::kLong));
  if (T > 0)
    launch_count_ge(last_mod.data_ptr<int32_t>(), last_mod.numel(), thr_c.data_ptr<int32_t>(), T,
                    buf.data_ptr<int64_t>(), cur_stream());
  return buf.narrow(0, T + 1, T);
}

static void check_account_hist(const at::Tensor& hist, const at::Tensor& meta, int64_t W,
                               const at::Tensor& client_dl, const at::Tensor& client_ul) {
  TORCH_CHECK(hist.scalar_type() == at::kInt && hist.is_contiguous() && hist.dim() == 1,
              "account_hist: hist int32 [bins]");
  TORCH_CHECK(meta.scalar_type() == at::kLong && meta.is_contiguous() && meta.numel() == 2 * W &&
                  meta.device() == hist.device(), "account_hist: meta = [last_seen | clients]");
  TORCH_CHECK(client_dl.scalar_type() == at::kDouble && client_ul.scalar_type() == at::kDouble &&
                  client_dl.is_contiguous() && client_ul.is_contiguous(), "account_hist: totals");
}

at::Tensor account_hist_cpu(const at::Tensor& hist, const at::Tensor& meta, int64_t W,
                            at::Tensor client_dl, at::Tensor client_ul, double upc) {
  check_account_hist(hist, meta, W, client_dl, client_ul);
  auto dl = at::empty({W}, hist.options().dtype(at::kDouble));
  cpu::account_hist(hist.data_ptr<int32_t>(), static_cast<int>(hist.numel()), meta.data_ptr<int64_t>(),
                    static_cast<int>(W), client_dl.data_ptr<double>(), client_ul.data_ptr<double>(),
                    upc, dl.data_ptr<double>());
  return dl;
}

at::Tensor account_hist_hip(const at::Tensor& hist, const at::Tensor& meta, int64_t W,
                            at::Tensor client_dl, at::Tensor client_ul, double upc) {
  check_account_hist(hist, meta, W, client_dl, client_ul);
  c10::hip::HIPGuardMasqueradingAsCUDA guard(hist.device());
  auto dl = at::empty({W}, hist.options().dtype(at::kDouble));
  launch_account_hist(hist.data_ptr<int32_t>(), static_cast<int>(hist.numel()), meta.data_ptr<int64_t>(),
                      static_cast<int>(W), client_dl.data_ptr<double>(), client_ul.data_ptr<double>(),
                      upc, dl.data_ptr<double>(), cur_stream());
  return dl;
}

at::Tensor account_round_hip(const at::Tensor& last_mod, const at::Tensor& meta, int64_t T, int64_t W,
                             at::Tensor client_dl, at::Tensor client_ul, double upc) {
  TORCH_CHECK(last_mod.scalar_type() == at::kInt && last_mod.is_contiguous(), "account_round: last_mod");
  TORCH_CHECK(meta.scalar_type() == at::kLong && meta.is_contiguous() && meta.numel() == T + 2 * W &&
                  meta.device() == last_mod.device(), "account_round: meta = [thr | inv | clients]");
  TORCH_CHECK(T >= 0 && T <= 1024 && W >= 0, "account_round: at most 1024 thresholds");
  TORCH_CHECK(client_dl.scalar_type() == at::kDouble && client_ul.scalar_type() == at::kDouble &&
                  client_dl.is_contiguous() && client_ul.is_contiguous(), "account_round: totals");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(last_mod.device());
  auto dl = at::empty({W}, last_mod.options().dtype(at::kDouble));
  if (W == 0) return dl;
  auto partial = at::empty({account_round_blocks(last_mod.numel()) * (T + 1)},
                           last_mod.options().dtype(at::kInt));
  launch_account_round(last_mod.data_ptr<int32_t>(), last_mod.numel(), meta.data_ptr<int64_t>(),
                       static_cast<int>(T), static_cast<int>(W),
                       reinterpret_cast<uint32_t*>(partial.data_ptr()), client_dl.data_ptr<double>(),
                       client_ul.data_ptr<double>(), upc, dl.data_ptr<double>(), cur_stream());
  return dl;
}

void axpby_hip(at::Tensor out, const at::Tensor& a, double alpha,
               const c10::optional<at::Tensor>& b, double beta) {
  check_f32(out, "out");
  check_f32(a, "a");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(out.device());
  launch_axpby(out.data_ptr<float>(), a.data_ptr<float>(), static_cast<float>(alpha), fptr(b),
               static_cast<float>(beta), out.numel(), cur_stream());
}

at::Tensor l2norm_hip(const at::Tensor& x) {
  check_f32(x, "x");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  auto partial = at::empty({1024}, x.options());
  auto out = at::empty({}, x.options());
  launch_l2norm(x.data_ptr<float>(), x.numel(), partial.data_ptr<float>(), out.data_ptr<float>(),
                cur_stream());
  return out;
}

void clip_noise_hip(at::Tensor x, const c10::optional<at::Tensor>& norm, double clip,
                    double noise_std, int64_t seed, int64_t offset) {
  check_f32(x, "x");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  launch_clip_noise(x.data_ptr<float>(), x.numel(), fptr(norm), static_cast<float>(clip),
                    static_cast<float>(noise_std), static_cast<uint64_t>(seed),
                    static_cast<uint64_t>(offset), cur_stream());
}

void client_state_hip(const at::Tensor& g, const c10::optional<at::Tensor>& u,
                      const c10::optional<at::Tensor>& e, double rho) {
  check_f32(g, "g");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(g.device());
  launch_client_state(g.data_ptr<float>(), fptr(u), fptr(e), g.numel(), static_cast<float>(rho),
                      cur_stream());
}

void client_tail_hip(at::Tensor g, const c10::optional<at::Tensor>& w, double wd, double scale,
                     const c10::optional<at::Tensor>& u, const c10::optional<at::Tensor>& e, double rho) {
  client_tail_check(g, w, u, e);
  c10::hip::HIPGuardMasqueradingAsCUDA guard(g.device());
  const int64_t n = g.numel();
  bool vec = n % 4 == 0;
  for (const void* p : {static_cast<const void*>(g.data_ptr<float>()), static_cast<const void*>(fptr(w)),
                        static_cast<const void*>(fptr(u)), static_cast<const void*>(fptr(e))})
    vec = vec && reinterpret_cast<uintptr_t>(p) % 16 == 0;
  if (!vec) {  // (never on the flat buffers) the unfused sequence on device
    if (w.has_value() && w->defined()) g.add_(*w, wd);
    g.mul_(scale);
    launch_client_state(g.data_ptr<float>(), fptr(u), fptr(e), n, static_cast<float>(rho), cur_stream());
    return;
  }
  launch_client_tail(g.data_ptr<float>(), fptr(w), static_cast<float>(wd), static_cast<float>(scale), fptr(u),
                     fptr(e), static_cast<float>(rho), n, cur_stream());
}

void zero_at_hip(const c10::optional<at::Tensor>& a, const c10::optional<at::Tensor>& b,
                 const c10::optional<at::Tensor>& c, const at::Tensor& idx) {
  c10::hip::HIPGuardMasqueradingAsCUDA guard(idx.device());
  launch_zero_at(fptr(a), fptr(b), fptr(c), idx.data_ptr<int64_t>(), idx.numel(), cur_stream());
}

at::Tensor scatter_dense_hip(const at::Tensor& idx, const at::Tensor& vals, int64_t n) {
  c10::hip::HIPGuardMasqueradingAsCUDA guard(vals.device());
  auto out = at::empty({n}, vals.options());
  launch_scatter_dense(out.data_ptr<float>(), n, idx.data_ptr<int64_t>(), vals.data_ptr<float>(),
                       idx.numel(), cur_stream());
  return out;
}

at::Tensor augment_run(const at::Tensor& data, const at::Tensor& idx, int64_t pad, bool flip,
                       const at::Tensor& mean, const at::Tensor& inv_std, int64_t seed,
                       bool out_bf16, const c10::optional<at::Tensor>& keys, const at::Tensor* targets,
                       at::Tensor* y) {
  TORCH_CHECK(data.scalar_type() == at::kByte && data.dim() == 4 && data.is_contiguous(),
              "data must be uint8 [N,H,W,C] contiguous");
  TORCH_CHECK(data.size(3) <= 4, "at most 4 channels");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(data.device());
  const int64_t B = idx.numel(), H = data.size(1), W = data.size(2), C = data.size(3);
  // 3-channel bf16 batches are stored with a 4-channel pixel stride (the native
  // input conv reads one 8-byte load per tap); the result is a [B, C, H, W] view
  const int64_t CS = (out_bf16 && C == 3) ? 4 : C;
  auto out = at::empty({B, H, W, CS}, data.options().dtype(at::kBFloat16));
  auto mc = mean.to(data.device(), at::kFloat).contiguous();
  auto sc = inv_std.to(data.device(), at::kFloat).contiguous();
  auto ic = idx.contiguous();
  const int64_t* tp = nullptr;
  int64_t* yp = nullptr;
  if (targets != nullptr) {
    TORCH_CHECK(targets->scalar_type() == at::kLong && targets->dim() == 1 && targets->is_contiguous() &&
                    targets->device() == data.device() && targets->size(0) == data.size(0),
                "augment: targets must be a contiguous int64 [N] on the data's device");
    *y = at::empty({B}, targets->options());
    tp = targets->data_ptr<int64_t>();
    yp = y->data_ptr<int64_t>();
  }
  launch_augment_u8_nhwc(data.data_ptr<uint8_t>(), ic.data_ptr<int64_t>(), B,
                         static_cast<int>(H), static_cast<int>(W), static_cast<int>(C),
                         static_cast<int>(pad), flip ? 1 : 0, mc.data_ptr<float>(),
                         sc.data_ptr<float>(), static_cast<uint64_t>(seed), key_ptr(keys, B),
                         reinterpret_cast<uint16_t*>(out.data_ptr()), static_cast<int>(CS),
                         cur_stream(), tp, yp);
  auto o = out.narrow(3, 0, C).permute({0, 3, 1, 2});
  return out_bf16 ? o : o.to(at::kFloat);
}

at::Tensor augment_hip(const at::Tensor& data, const at::Tensor& idx, int64_t pad, bool flip,
                       const at::Tensor& mean, const at::Tensor& inv_std, int64_t seed,
                       bool out_bf16, const c10::optional<at::Tensor>& keys) {
  return augment_run(data, idx, pad, flip, mean, inv_std, seed, out_bf16, keys, nullptr, nullptr);
}

// the augmented batch and its labels targets[idx] from one kernel
std::tuple<at::Tensor, at::Tensor> augment_y_hip(const at::Tensor& data, const at::Tensor& idx, int64_t pad,
                                                 bool flip, const at::Tensor& mean, const at::Tensor& inv_std,
                                                 int64_t seed, bool out_bf16, const c10::optional<at::Tensor>& keys,
                                                 const at::Tensor& targets) {
  at::Tensor y;
  auto x = augment_run(data, idx, pad, flip, mean, inv_std, seed, out_bf16, keys, &targets, &y);
  return {x, y};
}

// ------------------------------------------------------- planned sketch ops
at::Tensor cs_hash_all_hip(const at::Tensor& hashes, const at::Tensor& blk_off,
                           const at::Tensor& blk_sign, int64_t num_blocks, int64_t d, int64_t c,
                           const at::Tensor& like) {
  c10::hip::HIPGuardMasqueradingAsCUDA guard(like.device());
  auto ctx = make_ctx(hashes, blk_off, blk_sign, num_blocks, d, c, true);
  auto out = at::empty({d, static_cast<int64_t>(ctx.geom.r)}, like.options().dtype(at::kInt));
  launch_cs_hash_all(ctx.rows, ctx.geom, ctx.blk_off, ctx.blk_sign, out.data_ptr<int32_t>(),
                     cur_stream());
  return out;
}

// CPU twin of cs_hash_all (same host/device hash code): lets the plan
// builder and its invariants be tested without a GPU
at::Tensor cs_hash_all_cpu(const at::Tensor& hashes, const at::Tensor& blk_off,
                           const at::Tensor& blk_sign, int64_t num_blocks, int64_t d, int64_t c,
                           const at::Tensor& like) {
  auto ctx = make_ctx(hashes, blk_off, blk_sign, num_blocks, d, c, false);
  const int64_t r = ctx.geom.r;
  const int64_t nb = ctx.geom.num_blocks;
  auto out = at::empty({d, r}, like.options().dtype(at::kInt));
  int32_t* o = out.data_ptr<int32_t>();
  at::parallel_for(0, d, 1 << 14, [&](int64_t b, int64_t e) {
    for (int64_t i = b; i < e; ++i) {
      uint32_t blk, t;
      split_block(static_cast<uint32_t>(i), ctx.geom, &blk, &t);
      for (int64_t j = 0; j < r; ++j) {
        uint32_t bk;
        float s;
        hash_t(ctx.rows.row[j], t, blk, ctx.geom, ctx.blk_off + j * nb, ctx.blk_sign + j * nb, &bk,
               &s);
        o[i * r + j] = static_cast<int32_t>(bk | (s < 0.f ? 0x80000000u : 0u));
      }
    }
  });
  return out;
}

// the exact (atomic-free) plan when its LDS segment fits, else the dense one
bool any_plan_geometry(int64_t d, int64_t r, int64_t c, PlanGeom* p) {
  return planned_geometry(d, r, c, p) || planned_geometry_dense(d, r, c, p);
}

PlanGeom plan_geom_or_throw(int64_t d, int64_t r, int64_t c) {
  PlanGeom p;
  TORCH_CHECK(any_plan_geometry(d, r, c, &p), "planned sketch: unsupported geometry d=", d,
              " r=", r, " c=", c);
  return p;
}

PlannedArgs planned_args(at::TensorList plan, const PlanGeom& p, int64_t d, int64_t r) {
  // plan = [src_info i16, ent_info i16, perm i16, csr i32, base i32, off i32, seg i32,
  //         vals f32, p2_src i32, p2_pos i32]
  TORCH_CHECK(plan.size() == 10 || plan.size() == 11, "plan must have 10 or 11 tensors");
  const int64_t n = d * r;
  TORCH_CHECK(plan[0].numel() == n && plan[1].numel() == n && plan[2].numel() == n &&
                  plan[3].numel() == p.num_tiles * p.tile + 1 &&
                  plan[4].numel() == p.num_chunks * p.num_tiles &&
                  plan[5].numel() == p.num_chunks * (p.num_tiles + 1) &&
                  plan[6].numel() == p.num_tiles + 1 && plan[7].numel() >= n &&
                  plan[8].numel() == p.num_tiles * p.num_chunks &&
                  plan[9].numel() == p.num_tiles * (p.num_chunks + 1),
              "sketch plan does not match the geometry");
  for (int i = 0; i < 3; ++i)
    TORCH_CHECK(plan[i].scalar_type() == at::kShort && plan[i].is_contiguous(), "plan[", i,
                "] must be contiguous int16");
  for (int i : {3, 4, 5, 6, 8, 9})
    TORCH_CHECK(plan[i].scalar_type() == at::kInt && plan[i].is_contiguous(), "plan[", i,
                "] must be contiguous int32");
  TORCH_CHECK(plan[7].scalar_type() == at::kFloat, "plan[7] must be float32");
  PlannedArgs a;
  a.src_info = reinterpret_cast<const uint16_t*>(plan[0].data_ptr<int16_t>());
  a.ent_info = reinterpret_cast<const uint16_t*>(plan[1].data_ptr<int16_t>());
  a.perm = reinterpret_cast<const uint16_t*>(plan[2].data_ptr<int16_t>());
  a.csr = plan[3].data_ptr<int32_t>();
  a.base = plan[4].data_ptr<int32_t>();
  a.off = plan[5].data_ptr<int32_t>();
  a.seg = plan[6].data_ptr<int32_t>();
  a.vals = plan[7].data_ptr<float>();
  a.p2_src = plan[8].data_ptr<int32_t>();
  a.p2_pos = plan[9].data_ptr<int32_t>();
  if (plan.size() == 11 && p.dense) {
    // int64 split partials, then max|v| per chunk and overall (as floats)
    const int64_t nfx = p.p2_splits * p.num_tiles * p.tile;  // split stride num_tiles*tile
    TORCH_CHECK(plan[10].scalar_type() == at::kLong && plan[10].is_contiguous() &&
                    plan[10].numel() * 2 >= nfx * 2 + p.num_chunks + 1,
                "plan[10] must be the dense plan's int64 scratch");
    a.fx = plan[10].data_ptr<int64_t>();
    a.bmax = reinterpret_cast<float*>(a.fx + nfx);
    a.gmax = a.bmax + p.num_chunks;
  }
  return a;
}

void cs_encode_planned_hip(at::Tensor table, const at::Tensor& vec, double scale,
                           const c10::optional<at::Tensor>& wvec, double wscale, int64_t c,
                           at::TensorList plan, bool overwrite) {
  check_f32(table, "table");
  check_f32(vec, "vec");
  if (wvec.has_value() && wvec->defined()) {
    check_f32(*wvec, "wvec");
    TORCH_CHECK(wvec->numel() == vec.numel(), "wvec must match vec");
  }
  c10::hip::HIPGuardMasqueradingAsCUDA guard(table.device());
  const int64_t d = vec.numel(), r = table.numel() / c;
  const PlanGeom p = plan_geom_or_throw(d, r, c);
  launch_cs_encode_planned(table.data_ptr<float>(), vec.data_ptr<float>(), fptr(wvec),
                           static_cast<float>(scale), static_cast<float>(wscale), d,
                           static_cast<int>(r), c, p, planned_args(plan, p, d, r), overwrite, cur_stream());
}

// est [d]; with 0 <= c0 < c1 only the coordinates of plan chunks [c0, c1) are
// computed (a rank's shard of the unsketch; the rest of est is left unset)
at::Tensor cs_query_planned_hip(const at::Tensor& table, int64_t d, at::TensorList plan, int64_t c0,
                                int64_t c1) {
  check_f32(table, "table");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(table.device());
  const int64_t c = table.size(-1), r = table.numel() / c;
  const PlanGeom p = plan_geom_or_throw(d, r, c);
  TORCH_CHECK(c0 >= 0 && (c1 < 0 || (c1 > c0 && c1 <= p.num_chunks)),
              "cs_query_planned: chunk range out of bounds");
  auto est = at::empty({d}, table.options());
  launch_cs_query_planned(table.data_ptr<float>(), est.data_ptr<float>(), d, static_cast<int>(r),
                          c, p, planned_args(plan, p, d, r), cur_stream(), c0, c1);
  return est;
}

// [tile, num_tiles, chunk, num_chunks, dense, p2_splits] of the planned sketch, [] if unsupported
std::vector<int64_t> plan_geometry(int64_t d, int64_t r, int64_t c) {
  PlanGeom p;
  if (!any_plan_geometry(d, r, c, &p)) return {};
  return {p.tile, p.num_tiles, p.chunk, p.num_chunks, p.dense ? 1 : 0, p.p2_splits};
}

std::tuple<at::Tensor, at::Tensor> relu_maxpool_hip(const at::Tensor& x, int64_t k) {
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && x.dim() == 4 &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "relu_maxpool: x must be bf16 NCHW with channels_last memory");
  TORCH_CHECK(k == 2 || k == 4, "k must be 2 or 4");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(C % 8 == 0 && H % k == 0 && W % k == 0, "relu_maxpool: C%8, H%k, W%k");
  TORCH_CHECK(x.numel() < (int64_t(1) << 32) && x.size(0) * H * W < (int64_t(1) << 31),
              "relu_maxpool: 32-bit index range");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  auto y = at::empty({N, C, H / k, W / k}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto idx = at::empty({N, C, H / k, W / k},
                       x.options().dtype(at::kByte).memory_format(at::MemoryFormat::ChannelsLast));
  launch_relu_maxpool_fwd(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                          reinterpret_cast<uint16_t*>(y.data_ptr()), idx.data_ptr<uint8_t>(),
                          static_cast<int>(N), static_cast<int>(H), static_cast<int>(W),
                          static_cast<int>(C), static_cast<int>(k), cur_stream());
  return {y, idx};
}

at::Tensor relu_maxpool_backward_hip(const at::Tensor& gy, const at::Tensor& idx, int64_t k) {
  TORCH_CHECK(gy.scalar_type() == at::kBFloat16 && idx.scalar_type() == at::kByte, "dtypes");
  auto g = gy.contiguous(at::MemoryFormat::ChannelsLast);
  TORCH_CHECK(idx.is_contiguous(at::MemoryFormat::ChannelsLast), "idx layout");
  const int64_t N = g.size(0), C = g.size(1), OH = g.size(2), OW = g.size(3);
  c10::hip::HIPGuardMasqueradingAsCUDA guard(gy.device());
  auto gx = at::empty({N, C, OH * k, OW * k},
                      gy.options().memory_format(at::MemoryFormat::ChannelsLast));
  launch_relu_maxpool_bwd(reinterpret_cast<const uint16_t*>(g.data_ptr()), idx.data_ptr<uint8_t>(),
                          reinterpret_cast<uint16_t*>(gx.data_ptr()), static_cast<int>(N),
                          static_cast<int>(OH * k), static_cast<int>(OW * k),
                          static_cast<int>(C), static_cast<int>(k), cur_stream());
  return gx;
}

// --------------------------------------------------------------- im2col
const uint16_t* bf16_ptr(const at::Tensor& t);
void check_nhwc_bf16(const at::Tensor& t, const char* name);

int64_t conv_out_size(int64_t in, int64_t k, int64_t stride, int64_t pad) {
  return (in + 2 * pad - k) / stride + 1;
}

// col [N*OH*OW, Kc] of x (bf16, channels innermost: x.stride(1) == 1, any
// pixel stride -- the augmentation kernel's 4-channel layout included)
at::Tensor im2col_hip(const at::Tensor& x, int64_t R, int64_t S, int64_t stride, int64_t pad,
                      int64_t Kc) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 4 && x.stride(1) == 1,
              "im2col: x must be a bf16 NCHW tensor with channels innermost");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(R >= 1 && S >= 1 && stride >= 1 && pad >= 0 && pad < R && pad < S, "im2col: geometry");
  const int64_t OH = conv_out_size(H, R, stride, pad), OW = conv_out_size(W, S, stride, pad);
  TORCH_CHECK(OH > 0 && OW > 0, "im2col: empty output");
  TORCH_CHECK(Kc % 8 == 0 && Kc >= R * S * C, "im2col: Kc must be a multiple of 8 and >= R*S*C");
  const int64_t P = N * OH * OW;
  TORCH_CHECK(P * (Kc / 8) < (int64_t(1) << 32) && P < (int64_t(1) << 31) &&
                  x.stride(0) * N < (int64_t(1) << 31),
              "im2col: 32-bit index range");
  TORCH_CHECK(x.stride(2) >= 0 && x.stride(3) >= C, "im2col: pixel strides");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  auto col = at::empty({P, Kc}, x.options());
  Im2colArgs a{};
  a.x = reinterpret_cast<const uint16_t*>(x.data_ptr());
  a.col = reinterpret_cast<uint16_t*>(col.data_ptr());
  a.N = static_cast<int>(N); a.H = static_cast<int>(H); a.W = static_cast<int>(W);
  a.C = static_cast<int>(C); a.OH = static_cast<int>(OH); a.OW = static_cast<int>(OW);
  a.R = static_cast<int>(R); a.S = static_cast<int>(S);
  a.stride = static_cast<int>(stride); a.pad = static_cast<int>(pad); a.Kc = static_cast<int>(Kc);
  a.sN = x.stride(0); a.sH = x.stride(2); a.sW = x.stride(3);
  a.vec = C % 8 == 0 && a.sN % 8 == 0 && a.sH % 8 == 0 && a.sW % 8 == 0 &&
          reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0;
  launch_im2col(a, cur_stream());
  return col;
}

// gx [N, C, H, W] (channels_last) of the column-image gradient gcol [N*OH*OW, Kc]
at::Tensor col2im_hip(const at::Tensor& gcol, int64_t N, int64_t H, int64_t W, int64_t C, int64_t R,
                      int64_t S, int64_t stride, int64_t pad) {
  TORCH_CHECK(gcol.is_cuda() && gcol.scalar_type() == at::kBFloat16 && gcol.dim() == 2 &&
                  gcol.is_contiguous(),
              "col2im: gcol must be a contiguous bf16 [P, Kc] tensor");
  TORCH_CHECK(C % 8 == 0 && R >= 1 && S >= 1 && stride >= 1 && pad >= 0 && pad < R && pad < S,
              "col2im: geometry (C % 8 == 0)");
  const int64_t OH = conv_out_size(H, R, stride, pad), OW = conv_out_size(W, S, stride, pad);
  const int64_t Kc = gcol.size(1);
  TORCH_CHECK(gcol.size(0) == N * OH * OW && Kc % 8 == 0 && Kc >= R * S * C, "col2im: gcol shape");
  TORCH_CHECK(N * H * W * C < (int64_t(1) << 34) && gcol.numel() < (int64_t(1) << 40) &&
                  N * H * W * (C / 8) < (int64_t(1) << 32),
              "col2im: index range");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(gcol.device());
  auto gx = at::empty({N, C, H, W}, gcol.options().memory_format(at::MemoryFormat::ChannelsLast));
  Im2colArgs a{};
  a.N = static_cast<int>(N); a.H = static_cast<int>(H); a.W = static_cast<int>(W);
  a.C = static_cast<int>(C); a.OH = static_cast<int>(OH); a.OW = static_cast<int>(OW);
  a.R = static_cast<int>(R); a.S = static_cast<int>(S);
  a.stride = static_cast<int>(stride); a.pad = static_cast<int>(pad); a.Kc = static_cast<int>(Kc);
  launch_col2im(a, reinterpret_cast<const uint16_t*>(gcol.data_ptr()),
                reinterpret_cast<uint16_t*>(gx.data_ptr()), cur_stream());
  return gx;
}

// bf16 [K, Kc] GEMM image of an fp32 [K, C, R, S] conv weight (column (r*S+s)*C + c)
at::Tensor conv_weight_rsc_hip(const at::Tensor& w, int64_t Kc) {
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kFloat && w.dim() == 4 && w.is_contiguous(),
              "conv_weight_rsc: w must be a contiguous fp32 [K, C, R, S] tensor");
  const int64_t K = w.size(0), C = w.size(1), RS = w.size(2) * w.size(3);
  TORCH_CHECK(Kc % 8 == 0 && Kc >= RS * C, "conv_weight_rsc: Kc");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(w.device());
  auto out = at::empty({K, Kc}, w.options().dtype(at::kBFloat16));
  launch_weight_rsc(w.data_ptr<float>(), reinterpret_cast<uint16_t*>(out.data_ptr()),
                    static_cast<int>(K), static_cast<int>(C), static_cast<int>(RS),
                    static_cast<int>(Kc), cur_stream());
  return out;
}

// dst [G, K, C*RS] fp32 (rows may be strided) (+)= the (c, r, s)-ordered sum of
// the split-K partial products src [G*splits, K, Kc] ((r, s, c) columns)
void wgrad_rsc_add_hip(at::Tensor dst, const at::Tensor& src, int64_t splits, int64_t C, int64_t RS,
                       bool accumulate) {
  TORCH_CHECK(dst.is_cuda() && dst.scalar_type() == at::kFloat && dst.dim() == 3 && dst.stride(2) == 1 &&
                  dst.stride(1) == dst.size(2) && dst.size(2) == C * RS,
              "wgrad_rsc_add: dst must be fp32 [G, K, C*RS] with contiguous rows");
  const int64_t G = dst.size(0), K = dst.size(1);
  TORCH_CHECK(src.is_cuda() && src.scalar_type() == at::kFloat && src.dim() == 3 && src.is_contiguous() &&
                  src.size(0) == G * splits && src.size(1) == K && src.size(2) >= C * RS,
              "wgrad_rsc_add: src must be contiguous fp32 [G*splits, K, Kc]");
  TORCH_CHECK(K * C * RS < (int64_t(1) << 31), "wgrad_rsc_add: size");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(dst.device());
  launch_wgrad_rsc_add(dst.data_ptr<float>(), G > 1 ? dst.stride(0) : 0, src.data_ptr<float>(),
                       static_cast<int>(G), static_cast<int>(splits), static_cast<int>(K),
                       static_cast<int>(C), static_cast<int>(RS), static_cast<int>(src.size(2)),
                       accumulate, cur_stream());
}

std::tuple<at::Tensor, at::Tensor> maxpool_fwd_hip(const at::Tensor& x, int64_t k, int64_t s, int64_t p) {
  check_nhwc_bf16(x, "maxpool: x");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(C % 8 == 0 && k >= 1 && k <= 15 && s >= 1 && p >= 0 && 2 * p <= k, "maxpool: geometry");
  const int64_t OH = conv_out_size(H, k, s, p), OW = conv_out_size(W, k, s, p);
  TORCH_CHECK(OH > 0 && OW > 0 && N * OH * OW * (C / 8) < (int64_t(1) << 32), "maxpool: size");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  auto y = at::empty({N, C, OH, OW}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto codes = at::empty({N, C, OH, OW},
                         x.options().dtype(at::kByte).memory_format(at::MemoryFormat::ChannelsLast));
  launch_maxpool_fwd(bf16_ptr(x), reinterpret_cast<uint16_t*>(y.data_ptr()), codes.data_ptr<uint8_t>(),
                     static_cast<int>(N), static_cast<int>(H), static_cast<int>(W), static_cast<int>(C),
                     static_cast<int>(k), static_cast<int>(s), static_cast<int>(p), cur_stream());
  return {y, codes};
}

at::Tensor maxpool_bwd_hip(const at::Tensor& gy, const at::Tensor& codes, int64_t H, int64_t W, int64_t k,
                           int64_t s, int64_t p) {
  TORCH_CHECK(gy.scalar_type() == at::kBFloat16 && codes.scalar_type() == at::kByte, "maxpool_bwd: dtypes");
  auto g = gy.contiguous(at::MemoryFormat::ChannelsLast);
  TORCH_CHECK(codes.is_contiguous(at::MemoryFormat::ChannelsLast) && codes.sizes() == g.sizes(),
              "maxpool_bwd: codes layout");
  const int64_t N = g.size(0), C = g.size(1);
  TORCH_CHECK(C % 8 == 0 && g.size(2) == conv_out_size(H, k, s, p) && g.size(3) == conv_out_size(W, k, s, p),
              "maxpool_bwd: geometry");
  TORCH_CHECK(N * H * W * (C / 8) < (int64_t(1) << 32), "maxpool_bwd: size");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(gy.device());
  auto gx = at::empty({N, C, H, W}, gy.options().memory_format(at::MemoryFormat::ChannelsLast));
  launch_maxpool_bwd(bf16_ptr(g), codes.data_ptr<uint8_t>(), reinterpret_cast<uint16_t*>(gx.data_ptr()),
                     static_cast<int>(N), static_cast<int>(H), static_cast<int>(W), static_cast<int>(C),
                     static_cast<int>(k), static_cast<int>(s), static_cast<int>(p), cur_stream());
  return gx;
}

// --------------------------------------------------------------- conv3x3
const uint16_t* bf16_ptr(const at::Tensor& t) {
  return reinterpret_cast<const uint16_t*>(t.data_ptr());
}

void check_nhwc_bf16(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16 && t.dim() == 4 &&
                  t.is_contiguous(at::MemoryFormat::ChannelsLast),
              name, " must be a bf16 NCHW tensor with channels_last memory");
}

const uint16_t* opt_like(const c10::optional<at::Tensor>& t, const at::Tensor& y, const char* name) {
  if (!t.has_value() || !t->defined()) return nullptr;
  check_nhwc_bf16(*t, name);
  TORCH_CHECK(t->sizes() == y.sizes(), name, " must have the output's shape");
  return bf16_ptr(*t);
}

// launch_conv3x3_fwd with its split-K workspace (if the launch wants one:
// a grid of few tiles) from the caching allocator -- stream-ordered reuse,
// and under a tape recording the capture's private pool keeps its address
void run_conv3x3_fwd(ConvFwdArgs& a) {
  const int64_t ws = conv3x3_fwd_split_floats(a);
  at::Tensor part;
  if (ws > 0) {
    part = at::empty({ws}, at::TensorOptions().dtype(at::kFloat).device(
                               at::Device(at::kCUDA, c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().device_index())));
    a.part = part.data_ptr<float>();
  }
  launch_conv3x3_fwd(a, cur_stream());
}

// y = act(conv3x3(x, w)) ; w bf16 [K][3][3][C] contiguous
at::Tensor conv3x3_fwd_impl(const at::Tensor& x, const at::Tensor& w, bool relu,
                            const c10::optional<at::Tensor>& mask,
                            const c10::optional<at::Tensor>& addend, at::Tensor* pre) {
  check_nhwc_bf16(x, "conv3x3: x");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(w.scalar_type() == at::kBFloat16 && w.is_contiguous() && w.dim() == 4 &&
                  w.size(1) == 3 && w.size(2) == 3 && w.size(3) == C,
              "conv3x3: w must be contiguous bf16 [K, 3, 3, C]");
  const int64_t K = w.size(0);
  TORCH_CHECK(conv3x3_supported(static_cast<int>(C), static_cast<int>(K)),
              "conv3x3: C and K must be multiples of 64");
  TORCH_CHECK(N * H * W < (1ll << 31) && N * H * W * std::max(C, K) < (1ll << 40), "conv3x3: size");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  auto y = at::empty({N, K, H, W}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  ConvFwdArgs a;
  a.x = bf16_ptr(x);
  a.w = bf16_ptr(w);
  a.y = reinterpret_cast<uint16_t*>(y.data_ptr());
  a.mask = opt_like(mask, y, "conv3x3: mask");
  a.addend = opt_like(addend, y, "conv3x3: addend");
  a.P = static_cast<int>(N * H * W);
  a.H = static_cast<int>(H);
  a.W = static_cast<int>(W);
  a.C = static_cast<int>(C);
  a.K = static_cast<int>(K);
  a.relu = relu ? 1 : 0;
  a.y_pre = nullptr;
  a.pool_idx = nullptr;
  a.pool = 0;
  if (pre != nullptr) {
    TORCH_CHECK(a.addend != nullptr, "conv3x3: the pre-add output needs an addend");
    *pre = at::empty_like(y, y.options().memory_format(at::MemoryFormat::ChannelsLast));
    a.y_pre = reinterpret_cast<uint16_t*>(pre->data_ptr());
  }
  if (a.P > 0) run_conv3x3_fwd(a);
  return y;
}

// Grouped 3x3 conv (stride 1, pad 1) on channel-stacked images, batched
// FedAvg (ops/nn.py _GConv3x3): x [N, G*C, H, W] channels_last bf16, w the
// [G*kg, 3, 3, C] bf16 image of G per-group weights [kg, C, 3, 3]; output
// channel group g reads input channels [g C, (g+1) C).  An empty tensor when
// the halo kernels have no tiling for the shape (the caller falls back).
at::Tensor conv3x3_fwd_grouped_hip(const at::Tensor& x, const at::Tensor& w, int64_t G) {
  check_nhwc_bf16(x, "conv3x3_fwd_grouped: x");
  const int64_t N = x.size(0), GC = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(G >= 1 && GC % G == 0, "conv3x3_fwd_grouped: channels not a multiple of G");
  const int64_t C = GC / G;
  TORCH_CHECK(w.scalar_type() == at::kBFloat16 && w.is_contiguous() && w.dim() == 4 &&
                  w.size(1) == 3 && w.size(2) == 3 && w.size(3) == C && w.size(0) % G == 0,
              "conv3x3_fwd_grouped: w must be contiguous bf16 [G*kg, 3, 3, C]");
  const int64_t K = w.size(0), kg = K / G;
  TORCH_CHECK(N * H * W * std::max(GC, K) < (1ll << 31), "conv3x3_fwd_grouped: size");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  auto y = at::empty({N, K, H, W}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  ConvFwdArgs a;
  a.x = bf16_ptr(x);
  a.w = bf16_ptr(w);
  a.y = reinterpret_cast<uint16_t*>(y.data_ptr());
  a.mask = nullptr;
  a.addend = nullptr;
  a.y_pre = nullptr;
  a.pool_idx = nullptr;
  a.pool = 0;
  a.relu = 0;
  a.P = static_cast<int>(N * H * W);
  a.H = static_cast<int>(H);
  a.W = static_cast<int>(W);
  a.C = static_cast<int>(C);
  a.K = static_cast<int>(K);
  a.x_stride = static_cast<int>(GC);
  a.kg = static_cast<int>(kg);
  if (a.P == 0) return y;
  if (!launch_conv3x3_fwd_grouped(a, cur_stream())) return at::empty({0}, x.options());
  return y;
}

// dW [G*kg, C, 3, 3] fp32 of the grouped conv above (dy [N, G*kg, H, W], x
// [N, G*C, H, W], channels_last bf16); empty when unsupported
at::Tensor conv3x3_wgrad_grouped_ch_hip(const at::Tensor& dy, const at::Tensor& x, int64_t G) {
  check_nhwc_bf16(dy, "conv3x3_wgrad_grouped_ch: dy");
  check_nhwc_bf16(x, "conv3x3_wgrad_grouped_ch: x");
  const int64_t N = x.size(0), GC = x.size(1), H = x.size(2), W = x.size(3), K = dy.size(1);
  TORCH_CHECK(dy.size(0) == N && dy.size(2) == H && dy.size(3) == W && G >= 1 && GC % G == 0 && K % G == 0,
              "conv3x3_wgrad_grouped_ch: shapes");
  const int64_t C = GC / G, kg = K / G;
  if (!conv3x3_wgrad_grouped_supported(static_cast<int>(H), static_cast<int>(W), static_cast<int>(K),
                                       static_cast<int>(C), static_cast<int>(kg)))
    return at::empty({0}, x.options().dtype(at::kFloat));
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  auto dw = at::empty({K, C, 3, 3}, x.options().dtype(at::kFloat).memory_format(at::MemoryFormat::Contiguous));
  const int P = static_cast<int>(N * H * W);
  const int splits = conv3x3_wgrad_splits(P, static_cast<int>(H), static_cast<int>(W), static_cast<int>(K),
                                          static_cast<int>(C));
  auto slab = at::empty({splits * K * 9 * C}, dw.options());
  ConvWgradArgs a;
  a.dy = bf16_ptr(dy);
  a.x = bf16_ptr(x);
  a.slab = slab.data_ptr<float>();
  a.P = P;
  a.H = static_cast<int>(H);
  a.W = static_cast<int>(W);
  a.C = static_cast<int>(C);
  a.K = static_cast<int>(K);
  a.splits = splits;
  a.x_stride = static_cast<int>(GC);
  a.kg = static_cast<int>(kg);
  if (P > 0) launch_conv3x3_wgrad(a, dw.data_ptr<float>(), 0.f, cur_stream());
  else dw.zero_();
  return dw;
}

at::Tensor conv3x3_fwd_hip(const at::Tensor& x, const at::Tensor& w, bool relu,
                           const c10::optional<at::Tensor>& mask,
                           const c10::optional<at::Tensor>& addend) {
  return conv3x3_fwd_impl(x, w, relu, mask, addend, nullptr);
}

// y = conv3x3(x, w) and y_dual = y where dual_mask > 0 else 0 (two outputs of
// one epilogue: a dgrad and the relu backward of its consumer's other input)
std::tuple<at::Tensor, at::Tensor> conv3x3_fwd_dual_hip(const at::Tensor& x, const at::Tensor& w,
                                                        const at::Tensor& dual_mask) {
  check_nhwc_bf16(x, "conv3x3_dual: x");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(w.scalar_type() == at::kBFloat16 && w.is_contiguous() && w.dim() == 4 &&
                  w.size(1) == 3 && w.size(2) == 3 && w.size(3) == C,
              "conv3x3_dual: w must be contiguous bf16 [K, 3, 3, C]");
  const int64_t K = w.size(0);
  TORCH_CHECK(conv3x3_supported(static_cast<int>(C), static_cast<int>(K)),
              "conv3x3_dual: C and K must be multiples of 64");
  TORCH_CHECK(N * H * W < (1ll << 31), "conv3x3_dual: size");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  auto y = at::empty({N, K, H, W}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto yd = at::empty_like(y, y.options().memory_format(at::MemoryFormat::ChannelsLast));
  ConvFwdArgs a{};
  a.x = bf16_ptr(x);
  a.w = bf16_ptr(w);
  a.y = reinterpret_cast<uint16_t*>(y.data_ptr());
  a.mask = nullptr;
  a.addend = nullptr;
  a.y_pre = nullptr;
  a.pool_idx = nullptr;
  a.dual_mask = opt_like(c10::optional<at::Tensor>(dual_mask), y, "conv3x3_dual: dual_mask");
  a.y_dual = reinterpret_cast<uint16_t*>(yd.data_ptr());
  a.P = static_cast<int>(N * H * W);
  a.H = static_cast<int>(H);
  a.W = static_cast<int>(W);
  a.C = static_cast<int>(C);
  a.K = static_cast<int>(K);
  a.relu = 0;
  a.pool = 0;
  if (a.P > 0) run_conv3x3_fwd(a);
  return {y, yd};
}

// dgrad with the relu + 2x2 max-pool backward of the layer below fused into
// the epilogue: y [N, K, 2H, 2W] (channels_last) = unpool(conv3x3(x, w) +
// addend) with idx [N, K, H, W] the pool's window codes (conv3x3_fwd_pool2)
at::Tensor conv3x3_fwd_unpool_hip(const at::Tensor& x, const at::Tensor& w,
                                  const c10::optional<at::Tensor>& addend, const at::Tensor& idx) {
  check_nhwc_bf16(x, "conv3x3_unpool: x");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(w.scalar_type() == at::kBFloat16 && w.is_contiguous() && w.dim() == 4 &&
                  w.size(1) == 3 && w.size(2) == 3 && w.size(3) == C,
              "conv3x3_unpool: w must be contiguous bf16 [K, 3, 3, C]");
  const int64_t K = w.size(0);
  TORCH_CHECK(conv3x3_supported(static_cast<int>(C), static_cast<int>(K)),
              "conv3x3_unpool: C and K must be multiples of 64");
  TORCH_CHECK(N * 4 * H * W < (1ll << 31), "conv3x3_unpool: size");
  TORCH_CHECK(idx.scalar_type() == at::kByte && idx.dim() == 4 && idx.size(0) == N &&
                  idx.size(1) == K && idx.size(2) == H && idx.size(3) == W && idx.device() == x.device() &&
                  idx.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv3x3_unpool: idx must be uint8 channels_last [N, K, H, W]");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  auto y = at::empty({N, K, 2 * H, 2 * W}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto pooled = at::empty({N, K, H, W}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  ConvFwdArgs a{};
  a.x = bf16_ptr(x);
  a.w = bf16_ptr(w);
  a.y = reinterpret_cast<uint16_t*>(y.data_ptr());
  a.mask = nullptr;
  a.addend = opt_like(addend, pooled, "conv3x3_unpool: addend");
  a.y_pre = nullptr;
  a.pool_idx = nullptr;
  a.unpool_idx = idx.data_ptr<uint8_t>();
  a.P = static_cast<int>(N * H * W);
  a.H = static_cast<int>(H);
  a.W = static_cast<int>(W);
  a.C = static_cast<int>(C);
  a.K = static_cast<int>(K);
  a.relu = 0;
  a.pool = 0;
  if (a.P > 0) run_conv3x3_fwd(a);
  return y;
}

// y = maxpool2(relu(conv3x3(x, w))) [N, K, H/2, W/2] (channels_last) and the
// 1-byte window codes of csrc/pool.hip (for relu_maxpool_backward)
std::tuple<at::Tensor, at::Tensor> conv3x3_fwd_pool2_hip(const at::Tensor& x, const at::Tensor& w) {
  check_nhwc_bf16(x, "conv3x3_pool: x");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(w.scalar_type() == at::kBFloat16 && w.is_contiguous() && w.dim() == 4 &&
                  w.size(1) == 3 && w.size(2) == 3 && w.size(3) == C,
              "conv3x3_pool: w must be contiguous bf16 [K, 3, 3, C]");
  const int64_t K = w.size(0);
  TORCH_CHECK(conv3x3_supported(static_cast<int>(C), static_cast<int>(K)) &&
                  conv3x3_pool_supported(static_cast<int>(H), static_cast<int>(W), static_cast<int>(K)),
              "conv3x3_pool: unsupported shape");
  TORCH_CHECK(N * H * W < (1ll << 31), "conv3x3_pool: size");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  auto y = at::empty({N, K, H / 2, W / 2}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto idx = at::empty({N, K, H / 2, W / 2},
                       x.options().dtype(at::kByte).memory_format(at::MemoryFormat::ChannelsLast));
  ConvFwdArgs a{};
  a.x = bf16_ptr(x);
  a.w = bf16_ptr(w);
  a.y = reinterpret_cast<uint16_t*>(y.data_ptr());
  a.mask = nullptr;
  a.addend = nullptr;
  a.y_pre = nullptr;
  a.pool_idx = idx.data_ptr<uint8_t>();
  a.P = static_cast<int>(N * H * W);
  a.H = static_cast<int>(H);
  a.W = static_cast<int>(W);
  a.C = static_cast<int>(C);
  a.K = static_cast<int>(K);
  a.relu = 1;
  a.pool = 2;
  if (a.P > 0) run_conv3x3_fwd(a);
  return {y, idx};
}

// ---- ResNet-9 head (head.hip): x = res3 output [B, C, h, w] bf16 channels_last,
// w = linear weight fp32 [classes, C]
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor> head_fwd_hip(
    const at::Tensor& x, const at::Tensor& w, const at::Tensor& targets, double scale) {
  check_nhwc_bf16(x, "head: x");
  check_f32(w, "head: w");
  const int64_t B = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3), K = w.size(0);
  TORCH_CHECK(w.dim() == 2 && w.size(1) == C && head_supported(static_cast<int>(C), static_cast<int>(K)),
              "head: w must be [classes <= 128, C], C % 8 == 0");
  TORCH_CHECK(targets.scalar_type() == at::kLong && targets.is_contiguous() && targets.numel() == B,
              "head: targets int64 [B]");
  TORCH_CHECK(H * W <= 255, "head: at most 255 pooled pixels");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  auto f = x.options().dtype(at::kFloat);
  auto loss = at::empty({B}, f), correct = at::empty({B}, f), gunit = at::empty({B, K}, f);
  auto pooled = at::empty({B, C}, x.options());
  auto codes = at::empty({B, C}, x.options().dtype(at::kByte));
  launch_head_fwd(bf16_ptr(x), w.data_ptr<float>(), targets.data_ptr<int64_t>(), static_cast<int>(B),
                  static_cast<int>(C), static_cast<int>(H * W), static_cast<int>(K), static_cast<float>(scale),
                  loss.data_ptr<float>(), correct.data_ptr<float>(), gunit.data_ptr<float>(),
                  reinterpret_cast<uint16_t*>(pooled.data_ptr()), codes.data_ptr<uint8_t>(), cur_stream());
  return {loss, correct, gunit, pooled, codes};
}

// returns dx [B, C, h, w] (channels_last bf16); dw = beta * dw + dW
at::Tensor head_bwd_run(const at::Tensor& gl, const at::Tensor& gunit, const at::Tensor& w,
                        const at::Tensor& pooled, const at::Tensor& codes, int64_t H, int64_t W,
                        double scale, at::Tensor dw, double beta, const at::Tensor* ymask, at::Tensor* dxm) {
  check_f32(w, "head: w");
  const int64_t B = pooled.size(0), C = pooled.size(1), K = w.size(0);
  TORCH_CHECK(gunit.is_contiguous() && gunit.size(0) == B && gunit.size(1) == K && codes.is_contiguous() &&
                  pooled.is_contiguous(), "head_bwd: saved tensors");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(w.device());
  auto g = gl.to(at::kFloat).contiguous();
  TORCH_CHECK(g.numel() == B, "head_bwd: grad of loss [B]");
  auto dx = at::empty({B, C, H, W}, pooled.options().memory_format(at::MemoryFormat::ChannelsLast));
  check_f32(dw, "head_bwd: dw");
  TORCH_CHECK(dw.sizes() == w.sizes(), "head_bwd: dw shape");
  const uint16_t* ym = nullptr;
  uint16_t* dm = nullptr;
  if (ymask != nullptr) {
    TORCH_CHECK(ymask->scalar_type() == at::kBFloat16 && ymask->sizes() == dx.sizes() &&
                    ymask->is_contiguous(at::MemoryFormat::ChannelsLast) && ymask->device() == dx.device(),
                "head_bwd_dual: ymask must be bf16 channels_last like x");
    *dxm = at::empty_like(dx);
    ym = reinterpret_cast<const uint16_t*>(ymask->data_ptr());
    dm = reinterpret_cast<uint16_t*>(dxm->data_ptr());
  }
  launch_head_bwd(g.data_ptr<float>(), gunit.data_ptr<float>(), w.data_ptr<float>(),
                  reinterpret_cast<const uint16_t*>(pooled.data_ptr()), codes.data_ptr<uint8_t>(),
                  static_cast<int>(B), static_cast<int>(C), static_cast<int>(H * W), static_cast<int>(K),
                  static_cast<float>(scale), reinterpret_cast<uint16_t*>(dx.data_ptr()), dw.data_ptr<float>(),
                  static_cast<float>(beta), cur_stream(), ym, dm);
  return dx;
}

at::Tensor head_bwd_hip(const at::Tensor& gl, const at::Tensor& gunit, const at::Tensor& w,
                        const at::Tensor& pooled, const at::Tensor& codes, int64_t H, int64_t W,
                        double scale, at::Tensor dw, double beta) {
  return head_bwd_run(gl, gunit, w, pooled, codes, H, W, scale, dw, beta, nullptr, nullptr);
}

// dx and dx masked by ymask > 0 (the producer's ReLU backward) from one kernel
std::tuple<at::Tensor, at::Tensor> head_bwd_dual_hip(const at::Tensor& gl, const at::Tensor& gunit,
                                                     const at::Tensor& w, const at::Tensor& pooled,
                                                     const at::Tensor& codes, int64_t H, int64_t W, double scale,
                                                     at::Tensor dw, double beta, const at::Tensor& ymask) {
  at::Tensor dxm;
  auto dx = head_bwd_run(gl, gunit, w, pooled, codes, H, W, scale, dw, beta, &ymask, &dxm);
  return {dx, dxm};
}

// ghost batch norm: x [N, C, H, W] bf16 channels_last, G | N groups.
// returns (y, stat [G, 2, C] = mean, rstd, relu_bits [N*H*W*C/8] uint8: bit
// c % 8 of byte (pixel*C + c) / 8 set where y > 0 -- empty without relu);
// running stats updated in place
std::tuple<at::Tensor, at::Tensor, at::Tensor> ghost_bn_fwd_hip(const at::Tensor& x, const c10::optional<at::Tensor>& w,
                                                    const c10::optional<at::Tensor>& b, int64_t G, double eps,
                                                    double momentum, const c10::optional<at::Tensor>& run_mean,
                                                    const c10::optional<at::Tensor>& run_var, bool relu,
                                                    const c10::optional<at::Tensor>& nbt,
                                                    const c10::optional<at::Tensor>& addend,
                                                    const c10::optional<at::Tensor>& tstats) {
  check_nhwc_bf16(x, "ghost_bn: x");
  const bool has_add = addend.has_value() && addend->defined();
  if (has_add) {
    check_nhwc_bf16(*addend, "ghost_bn: addend");
    TORCH_CHECK(addend->sizes() == x.sizes(), "ghost_bn: addend must have x's shape");
  }
  const int64_t N = x.size(0), C = x.size(1), HW = x.size(2) * x.size(3);
  TORCH_CHECK(G >= 1 && N % G == 0 && C % 8 == 0 && C <= 2048, "ghost_bn: G | N, C % 8 == 0, C <= 2048");
  const int64_t M = N / G * HW;
  TORCH_CHECK(G * M * C / 8 < (int64_t{1} << 31), "ghost_bn: tensor too large");
  auto f32 = [&](const c10::optional<at::Tensor>& t, const char* n) -> float* {
    if (!t.has_value() || !t->defined()) return nullptr;
    TORCH_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous() && t->numel() == C, n);
    return t->data_ptr<float>();
  };
  float* wp = f32(w, "ghost_bn: weight f32 [C]");
  float* bp = f32(b, "ghost_bn: bias f32 [C]");
  TORCH_CHECK((wp == nullptr) == (bp == nullptr), "ghost_bn: weight and bias together");
  float* rm = f32(run_mean, "ghost_bn: running_mean f32 [C]");
  float* rv = f32(run_var, "ghost_bn: running_var f32 [C]");
  TORCH_CHECK((rm == nullptr) == (rv == nullptr), "ghost_bn: running stats together");
  int64_t* nb = nullptr;
  if (nbt.has_value() && nbt->defined()) {
    TORCH_CHECK(nbt->scalar_type() == at::kLong && nbt->numel() == 1, "ghost_bn: num_batches_tracked int64 []");
    nb = nbt->data_ptr<int64_t>();
  }
  const bool has_ts = tstats.has_value() && tstats->defined();
  if (has_ts) {  // per-128-row-tile moments from the producing GEMM (mm_nt_bnstats)
    TORCH_CHECK(tstats->is_cuda() && tstats->scalar_type() == at::kFloat && tstats->is_contiguous() &&
                    tstats->numel() == (G * M + kBnStatTile - 1) / kBnStatTile * 4 * C && M >= kBnStatTile,
                "ghost_bn: tile statistics must be fp32 [ceil(N*H*W / 128), 4, C] with >= 128 rows per group");
  }
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  const int S = bn_slabs(static_cast<int>(G), static_cast<int>(M));
  auto fo = x.options().dtype(at::kFloat);
  auto part = at::empty({bn_scratch_floats(static_cast<int>(G), static_cast<int>(M), static_cast<int>(C))}, fo);
  auto stat = at::empty({G, 2, C}, fo);
  auto ab = at::empty({G, 2, C}, fo);
  auto y = at::empty_like(x, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto bits = at::empty({relu ? x.numel() / 8 : 0}, x.options().dtype(at::kByte));
  launch_bn_fwd(bf16_ptr(x), wp, bp, static_cast<int>(G), static_cast<int>(M), static_cast<int>(C),
                static_cast<float>(eps), static_cast<float>(momentum), rm, rv, part.data_ptr<float>(),
                stat.data_ptr<float>(), ab.data_ptr<float>(), relu, nb,
                reinterpret_cast<uint16_t*>(y.data_ptr()), cur_stream(),
                has_add ? bf16_ptr(*addend) : nullptr, relu ? bits.data_ptr<uint8_t>() : nullptr,
                has_ts ? tstats->data_ptr<float>() : nullptr);
  return {y, stat, bits};
}

// returns (dx, dweight, dbias) (dweight / dbias undefined without affine, or
// when gw / gb -- existing fp32 .grad tensors -- receive them: += in place)
std::tuple<at::Tensor, at::Tensor, at::Tensor> ghost_bn_bwd_hip(const at::Tensor& dy, const at::Tensor& x,
                                                                const at::Tensor& stat,
                                                                const c10::optional<at::Tensor>& w, int64_t G,
                                                                const c10::optional<at::Tensor>& y_relu,
                                                                const c10::optional<at::Tensor>& gw,
                                                                const c10::optional<at::Tensor>& gb,
                                                                const c10::optional<at::Tensor>& ggw,
                                                                const c10::optional<at::Tensor>& ggb,
                                                                const c10::optional<at::Tensor>& dadd) {
  check_nhwc_bf16(x, "ghost_bn_bwd: x");
  check_nhwc_bf16(dy, "ghost_bn_bwd: dy");
  TORCH_CHECK(dy.sizes() == x.sizes(), "ghost_bn_bwd: dy shape");
  const bool fused_relu = y_relu.has_value() && y_relu->defined();
  if (fused_relu) {  // the forward's 1-bit ReLU mask
    TORCH_CHECK(y_relu->is_cuda() && y_relu->scalar_type() == at::kByte && y_relu->is_contiguous() &&
                    y_relu->numel() == x.numel() / 8,
                "ghost_bn_bwd: y_relu must be the forward's uint8 [numel / 8] ReLU bits");
  }
  if (dadd.has_value() && dadd->defined()) {  // receives the ReLU-masked dy
    check_nhwc_bf16(*dadd, "ghost_bn_bwd: dadd");
    TORCH_CHECK(dadd->sizes() == x.sizes() && fused_relu, "ghost_bn_bwd: dadd needs y and x's shape");
  }
  const int64_t N = x.size(0), C = x.size(1), HW = x.size(2) * x.size(3);
  const int64_t M = N / G * HW;
  TORCH_CHECK(stat.scalar_type() == at::kFloat && stat.is_contiguous() && stat.numel() == G * 2 * C,
              "ghost_bn_bwd: stat");
  const bool affine = w.has_value() && w->defined();
  const bool into = affine && gw.has_value() && gw->defined() && gb.has_value() && gb->defined();
  if (into) {
    check_f32(*gw, "ghost_bn_bwd: weight grad");
    check_f32(*gb, "ghost_bn_bwd: bias grad");
    TORCH_CHECK(gw->numel() == C && gb->numel() == C, "ghost_bn_bwd: grad shapes");
  }
  // grouped (per-client) dweight / dbias: [G, C] fp32 rows of any row stride
  // (views of the client-major grouped gradient buffer, parallel/grouped.py)
  const bool grouped = affine && ggw.has_value() && ggw->defined() && ggb.has_value() && ggb->defined();
  if (grouped) {
    TORCH_CHECK(!into, "ghost_bn_bwd: flat and grouped gradients are exclusive");
    for (const auto* t : {&*ggw, &*ggb}) {
      TORCH_CHECK(t->scalar_type() == at::kFloat && t->dim() == 2 && t->size(0) == G && t->size(1) == C &&
                      t->stride(1) == 1 && t->stride(0) == ggw->stride(0) && t->device() == x.device(),
                  "ghost_bn_bwd: grouped grads must be f32 [G, C] rows of one stride");
    }
  }
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  const int S = bn_slabs(static_cast<int>(G), static_cast<int>(M));
  auto fo = x.options().dtype(at::kFloat);
  auto part = at::empty({bn_scratch_floats(static_cast<int>(G), static_cast<int>(M), static_cast<int>(C))}, fo);
  auto coef = at::empty({G * 3 * C}, fo);
  at::Tensor dw, db;
  if (affine && !into && !grouped) {
    dw = at::empty({C}, fo);
    db = at::empty({C}, fo);
  }
  float* dwp = into ? gw->data_ptr<float>() : (affine && !grouped ? dw.data_ptr<float>() : nullptr);
  float* dbp = into ? gb->data_ptr<float>() : (affine && !grouped ? db.data_ptr<float>() : nullptr);
  auto dx = at::empty_like(x, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  launch_bn_bwd(bf16_ptr(x), bf16_ptr(dy), fused_relu ? y_relu->data_ptr<uint8_t>() : nullptr, stat.data_ptr<float>(),
                affine ? w->data_ptr<float>() : nullptr, static_cast<int>(G), static_cast<int>(M),
                static_cast<int>(C), part.data_ptr<float>(), coef.data_ptr<float>(), dwp, dbp,
                into ? 1.f : 0.f, reinterpret_cast<uint16_t*>(dx.data_ptr()), cur_stream(),
                grouped ? ggw->data_ptr<float>() : nullptr, grouped ? ggb->data_ptr<float>() : nullptr,
                grouped ? ggw->stride(0) : 0,
                (dadd.has_value() && dadd->defined()) ? reinterpret_cast<uint16_t*>(dadd->data_ptr())
                                                      : nullptr);
  return {dx, dw, db};
}

// per-client mean metrics into out [m, W] (f32, contiguous): see loss.hip
void client_means_hip(at::Tensor out, at::TensorList rows, const at::Tensor& slot,
                      const at::Tensor& counts) {
  const int64_t m = static_cast<int64_t>(rows.size());
  TORCH_CHECK(m >= 1 && m <= kClientMeanRows, "client_means: 1..4 metric rows");
  TORCH_CHECK(out.scalar_type() == at::kFloat && out.is_contiguous() && out.dim() == 2 && out.size(0) == m,
              "client_means: out f32 [m, W]");
  const int64_t W = out.size(1), n = slot.numel();
  TORCH_CHECK(slot.scalar_type() == at::kLong && slot.is_contiguous(), "client_means: slot int64");
  TORCH_CHECK(counts.numel() == W && counts.is_contiguous() &&
                  (counts.scalar_type() == at::kLong || counts.scalar_type() == at::kFloat),
              "client_means: counts int64/f32 [W]");
  ClientMeanRows r{};
  r.m = static_cast<int>(m);
  for (int64_t i = 0; i < m; ++i) {
    TORCH_CHECK(rows[i].scalar_type() == at::kFloat && rows[i].is_contiguous() && rows[i].numel() == n,
                "client_means: rows f32 [n]");
    r.p[i] = rows[i].data_ptr<float>();
  }
  for (int64_t i = m; i < kClientMeanRows; ++i) r.p[i] = r.p[0];
  c10::hip::HIPGuardMasqueradingAsCUDA guard(out.device());
  launch_client_means(r, slot.data_ptr<int64_t>(), static_cast<int>(n), counts.data_ptr(),
                      counts.scalar_type() == at::kFloat, static_cast<int>(W), out.data_ptr<float>(),
                      cur_stream());
}

// fused per-example cross-entropy: (loss f32 [B], correct f32 [B], softmax - onehot [B, C]);
// logits may be rows of a wider buffer (unit column stride, row stride >= C: the
// tied LM head's padded logits), the gradient then has the same row stride
std::tuple<at::Tensor, at::Tensor, at::Tensor> ce_fwd_hip(const at::Tensor& logits,
                                                          const at::Tensor& targets) {
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1 && logits.stride(0) >= logits.size(1) &&
                  (logits.scalar_type() == at::kBFloat16 || logits.scalar_type() == at::kFloat),
              "ce_fwd: logits must be bf16/f32 [B, C] rows with unit column stride");
  TORCH_CHECK(targets.scalar_type() == at::kLong && targets.is_contiguous() &&
                  targets.numel() == logits.size(0),
              "ce_fwd: targets must be contiguous int64 [B]");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(logits.device());
  const int64_t B = logits.size(0), C = logits.size(1), ld = B > 1 ? logits.stride(0) : C;
  auto loss = at::empty({B}, logits.options().dtype(at::kFloat));
  auto correct = at::empty({B}, logits.options().dtype(at::kFloat));
  auto grad = at::empty({B, ld}, logits.options()).narrow(1, 0, C);
  launch_ce_fwd(logits.data_ptr(), logits.scalar_type() == at::kBFloat16,
                targets.data_ptr<int64_t>(), B, static_cast<int>(C), ld,
                loss.data_ptr<float>(), correct.data_ptr<float>(), grad.data_ptr(), cur_stream());
  return {loss, correct, grad};
}

// g [B, C] (bf16 / f32, unit column stride) *= s [B] row by row, in place
void scale_rows_hip(at::Tensor g, const at::Tensor& s) {
  TORCH_CHECK(g.dim() == 2 && g.stride(1) == 1 && g.stride(0) >= g.size(1) &&
                  (g.scalar_type() == at::kBFloat16 || g.scalar_type() == at::kFloat),
              "scale_rows: g must be bf16/f32 [B, C] rows with unit column stride");
  TORCH_CHECK(s.scalar_type() == at::kFloat && s.is_contiguous() && s.numel() == g.size(0) &&
                  s.device() == g.device(),
              "scale_rows: s must be contiguous f32 [B]");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(g.device());
  const int64_t ld = g.size(0) > 1 ? g.stride(0) : g.size(1);
  launch_scale_rows(g.data_ptr(), g.scalar_type() == at::kBFloat16, s.data_ptr<float>(), g.size(0),
                    static_cast<int>(g.size(1)), ld, cur_stream());
}

// residual unit tail: out = relu(conv3x3(x, w)) + addend, and pre = relu(conv3x3(x, w))
std::tuple<at::Tensor, at::Tensor> conv3x3_relu_add_hip(const at::Tensor& x, const at::Tensor& w,
                                                        const at::Tensor& addend) {
  at::Tensor pre;
  auto out = conv3x3_fwd_impl(x, w, true, c10::nullopt, addend, &pre);
  return {out, pre};
}

// dw [K][C][3][3] fp32 = sum_p dy[p, k] x[p + (r-1, s-1), c]
void conv3x3_wgrad_run(const at::Tensor& dy, const at::Tensor& x, int64_t splits, at::Tensor& dw,
                       float beta);

at::Tensor conv3x3_wgrad_hip(const at::Tensor& dy, const at::Tensor& x, int64_t splits) {
  auto dw = at::empty({dy.size(1), x.size(1), 3, 3},
                      x.options().dtype(at::kFloat).memory_format(at::MemoryFormat::Contiguous));
  conv3x3_wgrad_run(dy, x, splits, dw, 0.f);
  return dw;
}

// dw += wgrad (accumulate straight into an existing fp32 gradient, e.g. a
// view of the flat gradient buffer: no separate AccumulateGrad pass)
void conv3x3_wgrad_into_hip(const at::Tensor& dy, const at::Tensor& x, at::Tensor dw,
                            int64_t splits) {
  check_f32(dw, "conv3x3_wgrad_into: dw");
  TORCH_CHECK(dw.dim() == 4 && dw.size(0) == dy.size(1) && dw.size(1) == x.size(1) &&
                  dw.size(2) == 3 && dw.size(3) == 3,
              "conv3x3_wgrad_into: dw must be [K, C, 3, 3]");
  conv3x3_wgrad_run(dy, x, splits, dw, 1.f);
}

// grouped (per-client) weight gradients: dw [G, K*C*9] fp32 rows (any row
// stride) += the wgrad of each of G equal pixel groups -- one GEMM launch for
// every group's split-K slabs and one per-group reduction (ops/grouped.py)
void conv3x3_wgrad_grouped_hip(const at::Tensor& dy, const at::Tensor& x, int64_t G, at::Tensor dw) {
  check_nhwc_bf16(dy, "conv3x3_wgrad_grouped: dy");
  check_nhwc_bf16(x, "conv3x3_wgrad_grouped: x");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3), K = dy.size(1);
  TORCH_CHECK(dy.size(0) == N && dy.size(2) == H && dy.size(3) == W, "conv3x3_wgrad_grouped: shapes");
  TORCH_CHECK(conv3x3_supported(static_cast<int>(C), static_cast<int>(K)) && K % 128 == 0,
              "conv3x3_wgrad_grouped: C % 64 and K % 128 must be 0");
  TORCH_CHECK(G >= 1 && N % G == 0, "conv3x3_wgrad_grouped: G must divide the batch");
  TORCH_CHECK(dw.scalar_type() == at::kFloat && dw.dim() == 2 && dw.size(0) == G &&
                  dw.size(1) == K * C * 9 && dw.stride(1) == 1 && dw.device() == x.device(),
              "conv3x3_wgrad_grouped: dw must be f32 [G, K*C*9] rows");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  const int P = static_cast<int>(N * H * W);
  const int Pg = P / static_cast<int>(G);
  const int total = conv3x3_wgrad_splits(P, static_cast<int>(H), static_cast<int>(W), static_cast<int>(K), static_cast<int>(C));
  int spg = static_cast<int>((total + G - 1) / G);
  const int steps_g = (Pg + 63) / 64;
  const int min_steps = 16;  // a split keeps >= 16 K-steps
  if (spg > steps_g / min_steps) spg = steps_g / min_steps;
  if (spg < 1) spg = 1;
  auto slab = at::empty({G * spg * K * 9 * C}, dw.options());
  ConvWgradArgs a;
  a.dy = bf16_ptr(dy);
  a.x = bf16_ptr(x);
  a.slab = slab.data_ptr<float>();
  a.P = P;
  a.H = static_cast<int>(H);
  a.W = static_cast<int>(W);
  a.C = static_cast<int>(C);
  a.K = static_cast<int>(K);
  a.splits = static_cast<int>(G) * spg;
  launch_conv3x3_wgrad_grouped(a, static_cast<int>(G), dw.data_ptr<float>(), dw.stride(0), 1.f,
                               cur_stream());
}

void conv3x3_wgrad_run(const at::Tensor& dy, const at::Tensor& x, int64_t splits, at::Tensor& dw,
                       float beta) {
  check_nhwc_bf16(dy, "conv3x3_wgrad: dy");
  check_nhwc_bf16(x, "conv3x3_wgrad: x");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3), K = dy.size(1);
  TORCH_CHECK(dy.size(0) == N && dy.size(2) == H && dy.size(3) == W, "conv3x3_wgrad: shapes");
  TORCH_CHECK(conv3x3_supported(static_cast<int>(C), static_cast<int>(K)) && K % 128 == 0,
              "conv3x3_wgrad: C % 64 and K % 128 must be 0");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  const int P = static_cast<int>(N * H * W);
  if (splits <= 0) splits = conv3x3_wgrad_splits(P, static_cast<int>(H), static_cast<int>(W), static_cast<int>(K), static_cast<int>(C));
  auto slab = at::empty({splits * K * 9 * C}, dw.options());
  ConvWgradArgs a;
  a.dy = bf16_ptr(dy);
  a.x = bf16_ptr(x);
  a.slab = slab.data_ptr<float>();
  a.P = P;
  a.H = static_cast<int>(H);
  a.W = static_cast<int>(W);
  a.C = static_cast<int>(C);
  a.K = static_cast<int>(K);
  a.splits = static_cast<int>(splits);
  launch_conv3x3_wgrad(a, dw.data_ptr<float>(), beta, cur_stream());
}

// w fp32 [K][C][3][3] -> (wf bf16 [K][3][3][C], wt bf16 [C][3][3][K] flipped)
std::vector<at::Tensor> conv_weight_prep_multi_hip(at::TensorList ws) {
  TORCH_CHECK(!ws.empty(), "conv_weight_prep: no weights");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(ws[0].device());
  std::vector<at::Tensor> out;
  ConvPrepBatch b{};
  b.n = 0;
  auto flush = [&]() {
    if (b.n > 0) launch_conv_weight_prep(b, cur_stream());
    b.n = 0;
  };
  for (const auto& w : ws) {
    check_f32(w, "conv_weight_prep: w");
    TORCH_CHECK(w.dim() == 4 && w.size(2) == 3 && w.size(3) == 3, "conv_weight_prep: [K, C, 3, 3]");
    TORCH_CHECK(w.device() == ws[0].device(), "conv_weight_prep: one device");
    const int64_t K = w.size(0), C = w.size(1);
    auto wf = at::empty({K, 3, 3, C}, w.options().dtype(at::kBFloat16));
    auto wt = at::empty({C, 3, 3, K}, w.options().dtype(at::kBFloat16));
    if (b.n == kPrepMax) flush();
    b.t[b.n++] = ConvPrepItem{w.data_ptr<float>(), reinterpret_cast<uint16_t*>(wf.data_ptr()),
                              reinterpret_cast<uint16_t*>(wt.data_ptr()), static_cast<int>(K),
                              static_cast<int>(C), 0};
    out.push_back(wf);
    out.push_back(wt);
  }
  flush();
  return out;
}

// images = [wf0, wt0, wf1, wt1, ...] of ``weights`` (views into w_flat)
void conv_images_patch_hip(const at::Tensor& w_flat, const at::Tensor& idx, at::TensorList weights,
                           at::TensorList images) {
  check_f32(w_flat, "conv_images_patch: w_flat");
  TORCH_CHECK(idx.scalar_type() == at::kLong && idx.dim() == 1 && idx.is_contiguous() &&
                  idx.device() == w_flat.device(), "conv_images_patch: idx must be int64 [k]");
  TORCH_CHECK(images.size() == 2 * weights.size() && weights.size() <= static_cast<size_t>(kPrepMax),
              "conv_images_patch: 2 images per weight, <= ", kPrepMax, " weights");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(w_flat.device());
  ConvPatchBatch b{};
  b.w_flat = w_flat.data_ptr<float>();
  b.n = 0;
  const int64_t d = w_flat.numel();
  for (size_t j = 0; j < weights.size(); ++j) {
    const auto& w = weights[j];
    TORCH_CHECK(w.scalar_type() == at::kFloat && w.dim() == 4 && w.size(2) == 3 && w.size(3) == 3 &&
                    w.is_contiguous(), "conv_images_patch: weights must be contiguous f32 [K, C, 3, 3]");
    const int64_t off = (reinterpret_cast<const char*>(w.data_ptr()) -
                         reinterpret_cast<const char*>(w_flat.data_ptr())) / 4;
    TORCH_CHECK(off >= 0 && off + w.numel() <= d, "conv_images_patch: weight is not a view of w_flat");
    const int64_t K = w.size(0), C = w.size(1);
    const auto& wf = images[2 * j];
    const auto& wt = images[2 * j + 1];
    TORCH_CHECK(wf.scalar_type() == at::kBFloat16 && wt.scalar_type() == at::kBFloat16 &&
                    wf.is_contiguous() && wt.is_contiguous() && wf.numel() == w.numel() &&
                    wt.numel() == w.numel(), "conv_images_patch: images must be contiguous bf16");
    b.off[b.n] = off;
    b.numel[b.n] = w.numel();
    b.wf[b.n] = reinterpret_cast<uint16_t*>(wf.data_ptr());
    b.wt[b.n] = reinterpret_cast<uint16_t*>(wt.data_ptr());
    b.K[b.n] = static_cast<int>(K);
    b.C[b.n] = static_cast<int>(C);
    ++b.n;
  }
  launch_conv_images_patch(b, idx.data_ptr<int64_t>(), idx.numel(), cur_stream());
}

std::tuple<at::Tensor, at::Tensor> conv_weight_prep_hip(const at::Tensor& w) {
  auto r = conv_weight_prep_multi_hip({w});
  return {r[0], r[1]};
}

// ---- ResNet-9 input conv (conv_prep.hip)
// x: [B, 3, H, W] bf16 view of a 4-channel-stride pixel buffer (the layout the
// augmentation kernel writes)
void check_prep_input(const at::Tensor& x) {
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && x.dim() == 4 && x.size(1) == 3,
              "conv_prep: x must be bf16 [B, 3, H, W]");
  const int64_t H = x.size(2), W = x.size(3);
  TORCH_CHECK(x.stride(1) == 1 && x.stride(3) == 4 && x.stride(2) == 4 * W && x.stride(0) == 4 * H * W,
              "conv_prep: x must have a 4-channel pixel stride (augment_u8_nhwc layout)");
  TORCH_CHECK(x.storage_offset() + x.size(0) * H * W * 4 <= static_cast<int64_t>(x.storage().nbytes() / 2),
              "conv_prep: x storage too small");
  TORCH_CHECK(x.size(0) * H * W < (int64_t(1) << 31), "conv_prep: 32-bit pixel index");
}

ConvPrepArgs prep_args(const at::Tensor& x) {
  ConvPrepArgs a{};
  a.x = reinterpret_cast<const uint16_t*>(x.data_ptr());
  a.P = static_cast<int>(x.size(0) * x.size(2) * x.size(3));
  a.H = static_cast<int>(x.size(2));
  a.W = static_cast<int>(x.size(3));
  a.Cin = static_cast<int>(x.size(1));
  return a;
}

std::tuple<at::Tensor, at::Tensor> conv_prep_fwd_hip(const at::Tensor& x, const at::Tensor& w) {
  check_prep_input(x);
  check_f32(w, "conv_prep: w");
  TORCH_CHECK(w.dim() == 4 && w.size(0) == 64 && w.size(1) == x.size(1) && w.size(2) == 3 &&
                  w.size(3) == 3, "conv_prep: w must be [64, 3, 3, 3]");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  const int64_t B = x.size(0), H = x.size(2), W = x.size(3);
  auto y = at::empty({B, 64, H, W}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto mask = at::empty({B * H * W, 2}, x.options().dtype(at::kInt));
  ConvPrepArgs a = prep_args(x);
  a.w = w.data_ptr<float>();
  a.y = reinterpret_cast<uint16_t*>(y.data_ptr());
  a.mask = reinterpret_cast<uint32_t*>(mask.data_ptr());
  launch_conv_prep_fwd(a, cur_stream());
  return {y, mask};
}

void conv_prep_wgrad_run(const at::Tensor& gy_in, const at::Tensor& mask, const at::Tensor& x,
                         at::Tensor& dw, float beta) {
  check_prep_input(x);
  auto gy = gy_in.to(at::kBFloat16).contiguous(at::MemoryFormat::ChannelsLast);
  const int64_t B = x.size(0), H = x.size(2), W = x.size(3);
  TORCH_CHECK(gy.dim() == 4 && gy.size(0) == B && gy.size(1) == 64 && gy.size(2) == H && gy.size(3) == W,
              "conv_prep_wgrad: gy shape");
  TORCH_CHECK(mask.scalar_type() == at::kInt && mask.is_contiguous() && mask.numel() == B * H * W * 2,
              "conv_prep_wgrad: mask");
  check_f32(dw, "conv_prep_wgrad: dw");
  TORCH_CHECK(dw.numel() == 64 * x.size(1) * 9, "conv_prep_wgrad: dw shape");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  ConvPrepArgs a = prep_args(x);
  auto partial = at::empty({conv_prep_wgrad_blocks(a.P), 64 * 64}, x.options().dtype(at::kFloat));
  a.gy = reinterpret_cast<const uint16_t*>(gy.data_ptr());
  a.mask_in = reinterpret_cast<const uint32_t*>(mask.data_ptr());
  a.partial = partial.data_ptr<float>();
  launch_conv_prep_wgrad(a, dw.data_ptr<float>(), beta, cur_stream());
}

at::Tensor conv_prep_wgrad_hip(const at::Tensor& gy, const at::Tensor& mask, const at::Tensor& x) {
  auto dw = at::empty({64, x.size(1), 3, 3}, x.options().dtype(at::kFloat));
  conv_prep_wgrad_run(gy, mask, x, dw, 0.f);
  return dw;
}

void conv_prep_wgrad_into_hip(const at::Tensor& gy, const at::Tensor& mask, const at::Tensor& x,
                              at::Tensor dw) {
  conv_prep_wgrad_run(gy, mask, x, dw, 1.f);
}

at::Tensor relu_mask_hip(const at::Tensor& gy, const at::Tensor& y) {
  check_nhwc_bf16(y, "relu_mask: y");
  auto g = gy.contiguous(at::MemoryFormat::ChannelsLast);
  check_nhwc_bf16(g, "relu_mask: gy");
  TORCH_CHECK(g.sizes() == y.sizes() && y.numel() % 8 == 0, "relu_mask: shapes");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(y.device());
  auto out = at::empty_like(g, g.options().memory_format(at::MemoryFormat::ChannelsLast));
  launch_relu_mask(bf16_ptr(g), bf16_ptr(y), reinterpret_cast<uint16_t*>(out.data_ptr()), y.numel(),
                   cur_stream());
  return out;
}

// One-time layout of the binned encode for a sketch geometry (hashes are
// data-independent): counts[chunk, tile], base[chunk, tile] (global entry
// index of the chunk's run in the tile's segment), seg[tile] (segment starts,
// num_tiles + 1).  All int32 on the device of `like`.
std::tuple<at::Tensor, at::Tensor, at::Tensor> cs_layout_hip(
    const at::Tensor& hashes, const at::Tensor& blk_off, const at::Tensor& blk_sign,
    int64_t num_blocks, int64_t d, int64_t c, const at::Tensor& like) {
  c10::hip::HIPGuardMasqueradingAsCUDA guard(like.device());
  auto ctx = make_ctx(hashes, blk_off, blk_sign, num_blocks, d, c, true);
  BinPlan plan = plan_cs_encode_binned(ctx.geom);
  TORCH_CHECK(cs_binned_supported(plan), "sketch geometry too large for the binned encode");
  auto opt = like.options().dtype(at::kInt);
  auto counts = at::empty({plan.num_chunks, plan.num_tiles}, opt);
  launch_cs_layout(ctx.rows, ctx.geom, ctx.blk_off, ctx.blk_sign, plan,
                   reinterpret_cast<uint32_t*>(counts.data_ptr<int32_t>()), cur_stream());
  auto c64 = counts.to(at::kLong);
  auto tile_tot = c64.sum(0);
  auto seg = at::cat({at::zeros({1}, tile_tot.options()), at::cumsum(tile_tot, 0)});
  auto base = at::cumsum(c64, 0) - c64 + seg.narrow(0, 0, plan.num_tiles).unsqueeze(0);
  return {counts, base.to(at::kInt).contiguous(), seg.to(at::kInt).contiguous()};
}

int64_t binned_scratch_bytes(int64_t d, int64_t r, int64_t c, int64_t num_blocks) {
  SketchGeom g = make_geom(static_cast<uint32_t>(d), static_cast<uint32_t>(r),
                           static_cast<uint32_t>(c), static_cast<uint32_t>(num_blocks));
  return cs_encode_binned_scratch_bytes(plan_cs_encode_binned(g));
}

// ------------------------------------------------- GPT-2 block junctions --
void check_rows_bf16(const at::Tensor& t, int64_t M, int64_t H, const char* name) {
  TORCH_CHECK(t.scalar_type() == at::kBFloat16 && t.is_contiguous() && t.dim() == 2 &&
                  t.size(0) == M && t.size(1) == H,
              name, " must be contiguous bf16 [", M, ", ", H, "]");
}

void check_vec_bf16(const at::Tensor& t, int64_t H, const char* name) {
  TORCH_CHECK(t.scalar_type() == at::kBFloat16 && t.is_contiguous() && t.numel() == H, name,
              " must be contiguous bf16 [", H, "]");
}

const void* opt_ptr(const c10::optional<at::Tensor>& t) {
  return t.has_value() && t->defined() ? t->data_ptr() : nullptr;
}

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> resid_ln_fwd_hip(
    const at::Tensor& x, const c10::optional<at::Tensor>& p, const c10::optional<at::Tensor>& bias,
    const at::Tensor& gamma, const at::Tensor& beta, double p_drop, int64_t seed, double eps,
    bool want_h) {
  TORCH_CHECK(x.dim() == 2, "resid_ln_fwd: x must be [M, H]");
  const int64_t M = x.size(0), H = x.size(1);
  TORCH_CHECK(resid_ln_supported(H), "resid_ln_fwd: H must be 256*V, V in 1..6 (got ", H, ")");
  check_rows_bf16(x, M, H, "resid_ln_fwd: x");
  if (p.has_value() && p->defined()) check_rows_bf16(*p, M, H, "resid_ln_fwd: p");
  if (bias.has_value() && bias->defined()) check_vec_bf16(*bias, H, "resid_ln_fwd: bias");
  check_vec_bf16(gamma, H, "resid_ln_fwd: gamma");
  check_vec_bf16(beta, H, "resid_ln_fwd: beta");
  TORCH_CHECK(p_drop >= 0.0 && p_drop < 1.0, "resid_ln_fwd: p_drop must be in [0, 1)");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  auto h = want_h ? at::empty_like(x) : at::empty({0}, x.options());
  auto y = at::empty_like(x);
  auto f = x.options().dtype(at::kFloat);
  auto mean = at::empty({M}, f), rstd = at::empty({M}, f);
  launch_resid_ln_fwd(x.data_ptr(), opt_ptr(p), opt_ptr(bias), gamma.data_ptr(), beta.data_ptr(),
                      want_h ? h.data_ptr() : nullptr, y.data_ptr(), mean.data_ptr<float>(),
                      rstd.data_ptr<float>(), M, H, static_cast<float>(p_drop),
                      static_cast<uint32_t>(seed), static_cast<float>(eps), cur_stream());
  return {h, y, mean, rstd};
}

// an optional fp32 gradient sink: out += colsum (mode 2) instead of a new bf16 tensor
void* sink_ptr(const c10::optional<at::Tensor>& sink, int64_t n, const char* name) {
  if (!sink.has_value() || !sink->defined()) return nullptr;
  TORCH_CHECK(sink->scalar_type() == at::kFloat && sink->is_contiguous() && sink->numel() == n,
              name, " sink must be contiguous float32 [", n, "]");
  return sink->data_ptr();
}

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor> resid_ln_bwd_hip(
    const at::Tensor& gy, const c10::optional<at::Tensor>& gh, const at::Tensor& h,
    const at::Tensor& mean, const at::Tensor& rstd, const at::Tensor& gamma, double p_drop,
    int64_t seed, bool want_dp, bool want_dbias, const c10::optional<at::Tensor>& sgamma,
    const c10::optional<at::Tensor>& sbeta, const c10::optional<at::Tensor>& sbias) {
  TORCH_CHECK(h.dim() == 2, "resid_ln_bwd: h must be [M, H]");
  const int64_t M = h.size(0), H = h.size(1);
  TORCH_CHECK(resid_ln_supported(H), "resid_ln_bwd: unsupported H ", H);
  check_rows_bf16(h, M, H, "resid_ln_bwd: h");
  check_rows_bf16(gy, M, H, "resid_ln_bwd: gy");
  if (gh.has_value() && gh->defined()) check_rows_bf16(*gh, M, H, "resid_ln_bwd: gh");
  check_vec_bf16(gamma, H, "resid_ln_bwd: gamma");
  TORCH_CHECK(mean.scalar_type() == at::kFloat && mean.numel() == M && rstd.numel() == M &&
                  rstd.scalar_type() == at::kFloat,
              "resid_ln_bwd: mean/rstd must be float32 [M]");
  TORCH_CHECK(want_dp || !want_dbias, "resid_ln_bwd: dbias needs dp");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(h.device());
  void* pg = sink_ptr(sgamma, H, "resid_ln_bwd: gamma");
  void* pb = sink_ptr(sbeta, H, "resid_ln_bwd: beta");
  void* pc = want_dbias ? sink_ptr(sbias, H, "resid_ln_bwd: bias") : nullptr;
  auto empty = at::empty({0}, gamma.options());
  auto dh = at::empty_like(h);
  auto dp = want_dp ? at::empty_like(h) : at::empty({0}, h.options());
  auto dgamma = pg ? empty : at::empty({H}, gamma.options());
  auto dbeta = pb ? empty : at::empty({H}, gamma.options());
  auto dbias = (want_dbias && !pc) ? at::empty({H}, gamma.options()) : empty;
  const int G = resid_ln_bwd_blocks(M);
  auto part = at::empty({G, 3, H}, h.options().dtype(at::kFloat));
  launch_resid_ln_bwd(gy.data_ptr(), opt_ptr(gh), h.data_ptr(), mean.data_ptr<float>(),
                      rstd.data_ptr<float>(), gamma.data_ptr(), dh.data_ptr(),
                      want_dp ? dp.data_ptr() : nullptr, part.data_ptr<float>(), M, H,
                      static_cast<float>(p_drop), static_cast<uint32_t>(seed), cur_stream());
  ColsumOut out{{pg ? pg : dgamma.data_ptr(), pb ? pb : dbeta.data_ptr(),
                 want_dbias ? (pc ? pc : dbias.data_ptr()) : nullptr},
                {pg ? 2 : 0, pb ? 2 : 0, pc ? 2 : 0}};
  launch_colsum_final(part.data_ptr<float>(), G, want_dbias ? 3 : 2, H, 3 * H, out, cur_stream());
  return {dh, dp, dgamma, dbeta, dbias};
}

at::Tensor bias_gelu_fwd_hip(const at::Tensor& u, const at::Tensor& b) {
  TORCH_CHECK(u.dim() == 2 && u.size(1) % 8 == 0, "bias_gelu_fwd: u must be [M, N], N % 8 == 0");
  check_rows_bf16(u, u.size(0), u.size(1), "bias_gelu_fwd: u");
  check_vec_bf16(b, u.size(1), "bias_gelu_fwd: b");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(u.device());
  auto f = at::empty_like(u);
  launch_bias_gelu_fwd(u.data_ptr(), b.data_ptr(), f.data_ptr(), u.size(0), u.size(1), cur_stream());
  return f;
}

std::tuple<at::Tensor, at::Tensor> bias_act_bwd_hip(const at::Tensor& gf,
                                                    const c10::optional<at::Tensor>& u,
                                                    const at::Tensor& b, bool gelu,
                                                    const c10::optional<at::Tensor>& sbias) {
  TORCH_CHECK(gf.dim() == 2 && gf.size(1) % 8 == 0 && gf.size(1) / 8 <= 1024,
              "bias_act_bwd: gf must be [M, N], N % 8 == 0, N <= 8192");
  const int64_t M = gf.size(0), N = gf.size(1);
  check_rows_bf16(gf, M, N, "bias_act_bwd: gf");
  check_vec_bf16(b, N, "bias_act_bwd: b");
  if (gelu) {
    TORCH_CHECK(u.has_value() && u->defined(), "bias_act_bwd: gelu needs u");
    check_rows_bf16(*u, M, N, "bias_act_bwd: u");
  }
  c10::hip::HIPGuardMasqueradingAsCUDA guard(gf.device());
  void* ps = sink_ptr(sbias, N, "bias_act_bwd: bias");
  auto du = gelu ? at::empty_like(gf) : at::empty({0}, gf.options());
  auto db = ps ? at::empty({0}, b.options()) : at::empty({N}, b.options());
  if (M == 0) {
    if (!ps) db.zero_();
    return {du, db};
  }
  const int G = bias_act_bwd_blocks(M);
  auto part = at::empty({G, N}, gf.options().dtype(at::kFloat));
  launch_bias_act_bwd(gf.data_ptr(), gelu ? u->data_ptr() : nullptr, b.data_ptr(),
                      gelu ? du.data_ptr() : nullptr, part.data_ptr<float>(), M, N, gelu,
                      cur_stream());
  ColsumOut out{{ps ? ps : db.data_ptr(), nullptr, nullptr}, {ps ? 2 : 0, 0, 0}};
  launch_colsum_final(part.data_ptr<float>(), G, 1, N, N, out, cur_stream());
  return {du, db};
}

// The same backward passes with the column sums deferred: they return the
// block partials instead, and colsum_into reduces them into fp32 gradient
// sinks later -- on the weight-gradient side stream (ops/transformer.py), so
// the ~40 us of latency-bound column sums per junction leave the input-
// gradient critical path
std::tuple<at::Tensor, at::Tensor, at::Tensor> resid_ln_bwd_part_hip(
    const at::Tensor& gy, const c10::optional<at::Tensor>& gh, const at::Tensor& h,
    const at::Tensor& mean, const at::Tensor& rstd, const at::Tensor& gamma, double p_drop,
    int64_t seed, bool want_dp) {
  TORCH_CHECK(h.dim() == 2, "resid_ln_bwd_part: h must be [M, H]");
  const int64_t M = h.size(0), H = h.size(1);
  TORCH_CHECK(resid_ln_supported(H), "resid_ln_bwd_part: unsupported H ", H);
  check_rows_bf16(h, M, H, "resid_ln_bwd_part: h");
  check_rows_bf16(gy, M, H, "resid_ln_bwd_part: gy");
  if (gh.has_value() && gh->defined()) check_rows_bf16(*gh, M, H, "resid_ln_bwd_part: gh");
  check_vec_bf16(gamma, H, "resid_ln_bwd_part: gamma");
  TORCH_CHECK(mean.scalar_type() == at::kFloat && mean.numel() == M && rstd.numel() == M &&
                  rstd.scalar_type() == at::kFloat,
              "resid_ln_bwd_part: mean/rstd must be float32 [M]");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(h.device());
  auto dh = at::empty_like(h);
  auto dp = want_dp ? at::empty_like(h) : at::empty({0}, h.options());
  const int G = resid_ln_bwd_blocks(M);
  auto part = at::empty({G, 3, H}, h.options().dtype(at::kFloat));
  launch_resid_ln_bwd(gy.data_ptr(), opt_ptr(gh), h.data_ptr(), mean.data_ptr<float>(),
                      rstd.data_ptr<float>(), gamma.data_ptr(), dh.data_ptr(),
                      want_dp ? dp.data_ptr() : nullptr, part.data_ptr<float>(), M, H,
                      static_cast<float>(p_drop), static_cast<uint32_t>(seed), cur_stream());
  return {dh, dp, part};
}

std::tuple<at::Tensor, at::Tensor> bias_act_bwd_part_hip(const at::Tensor& gf,
                                                         const c10::optional<at::Tensor>& u,
                                                         const at::Tensor& b, bool gelu) {
  TORCH_CHECK(gf.dim() == 2 && gf.size(1) % 8 == 0 && gf.size(1) / 8 <= 1024,
              "bias_act_bwd_part: gf must be [M, N], N % 8 == 0, N <= 8192");
  const int64_t M = gf.size(0), N = gf.size(1);
  TORCH_CHECK(M > 0, "bias_act_bwd_part: no rows");
  check_rows_bf16(gf, M, N, "bias_act_bwd_part: gf");
  check_vec_bf16(b, N, "bias_act_bwd_part: b");
  if (gelu) {
    TORCH_CHECK(u.has_value() && u->defined(), "bias_act_bwd_part: gelu needs u");
    check_rows_bf16(*u, M, N, "bias_act_bwd_part: u");
  }
  c10::hip::HIPGuardMasqueradingAsCUDA guard(gf.device());
  auto du = gelu ? at::empty_like(gf) : at::empty({0}, gf.options());
  const int G = bias_act_bwd_blocks(M);
  auto part = at::empty({G, N}, gf.options().dtype(at::kFloat));
  launch_bias_act_bwd(gf.data_ptr(), gelu ? u->data_ptr() : nullptr, b.data_ptr(),
                      gelu ? du.data_ptr() : nullptr, part.data_ptr<float>(), M, N, gelu,
                      cur_stream());
  return {du, part};
}

// sink_q (fp32 [N]) += sum over the G blocks of part[g, q, :] (q < Q, part
// [G, Q*N] rows), fixed order (deterministic); a missing sink skips its q
void colsum_into_hip(const at::Tensor& part, int64_t Q, const c10::optional<at::Tensor>& s0,
                     const c10::optional<at::Tensor>& s1, const c10::optional<at::Tensor>& s2) {
  TORCH_CHECK(part.scalar_type() == at::kFloat && part.is_contiguous() && part.dim() >= 2 && Q >= 1 && Q <= 3 &&
                  part.numel() % (part.size(0) * Q) == 0,
              "colsum_into: part must be contiguous fp32 [G, Q, N]");
  const int64_t G = part.size(0), N = part.numel() / (G * Q);
  c10::hip::HIPGuardMasqueradingAsCUDA guard(part.device());
  void* p0 = sink_ptr(s0, N, "colsum_into: s0");
  void* p1 = Q > 1 ? sink_ptr(s1, N, "colsum_into: s1") : nullptr;
  void* p2 = Q > 2 ? sink_ptr(s2, N, "colsum_into: s2") : nullptr;
  ColsumOut out{{p0, p1, p2}, {2, 2, 2}};
  launch_colsum_final(part.data_ptr<float>(), static_cast<int>(G), static_cast<int>(Q), N, Q * N, out, cur_stream());
}

at::Tensor pad_rows_hip(const at::Tensor& src, const c10::optional<at::Tensor>& inv, int64_t rows) {
  TORCH_CHECK(src.scalar_type() == at::kBFloat16 && src.dim() == 2 && src.stride(1) == 1 &&
                  src.size(1) % 8 == 0 && src.stride(0) % 8 == 0 &&
                  reinterpret_cast<uintptr_t>(src.data_ptr()) % 16 == 0,
              "pad_rows: src must be bf16 [Mr, K] rows, K % 8 == 0, 16-byte aligned");
  const int32_t* ip = nullptr;
  if (inv.has_value() && inv->defined()) {
    TORCH_CHECK(inv->scalar_type() == at::kInt && inv->is_contiguous() && inv->numel() == rows,
                "pad_rows: inv must be int32 [rows]");
    ip = inv->data_ptr<int32_t>();
  } else {
    TORCH_CHECK(src.size(0) == rows, "pad_rows: without inv src must have `rows` rows");
  }
  c10::hip::HIPGuardMasqueradingAsCUDA guard(src.device());
  auto out = at::empty({rows, src.size(1)}, src.options());
  launch_pad_rows(src.data_ptr(), src.stride(0), src.size(1), ip, rows, out.data_ptr(), cur_stream());
  return out;
}

at::Tensor heads_to_rows_hip(at::TensorList srcs, const c10::optional<at::Tensor>& tok, int64_t Mr) {
  const int64_t P = static_cast<int64_t>(srcs.size());
  TORCH_CHECK(P >= 1 && P <= 3, "heads_to_rows: 1..3 sources");
  const auto& s0 = srcs[0];
  TORCH_CHECK(s0.dim() == 4, "heads_to_rows: sources must be [N, nh, L, hd]");
  const int64_t N = s0.size(0), nh = s0.size(1), L = s0.size(2), hd = s0.size(3);
  TORCH_CHECK(hd % 8 == 0, "heads_to_rows: head dim must be a multiple of 8");
  HeadSrcs hs{};
  for (int64_t p = 0; p < P; ++p) {
    const auto& s = srcs[p];
    TORCH_CHECK(s.scalar_type() == at::kBFloat16 && s.sizes() == s0.sizes() && s.stride(3) == 1 &&
                    s.stride(0) % 8 == 0 && s.stride(1) % 8 == 0 && s.stride(2) % 8 == 0 &&
                    reinterpret_cast<uintptr_t>(s.data_ptr()) % 16 == 0,
                "heads_to_rows: sources must be bf16 with 16-byte aligned head rows");
    hs.p[p] = s.data_ptr();
    hs.stride[p][0] = s.stride(0);
    hs.stride[p][1] = s.stride(1);
    hs.stride[p][2] = s.stride(2);
  }
  const int32_t* tp = nullptr;
  if (tok.has_value() && tok->defined()) {
    TORCH_CHECK(tok->scalar_type() == at::kInt && tok->is_contiguous() && tok->numel() == Mr,
                "heads_to_rows: tok must be int32 [Mr]");
    tp = tok->data_ptr<int32_t>();
  } else {
    TORCH_CHECK(Mr == N * L, "heads_to_rows: without tok Mr must be N*L");
  }
  c10::hip::HIPGuardMasqueradingAsCUDA guard(s0.device());
  auto out = at::empty({Mr, P * nh * hd}, s0.options());
  launch_heads_to_rows(hs, static_cast<int>(P), nh * hd, hd, L, tp, Mr, out.data_ptr(),
                       cur_stream());
  return out;
}

// sink_g (fp32 [M, N], row-contiguous) += a_g^T b_g for each of G groups of
// T rows: a [G T, M], b [G T, N] bf16 with unit column stride (gemm_tn.hip)
// slab_only: C is unused; returns the [G * splits, M, N] fp32 split products
// unsummed (a column-image weight gradient's parts, summed and permuted by
// wgrad_rsc_add)
// imp_R > 0: b is a channels-last bf16 image x [n, C, H, W] and the B operand
// its implicit imp_R x imp_R / imp_s / imp_pad column image [n OH OW, R R C]
// (gathered per tap in the kernel: GemmTnArgs::imp_*); each group whole images
static at::Tensor gemm_tn_run(float* sink, int64_t ldc, int64_t cg, const at::Tensor& a, const at::Tensor& b, int64_t G,
                       bool slab_only = false, int64_t imp_R = 0, int64_t imp_s = 1, int64_t imp_pad = 0) {
  const bool imp = imp_R > 0;
  int64_t OH = 0, OW = 0;
  if (imp) {
    TORCH_CHECK(b.scalar_type() == at::kBFloat16 && b.dim() == 4 && b.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                    b.size(1) % 8 == 0 && imp_s >= 1 && imp_pad >= 0 && imp_pad < imp_R,
                "gemm_tn_parts_imp: channels-last bf16 image with C % 8 == 0");
    OH = (b.size(2) + 2 * imp_pad - imp_R) / imp_s + 1;
    OW = (b.size(3) + 2 * imp_pad - imp_R) / imp_s + 1;
    TORCH_CHECK(a.dim() == 2 && a.size(0) == b.size(0) * OH * OW && G >= 1 && b.size(0) % G == 0,
                "gemm_tn_parts_imp: a [n OH OW, M], G | n");
  }
  TORCH_CHECK(a.scalar_type() == at::kBFloat16 && b.scalar_type() == at::kBFloat16 && a.dim() == 2 &&
                  (imp || (b.dim() == 2 && b.stride(1) == 1 && a.size(0) == b.size(0))) && a.stride(1) == 1,
              "gemm_tn_acc: a [T, M], b [T, N] bf16 with unit column stride");
  TORCH_CHECK(G >= 1 && a.size(0) % G == 0, "gemm_tn_acc: G must divide the rows");
  const int64_t M = a.size(1), N = imp ? imp_R * imp_R * b.size(1) : b.size(1), T = a.size(0) / G;
  const int64_t ldb = imp ? b.size(1) : b.stride(0);
  // M: a multiple of 64, or any M whose A rows hold the 8-column chunk past
  // M (a padded buffer: the tied LM head's 50,257-row weight gradient)
  const bool m_ok = M % 64 == 0 || a.stride(0) >= (M + 7) / 8 * 8;
  TORCH_CHECK(m_ok && N % 8 == 0 && a.stride(0) % 8 == 0 && ldb % 8 == 0 &&
                  reinterpret_cast<uintptr_t>(a.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(b.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(sink) % 16 == 0 && ldc % 4 == 0 && cg % 4 == 0,
              "gemm_tn_acc: M (or A's row stride) a multiple of 64, N of 8, 16-byte aligned rows");
  TORCH_CHECK(a.size(0) < (1ll << 31) && M * N < (1ll << 31), "gemm_tn_acc: size");
  if (T == 0) return at::Tensor();
  c10::hip::HIPGuardMasqueradingAsCUDA guard(a.device());
  static int cus = 0;
  if (cus == 0) {
    hipDeviceProp_t prop;
    int dev = 0;
    cus = 256;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
      cus = prop.multiProcessorCount;
  }
  GemmTnArgs g{};
  g.A = reinterpret_cast<const uint16_t*>(a.data_ptr());
  g.lda = a.stride(0);
  g.B = reinterpret_cast<const uint16_t*>(b.data_ptr());
  g.ldb = ldb;
  g.C = sink;
  g.ldc = ldc;
  g.M = static_cast<int>(M);
  g.N = static_cast<int>(N);
  g.T = static_cast<int>(T);
  g.G = static_cast<int>(G);
  g.cg = cg;
  if (imp) {
    g.sb = b.size(0) / G * b.size(2) * b.size(3) * ldb;  // a group's images
    g.imp_C = static_cast<int>(b.size(1));
    g.imp_H = static_cast<int>(b.size(2));
    g.imp_W = static_cast<int>(b.size(3));
    g.imp_OH = static_cast<int>(OH);
    g.imp_OW = static_cast<int>(OW);
    g.imp_R = static_cast<int>(imp_R);
    g.imp_s = static_cast<int>(imp_s);
    g.imp_pad = static_cast<int>(imp_pad);
  }
  // ~ one block per CU over all groups
  g.splits = gemm_tn_splits(g.M, g.N, g.T, cus / g.G > 0 ? cus / g.G : 1);
  g.slab_only = slab_only ? 1 : 0;
  at::Tensor slab;
  if (g.splits > 1 || slab_only) {
    slab = at::empty({G * g.splits, M, N}, a.options().dtype(at::kFloat));
    g.slab = slab.data_ptr<float>();
  }
  launch_gemm_tn_acc(g, cur_stream());
  return slab;
}

void gemm_tn_acc_hip(at::Tensor sink, const at::Tensor& a, const at::Tensor& b) {
  TORCH_CHECK(sink.scalar_type() == at::kFloat && sink.dim() == 2 && sink.stride(1) == 1 && sink.is_cuda(),
              "gemm_tn_acc: sink must be fp32 [M, N] with unit column stride");
  TORCH_CHECK(sink.size(0) == a.size(1) && sink.size(1) == b.size(1), "gemm_tn_acc: sink shape");
  gemm_tn_run(sink.data_ptr<float>(), sink.stride(0), 0, a, b, 1);
}

// grouped: sink [G, M, N] (unit column stride), a [G T, M], b [G T, N]
void gemm_tn_acc_grouped_hip(at::Tensor sink, const at::Tensor& a, const at::Tensor& b, int64_t G) {
  TORCH_CHECK(sink.scalar_type() == at::kFloat && sink.dim() == 3 && sink.stride(2) == 1 && sink.is_cuda(),
              "gemm_tn_acc_grouped: sink must be fp32 [G, M, N] with unit column stride");
  TORCH_CHECK(sink.size(0) == G && sink.size(1) == a.size(1) && sink.size(2) == b.size(1),
              "gemm_tn_acc_grouped: sink shape");
  gemm_tn_run(sink.data_ptr<float>(), sink.stride(1), sink.stride(0), a, b, G);
}

// (parts [G * S, M, N] fp32, S): the S split-K products of each group's
// a_g^T b_g, unsummed
std::tuple<at::Tensor, int64_t> gemm_tn_parts_hip(const at::Tensor& a, const at::Tensor& b, int64_t G) {
  TORCH_CHECK(a.is_cuda() && b.is_cuda(), "gemm_tn_parts: device tensors");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(a.device());
  // slab-only: the sink argument is never written (a's aligned address passes the checks)
  auto parts = gemm_tn_run(reinterpret_cast<float*>(a.data_ptr()), 4, 0, a, b, G, true);
  TORCH_CHECK(parts.defined(), "gemm_tn_parts: empty operands");
  return {parts, parts.size(0) / G};
}

// gemm_tn_parts with b the implicit R x R / stride / pad column image of the
// channels-last image x (a strided conv's weight gradient without im2col)
std::tuple<at::Tensor, int64_t> gemm_tn_parts_imp_hip(const at::Tensor& a, const at::Tensor& x, int64_t G, int64_t R,
                                                      int64_t stride, int64_t pad) {
  TORCH_CHECK(a.is_cuda() && x.is_cuda() && R >= 1, "gemm_tn_parts_imp: device tensors");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(a.device());
  auto parts = gemm_tn_run(reinterpret_cast<float*>(a.data_ptr()), 4, 0, a, x, G, true, R, stride, pad);
  TORCH_CHECK(parts.defined(), "gemm_tn_parts_imp: empty operands");
  return {parts, parts.size(0) / G};
}

void check_seqs(const at::Tensor& start, const at::Tensor& len) {
  TORCH_CHECK(start.scalar_type() == at::kInt && len.scalar_type() == at::kInt &&
                  start.is_contiguous() && len.is_contiguous() && start.numel() == len.numel(),
              "attn: start / len must be contiguous int32 [N]");
}

// LSE row stride for sequences of up to max_len tokens: 128 selects the
// all-in-LDS short kernels, longer sequences the flash-style kernels
int64_t attn_lse_ld(int64_t max_len) {
  TORCH_CHECK(max_len >= 0 && max_len <= 1024, "attn: sequences of up to 1024 tokens, got ", max_len);
  return max_len <= 128 ? 128 : (max_len + 127) / 128 * 128;
}

std::tuple<at::Tensor, at::Tensor> attn_fwd_hip(const at::Tensor& qkv, const at::Tensor& start,
                                                const at::Tensor& len, int64_t nh, double p_drop,
                                                int64_t seed, int64_t max_len) {
  TORCH_CHECK(qkv.scalar_type() == at::kBFloat16 && qkv.dim() == 2 && qkv.is_contiguous() &&
                  qkv.size(1) == 3 * nh * 64,
              "attn_fwd: qkv must be contiguous bf16 [M, 3 * nh * 64]");
  check_seqs(start, len);
  TORCH_CHECK(p_drop >= 0.0 && p_drop < 1.0, "attn_fwd: p_drop in [0, 1)");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(qkv.device());
  const int64_t M = qkv.size(0), N = start.numel(), H = nh * 64;
  auto o = at::empty({M, H}, qkv.options());
  const int64_t ld = attn_lse_ld(max_len);
  auto lse = at::empty({N * nh * ld}, qkv.options().dtype(at::kFloat));
  AttnArgs a{};
  a.lse_ld = static_cast<int>(ld);
  a.qkv = reinterpret_cast<const uint16_t*>(qkv.data_ptr());
  a.o = reinterpret_cast<uint16_t*>(o.data_ptr());
  a.lse = lse.data_ptr<float>();
  a.start = start.data_ptr<int32_t>();
  a.len = len.data_ptr<int32_t>();
  a.nh = static_cast<int>(nh);
  a.scale = 0.125f;  // 1 / sqrt(64)
  a.seed = static_cast<uint32_t>(seed);
  launch_attn_fwd(a, N, static_cast<float>(p_drop), cur_stream());
  return {o, lse};
}

at::Tensor attn_bwd_hip(const at::Tensor& qkv, const at::Tensor& o, const at::Tensor& dout,
                        const at::Tensor& lse, const at::Tensor& start, const at::Tensor& len,
                        int64_t nh, double p_drop, int64_t seed, int64_t max_len) {
  const int64_t H = nh * 64;
  TORCH_CHECK(qkv.scalar_type() == at::kBFloat16 && qkv.dim() == 2 && qkv.is_contiguous() &&
                  qkv.size(1) == 3 * H,
              "attn_bwd: qkv must be contiguous bf16 [M, 3H]");
  const int64_t M = qkv.size(0), N = start.numel();
  for (const at::Tensor* t : {&o, &dout})
    TORCH_CHECK(t->scalar_type() == at::kBFloat16 && t->is_contiguous() && t->dim() == 2 &&
                    t->size(0) == M && t->size(1) == H,
                "attn_bwd: o / dout must be contiguous bf16 [M, H]");
  const int64_t ld = attn_lse_ld(max_len);
  TORCH_CHECK(lse.scalar_type() == at::kFloat && lse.numel() == N * nh * ld, "attn_bwd: lse");
  check_seqs(start, len);
  c10::hip::HIPGuardMasqueradingAsCUDA guard(qkv.device());
  auto dqkv = at::empty_like(qkv);
  at::Tensor dbuf;
  AttnArgs a{};
  a.lse_ld = static_cast<int>(ld);
  if (ld > 128) {
    dbuf = at::empty({N * nh * ld}, lse.options());
    a.dbuf = dbuf.data_ptr<float>();
  }
  a.qkv = reinterpret_cast<const uint16_t*>(qkv.data_ptr());
  a.o = reinterpret_cast<uint16_t*>(o.data_ptr());
  a.lse = lse.data_ptr<float>();
  a.dout = reinterpret_cast<const uint16_t*>(dout.data_ptr());
  a.dqkv = reinterpret_cast<uint16_t*>(dqkv.data_ptr());
  a.start = start.data_ptr<int32_t>();
  a.len = len.data_ptr<int32_t>();
  a.nh = static_cast<int>(nh);
  a.scale = 0.125f;
  a.seed = static_cast<uint32_t>(seed);
  launch_attn_bwd(a, N, static_cast<float>(p_drop), cur_stream());
  return dqkv;
}

}  // namespace
}  // namespace commeff

TORCH_LIBRARY(commeff, m) {
  m.def("cs_encode(Tensor(a!) table, Tensor vec, Tensor hashes, Tensor blk_off, Tensor blk_sign, "
        "int num_blocks, float scale, Tensor? wvec, float wscale, Tensor[] layout) -> ()");
  m.def("cs_layout(Tensor hashes, Tensor blk_off, Tensor blk_sign, int num_blocks, int d, int c, "
        "Tensor like) -> (Tensor, Tensor, Tensor)");
  m.def("cs_hash_all(Tensor hashes, Tensor blk_off, Tensor blk_sign, int num_blocks, int d, int c, "
        "Tensor like) -> Tensor");
  m.def("cs_encode_planned(Tensor(a!) table, Tensor vec, float scale, Tensor? wvec, float wscale, "
        "int c, Tensor[] plan, bool overwrite=False) -> ()");
  m.def("cs_query_planned(Tensor table, int d, Tensor[] plan, int c0=0, int c1=-1) -> Tensor");
  m.def("plan_geometry(int d, int r, int c) -> int[]", &commeff::plan_geometry);
  m.def("relu_maxpool(Tensor x, int k) -> (Tensor, Tensor)");
  m.def("relu_maxpool_backward(Tensor gy, Tensor idx, int k) -> Tensor");
  m.def("conv3x3_fwd(Tensor x, Tensor w, bool relu, Tensor? mask=None, Tensor? addend=None) -> Tensor");
  m.def("conv3x3_fwd_unpool(Tensor x, Tensor w, Tensor? addend, Tensor idx) -> Tensor");
  m.def("conv3x3_fwd_dual(Tensor x, Tensor w, Tensor dual_mask) -> (Tensor, Tensor)");
  m.def("conv3x3_fwd_pool2(Tensor x, Tensor w) -> (Tensor, Tensor)");
  m.def("head_fwd(Tensor x, Tensor w, Tensor targets, float scale) -> (Tensor, Tensor, Tensor, Tensor, Tensor)");
  m.def("head_bwd(Tensor gl, Tensor gunit, Tensor w, Tensor pooled, Tensor codes, int H, int W, float scale, "
        "Tensor(a!) dw, float beta) -> Tensor");
  m.def("head_bwd_dual(Tensor gl, Tensor gunit, Tensor w, Tensor pooled, Tensor codes, int H, int W, "
        "float scale, Tensor(a!) dw, float beta, Tensor ymask) -> (Tensor, Tensor)");
  m.def("conv3x3_relu_add(Tensor x, Tensor w, Tensor addend) -> (Tensor, Tensor)");
  m.def("ce_fwd(Tensor logits, Tensor targets) -> (Tensor, Tensor, Tensor)");
  m.def("scale_rows(Tensor(a!) g, Tensor s) -> ()");
  m.def("client_means(Tensor(a!) out, Tensor[] rows, Tensor slot, Tensor counts) -> ()");
  m.def("ghost_bn_fwd(Tensor x, Tensor? w, Tensor? b, int G, float eps, float momentum, Tensor(a!)? run_mean, "
        "Tensor(b!)? run_var, bool relu=False, Tensor(c!)? num_batches_tracked=None, Tensor? addend=None, "
        "Tensor? tstats=None) -> (Tensor, Tensor, Tensor)");
  m.def("ghost_bn_bwd(Tensor dy, Tensor x, Tensor stat, Tensor? w, int G, Tensor? y_relu=None, "
        "Tensor(a!)? gw=None, Tensor(b!)? gb=None, Tensor(c!)? ggw=None, Tensor(d!)? ggb=None, "
        "Tensor(e!)? dadd=None) -> (Tensor, Tensor, Tensor)");
  m.def("conv3x3_wgrad(Tensor dy, Tensor x, int splits=0) -> Tensor");
  m.def("conv3x3_wgrad_into(Tensor dy, Tensor x, Tensor(a!) dw, int splits=0) -> ()");
  m.def("conv3x3_wgrad_auto_splits(int P, int H, int W, int K, int C) -> int",
        [](int64_t P, int64_t H, int64_t W, int64_t K, int64_t C) -> int64_t {
          return commeff::conv3x3_wgrad_splits(static_cast<int>(P), static_cast<int>(H), static_cast<int>(W),
                                               static_cast<int>(K), static_cast<int>(C));
        });
  m.def("conv3x3_fwd_grouped(Tensor x, Tensor w, int G) -> Tensor");
  m.def("conv3x3_wgrad_grouped_ch(Tensor dy, Tensor x, int G) -> Tensor");
  m.def("conv3x3_wgrad_grouped(Tensor dy, Tensor x, int G, Tensor(a!) dw) -> ()");
  m.def("conv_weight_prep(Tensor w) -> (Tensor, Tensor)");
  m.def("conv_weight_prep_multi(Tensor[] ws) -> Tensor[]");
  m.def("conv_images_patch(Tensor w_flat, Tensor idx, Tensor[] weights, Tensor[] images) -> ()");
  m.def("account_round(Tensor last_mod, Tensor meta, int T, int W, Tensor(a!) client_dl, "
        "Tensor(b!) client_ul, float upc) -> Tensor");
  m.def("conv_prep_fwd(Tensor x, Tensor w) -> (Tensor, Tensor)");
  m.def("conv_prep_wgrad(Tensor gy, Tensor mask, Tensor x) -> Tensor");
  m.def("conv_prep_wgrad_into(Tensor gy, Tensor mask, Tensor x, Tensor(a!) dw) -> ()");
  m.def("relu_mask(Tensor gy, Tensor y) -> Tensor");
  m.def("cs_query_rows(Tensor table, Tensor hashes, Tensor blk_off, Tensor blk_sign, int num_blocks, "
        "int d) -> Tensor");
  m.def("cs_query(Tensor table, Tensor hashes, Tensor blk_off, Tensor blk_sign, int num_blocks, "
        "int d) -> Tensor");
  m.def("cs_zero_buckets(Tensor(a!) t1, Tensor(b!)? t2, Tensor idx, Tensor? vals, Tensor hashes, "
        "Tensor blk_off, Tensor blk_sign, int num_blocks, int d) -> ()");
  m.def("cs_l2estimate(Tensor table) -> Tensor");
  m.def("cs_region_encode(Tensor(a!) table, Tensor(b!) vec, float scale, Tensor? wvec, float wscale, int m, "
        "int g, int W, Tensor perm, Tensor cinfo, Tensor lists, Tensor goffs, bool overwrite=False, "
        "bool zero_vec=False) -> ()");
  m.def("cs_region_query(Tensor table, int d, int m, int g, int W, Tensor perm, Tensor cinfo, Tensor lists, "
        "Tensor goffs, int q0=0, int q1=-1, int g0=0) -> Tensor");
  m.def("cs_region_topk(Tensor(a!) table, int d, int m, int g, int W, Tensor perm, Tensor cinfo, Tensor lists, "
        "Tensor goffs, int k, Tensor(d!)? hint=None, int q0=0, int q1=-1, Tensor(b!)? momV=None, Tensor? momG=None, "
        "float rho=0.0, float gscale=0.0, int mom_mode=0, Tensor(c!)? ws=None, int g0=0, Tensor? cpos=None, "
        "int ncoord=-1) -> (Tensor, Tensor)");
  m.def("cs_region_topk_ws_bytes(int d, int m, int q0, int q1) -> int", &commeff::cs_region_topk_ws_bytes);
  m.def("cs_region_zero(Tensor(a!) t1, Tensor(b!)? t2, Tensor idx, Tensor? vals, int d, int m, int g, "
        "Tensor perm, Tensor cinfo, int g0=0) -> ()");
  m.def("topk_abs(Tensor x, int k, Tensor(a!)? hint=None) -> (Tensor, Tensor)");
  m.def("momentum_ef(Tensor(a!) V, Tensor(b!)? E, Tensor G, float rho, float gscale, int mode) -> ()");
  m.def("sparse_apply(Tensor(a!) w, Tensor idx, Tensor vals, float lr, Tensor? lr_vec, "
        "Tensor(b!)? last_mod, int round, Tensor? step=None, Tensor(c!)? hist=None) -> ()");
  m.def("cs_region_zero_apply(Tensor(a!) t1, Tensor(b!)? t2, Tensor idx, Tensor vals, int d, int m, int g, "
        "Tensor perm, Tensor cinfo, Tensor(c!) w, float lr, Tensor? lr_vec, Tensor(d!)? last_mod, int round, "
        "Tensor(e!)? hist=None, Tensor? step=None, int g0=0) -> ()");
  m.def("dense_apply(Tensor(a!) w, Tensor delta, float lr, Tensor? lr_vec, Tensor(b!)? last_mod, "
        "int round, Tensor? step=None, Tensor(c!)? hist=None) -> ()");
  m.def("account_hist(Tensor hist, Tensor meta, int W, Tensor(a!) client_dl, Tensor(b!) client_ul, "
        "float upc) -> Tensor");
  m.def("count_ge(Tensor last_mod, Tensor thr) -> Tensor");
  m.def("axpby(Tensor(a!) out, Tensor a, float alpha, Tensor? b, float beta) -> ()");
  m.def("l2norm(Tensor x) -> Tensor");
  m.def("clip_noise(Tensor(a!) x, Tensor? norm, float clip, float noise_std, int seed, int offset) -> ()");
  m.def("client_state(Tensor g, Tensor(a!)? u, Tensor(b!)? e, float rho) -> ()");
  m.def("client_tail(Tensor(a!) g, Tensor? w, float wd, float scale, Tensor(b!)? u, Tensor(c!)? e, "
        "float rho) -> ()");
  m.def("zero_at(Tensor(a!)? a, Tensor(b!)? b, Tensor(c!)? c, Tensor idx) -> ()");
  m.def("scatter_dense(Tensor idx, Tensor vals, int n) -> Tensor");
  m.def("augment_u8_nhwc(Tensor data, Tensor idx, int pad, bool flip, Tensor mean, Tensor inv_std, "
        "int seed, bool out_bf16, Tensor? keys=None) -> Tensor");
  m.def("augment_u8_nhwc_y(Tensor data, Tensor idx, int pad, bool flip, Tensor mean, Tensor inv_std, "
        "int seed, bool out_bf16, Tensor? keys, Tensor targets) -> (Tensor, Tensor)");
  m.def("binned_scratch_bytes(int d, int r, int c, int num_blocks) -> int",
        &commeff::binned_scratch_bytes);
  m.def("resid_ln_fwd(Tensor x, Tensor? p, Tensor? bias, Tensor gamma, Tensor beta, float p_drop, "
        "int seed, float eps, bool want_h) -> (Tensor, Tensor, Tensor, Tensor)");
  m.def("resid_ln_bwd(Tensor gy, Tensor? gh, Tensor h, Tensor mean, Tensor rstd, Tensor gamma, "
        "float p_drop, int seed, bool want_dp, bool want_dbias, Tensor(a!)? sgamma=None, "
        "Tensor(b!)? sbeta=None, Tensor(c!)? sbias=None) "
        "-> (Tensor, Tensor, Tensor, Tensor, Tensor)");
  m.def("bias_gelu_fwd(Tensor u, Tensor b) -> Tensor");
  m.def("pad_rows(Tensor src, Tensor? inv, int rows) -> Tensor");
  m.def("attn_fwd(Tensor qkv, Tensor start, Tensor len, int nh, float p_drop, int seed, int max_len) -> (Tensor, Tensor)");
  m.def("attn_bwd(Tensor qkv, Tensor o, Tensor dout, Tensor lse, Tensor start, Tensor len, int nh, "
        "float p_drop, int seed, int max_len) -> Tensor");
  m.def("heads_to_rows(Tensor[] srcs, Tensor? tok, int Mr) -> Tensor");
  m.def("gemm_tn_acc(Tensor(a!) sink, Tensor a, Tensor b) -> ()");
  m.def("gemm_tn_acc_grouped(Tensor(a!) sink, Tensor a, Tensor b, int G) -> ()");
  m.def("gemm_tn_parts(Tensor a, Tensor b, int G) -> (Tensor, int)");
  m.def("gemm_tn_parts_imp(Tensor a, Tensor x, int G, int R, int stride, int pad) -> (Tensor, int)");
  m.def("im2col(Tensor x, int R, int S, int stride, int pad, int Kc) -> Tensor");
  m.def("col2im(Tensor gcol, int N, int H, int W, int C, int R, int S, int stride, int pad) -> Tensor");
  m.def("conv_weight_rsc(Tensor w, int Kc) -> Tensor");
  m.def("wgrad_rsc_add(Tensor(a!) dst, Tensor src, int splits, int C, int RS, bool accumulate) -> ()");
  m.def("maxpool_fwd(Tensor x, int k, int s, int p) -> (Tensor, Tensor)");
  m.def("maxpool_bwd(Tensor gy, Tensor codes, int H, int W, int k, int s, int p) -> Tensor");
  m.def("bias_act_bwd(Tensor gf, Tensor? u, Tensor b, bool gelu, Tensor(a!)? sbias=None) "
        "-> (Tensor, Tensor)");
  m.def("resid_ln_bwd_part(Tensor gy, Tensor? gh, Tensor h, Tensor mean, Tensor rstd, Tensor gamma, "
        "float p_drop, int seed, bool want_dp) -> (Tensor, Tensor, Tensor)");
  m.def("bias_act_bwd_part(Tensor gf, Tensor? u, Tensor b, bool gelu) -> (Tensor, Tensor)");
  m.def("colsum_into(Tensor part, int Q, Tensor(a!)? s0=None, Tensor(b!)? s1=None, Tensor(c!)? s2=None) -> ()");
}

TORCH_LIBRARY_IMPL(commeff, CPU, m) {
  using namespace commeff;
  m.impl("cs_encode", &cs_encode_cpu);
  m.impl("cs_query", &cs_query_cpu);
  m.impl("cs_zero_buckets", &cs_zero_buckets_cpu);
  m.impl("cs_l2estimate", &cs_l2estimate_cpu);
  m.impl("topk_abs", &topk_abs_cpu);
  m.impl("momentum_ef", &momentum_ef_cpu);
  m.impl("sparse_apply", &sparse_apply_cpu);
  m.impl("account_hist", &account_hist_cpu);
  m.impl("dense_apply", &dense_apply_cpu);
  m.impl("count_ge", &count_ge_cpu);
  m.impl("axpby", &axpby_cpu);
  m.impl("l2norm", &l2norm_cpu);
  m.impl("clip_noise", &clip_noise_cpu);
  m.impl("client_state", &client_state_cpu);
  m.impl("client_tail", &client_tail_cpu);
  m.impl("zero_at", &zero_at_cpu);
  m.impl("scatter_dense", &scatter_dense_cpu);
  m.impl("augment_u8_nhwc", &augment_cpu);
  m.impl("cs_hash_all", &cs_hash_all_cpu);
}

TORCH_LIBRARY_IMPL(commeff, CUDA, m) {
  using namespace commeff;
  m.impl("cs_encode", &cs_encode_hip);
  m.impl("cs_query", &cs_query_hip);
  m.impl("cs_query_rows", &cs_query_rows_hip);
  m.impl("cs_layout", &cs_layout_hip);
  m.impl("cs_hash_all", &cs_hash_all_hip);
  m.impl("cs_encode_planned", &cs_encode_planned_hip);
  m.impl("cs_query_planned", &cs_query_planned_hip);
  m.impl("relu_maxpool", &relu_maxpool_hip);
  m.impl("relu_maxpool_backward", &relu_maxpool_backward_hip);
  m.impl("conv3x3_fwd", &conv3x3_fwd_hip);
  m.impl("conv3x3_fwd_unpool", &conv3x3_fwd_unpool_hip);
  m.impl("conv3x3_fwd_dual", &conv3x3_fwd_dual_hip);
  m.impl("conv3x3_fwd_pool2", &conv3x3_fwd_pool2_hip);
  m.impl("head_fwd", &head_fwd_hip);
  m.impl("head_bwd", &head_bwd_hip);
  m.impl("head_bwd_dual", &head_bwd_dual_hip);
  m.impl("conv3x3_relu_add", &conv3x3_relu_add_hip);
  m.impl("ce_fwd", &ce_fwd_hip);
  m.impl("scale_rows", &scale_rows_hip);
  m.impl("client_means", &client_means_hip);
  m.impl("ghost_bn_fwd", &ghost_bn_fwd_hip);
  m.impl("ghost_bn_bwd", &ghost_bn_bwd_hip);
  m.impl("conv3x3_wgrad", &conv3x3_wgrad_hip);
  m.impl("conv3x3_wgrad_into", &conv3x3_wgrad_into_hip);
  m.impl("conv3x3_fwd_grouped", &conv3x3_fwd_grouped_hip);
  m.impl("conv3x3_wgrad_grouped_ch", &conv3x3_wgrad_grouped_ch_hip);
  m.impl("conv3x3_wgrad_grouped", &conv3x3_wgrad_grouped_hip);
  m.impl("conv_weight_prep", &conv_weight_prep_hip);
  m.impl("conv_weight_prep_multi", &conv_weight_prep_multi_hip);
  m.impl("conv_images_patch", &conv_images_patch_hip);
  m.impl("conv_prep_fwd", &conv_prep_fwd_hip);
  m.impl("conv_prep_wgrad", &conv_prep_wgrad_hip);
  m.impl("conv_prep_wgrad_into", &conv_prep_wgrad_into_hip);
  m.impl("relu_mask", &relu_mask_hip);
  m.impl("cs_zero_buckets", &cs_zero_buckets_hip);
  m.impl("cs_l2estimate", &cs_l2estimate_hip);
  m.impl("cs_region_encode", &cs_region_encode_hip);
  m.impl("cs_region_query", &cs_region_query_hip);
  m.impl("cs_region_zero", &cs_region_zero_hip);
  m.impl("cs_region_topk", &cs_region_topk_hip);
  m.impl("cs_region_zero_apply", &cs_region_zero_apply_hip);
  m.impl("topk_abs", &topk_abs_hip);
  m.impl("momentum_ef", &momentum_ef_hip);
  m.impl("sparse_apply", &sparse_apply_hip);
  m.impl("account_hist", &account_hist_hip);
  m.impl("dense_apply", &dense_apply_hip);
  m.impl("count_ge", &count_ge_hip);
  m.impl("account_round", &account_round_hip);
  m.impl("axpby", &axpby_hip);
  m.impl("l2norm", &l2norm_hip);
  m.impl("clip_noise", &clip_noise_hip);
  m.impl("client_state", &client_state_hip);
  m.impl("client_tail", &client_tail_hip);
  m.impl("zero_at", &zero_at_hip);
  m.impl("scatter_dense", &scatter_dense_hip);
  m.impl("augment_u8_nhwc", &augment_hip);
  m.impl("augment_u8_nhwc_y", &augment_y_hip);
  m.impl("resid_ln_fwd", &resid_ln_fwd_hip);
  m.impl("resid_ln_bwd", &resid_ln_bwd_hip);
  m.impl("bias_gelu_fwd", &bias_gelu_fwd_hip);
  m.impl("bias_act_bwd", &bias_act_bwd_hip);
  m.impl("resid_ln_bwd_part", &resid_ln_bwd_part_hip);
  m.impl("bias_act_bwd_part", &bias_act_bwd_part_hip);
  m.impl("colsum_into", &colsum_into_hip);
  m.impl("pad_rows", &pad_rows_hip);
  m.impl("gemm_tn_acc", &gemm_tn_acc_hip);
  m.impl("gemm_tn_acc_grouped", &gemm_tn_acc_grouped_hip);
  m.impl("gemm_tn_parts", &gemm_tn_parts_hip);
  m.impl("gemm_tn_parts_imp", &gemm_tn_parts_imp_hip);
  m.impl("attn_fwd", &attn_fwd_hip);
  m.impl("attn_bwd", &attn_bwd_hip);
  m.impl("heads_to_rows", &heads_to_rows_hip);
  m.impl("im2col", &im2col_hip);
  m.impl("col2im", &col2im_hip);
  m.impl("conv_weight_rsc", &conv_weight_rsc_hip);
  m.impl("wgrad_rsc_add", &wgrad_rsc_add_hip);
  m.impl("maxpool_fwd", &maxpool_fwd_hip);
  m.impl("maxpool_bwd", &maxpool_bwd_hip);
}
