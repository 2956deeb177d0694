// torch.ops.commeff registrations of the batched FedAvg engine
// (parallel/fedavg_native.py): grouped column images, channel-stacked batch
// norm, per-client weight images / gradient rows, the per-row SGD tail and the
// upload (csrc/fedavg.hip, csrc/im2col.hip, csrc/bn.hip, csrc/conv.hip).
// GPU only: the engine runs when the extension is loaded on a GPU; the CPU
// path of batched FedAvg is the vmap composition in parallel/fed_model.py.
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <torch/library.h>

#include <algorithm>

#include "kernels.h"

namespace commeff {

void launch_weight_image(const float* W, int64_t ld, int G, int K, int C, int RS, int Kc, int kind,
                         uint16_t* dst, hipStream_t stream);
void launch_row_sgd(float* W, int64_t ld, const float* src, int64_t sld, const float* Gr, int64_t gld, int G,
                    int64_t d4, float clip, float lr, float wd, float* part, uint16_t* Wb, hipStream_t stream);
int row_sgd_parts();
void launch_fedavg_upload(float* out, const float* w0, const float* W, int64_t ld, int G, int64_t d, float n,
                          const int32_t* perm, hipStream_t stream, int64_t dout);
void launch_gather_rows(float* dst, uint16_t* dstb, const float* src, const int32_t* perm, int64_t d,
                        hipStream_t stream, int64_t dsrc);
void launch_dgrad_image(const uint16_t* src, int64_t ld, int G, int K, int C, uint16_t* dst, hipStream_t stream);
void launch_bcast_rows(float* W, int64_t ld, const float* src, int G, int64_t d4, hipStream_t stream);
void launch_cast_rows(uint16_t* Wb, const float* W, int64_t ld, int G, int64_t off, int64_t n, hipStream_t stream);
void launch_avgmax_head_fwd(const uint16_t* x, int n, int HW, int G, int C, float* feat, uint8_t* codes,
                            hipStream_t stream);
void launch_avgmax_head_bwd(const float* df, const uint8_t* codes, int n, int HW, int G, int C, uint16_t* dx,
                            hipStream_t stream, int S);
void launch_ew_bf16(const uint16_t* a, const uint16_t* b, uint16_t* y, int64_t n8, int mode, hipStream_t stream);

namespace {

hipStream_t stream_now() { return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

void check_cl_bf16(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16 && t.dim() == 4 &&
                  t.is_contiguous(at::MemoryFormat::ChannelsLast),
              name, " must be a bf16 NCHW tensor with channels_last memory");
}

const uint16_t* bf(const at::Tensor& t) { return reinterpret_cast<const uint16_t*>(t.data_ptr()); }
uint16_t* bfw(at::Tensor& t) { return reinterpret_cast<uint16_t*>(t.data_ptr()); }

// fp32 parameter / gradient rows: a contiguous [rows, ld] (or flat) tensor
// holding `rows` rows of ld floats; [off, off + span) must lie inside a row
// (ld 0: one row shared by every group -- the server weights of the first local step)
void check_rows(const at::Tensor& t, int64_t ld, int64_t rows, int64_t off, int64_t span, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous(), name,
              " must be a contiguous fp32 device tensor");
  TORCH_CHECK(rows >= 1 && off >= 0 && span >= 0 && ld >= 0 && (ld == 0 || off + span <= ld) &&
                  (rows - 1) * ld + off + span <= t.numel(),
              name, ": [", off, ", ", off + span, ") of ", rows, " rows of ", ld, " floats exceeds ", t.numel());
}

// the current weights a fused SGD step scales (beta): fp32 rows sld apart (0:
// the shared server row of the first local step); none: the destination's own
const float* src_rows(const c10::optional<at::Tensor>& src, int64_t sld, int64_t rows, int64_t off, int64_t span,
                      const char* name) {
  if (!src.has_value() || !src->defined()) return nullptr;
  check_rows(*src, sld, rows, off, span, name);
  return src->data_ptr<float>();
}

int64_t out_size(int64_t in, int64_t k, int64_t stride, int64_t pad) { return (in + 2 * pad - k) / stride + 1; }

// per-client bf16 images of conv weights held in fp32 rows W[g*ld + off + (k*C + c)*RS + t]:
// kind 0 -> [G*K, R, S, C] (halo forward), 1 -> [G*C, R, S, K] (flipped, halo dgrad),
// 2 -> [G, K, Kc] (column-GEMM image, (r, s, c) columns, zero padding)
at::Tensor fa_weight_image(const at::Tensor& W, int64_t ld, int64_t G, int64_t off, int64_t K, int64_t C,
                           int64_t R, int64_t Kc, int64_t kind) {
  const int64_t RS = R * R;
  check_rows(W, ld, G, off, K * C * RS, "fa_weight_image: W");
  TORCH_CHECK(kind >= 0 && kind <= 2 && K >= 1 && C >= 1 && R >= 1, "fa_weight_image: kind / shape");
  TORCH_CHECK(kind != 2 || (Kc % 8 == 0 && Kc >= RS * C), "fa_weight_image: Kc");
  TORCH_CHECK(G * K * std::max(Kc, C * RS) < (int64_t{1} << 40), "fa_weight_image: size");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(W.device());
  auto o = W.options().dtype(at::kBFloat16);
  at::Tensor dst = kind == 0 ? at::empty({G * K, R, R, C}, o)
                   : kind == 1 ? at::empty({G * C, R, R, K}, o)
                               : at::empty({G, K, Kc}, o);
  launch_weight_image(W.data_ptr<float>() + off, ld, static_cast<int>(G), static_cast<int>(K),
                      static_cast<int>(C), static_cast<int>(RS), static_cast<int>(Kc), static_cast<int>(kind),
                      bfw(dst), stream_now());
  return dst;
}

// W[g] = src[g] - lr (scale_g G[g] + wd src[g]) for g < rows (src ld 0: one
// broadcast row); scale_g = min(1, clip / |G[g]|) when clip > 0
void fa_row_sgd(at::Tensor W, int64_t ld, const at::Tensor& src, int64_t sld, const at::Tensor& Gr, int64_t gld,
                int64_t rows, int64_t d, double clip, double lr, double wd, const c10::optional<at::Tensor>& Wb) {
  const int64_t d4 = (d + 3) / 4;
  TORCH_CHECK(ld % 4 == 0 && sld % 4 == 0 && gld % 4 == 0 && d4 * 4 <= std::min(ld, gld),
              "fa_row_sgd: row strides must be multiples of 4 holding d");
  check_rows(W, ld, rows, 0, d4 * 4, "fa_row_sgd: W");
  check_rows(Gr, gld, rows, 0, d4 * 4, "fa_row_sgd: G");
  TORCH_CHECK(src.is_cuda() && src.scalar_type() == at::kFloat && src.is_contiguous() &&
                  src.numel() >= (sld == 0 ? d4 * 4 : rows * sld) && (sld == 0 || sld >= d4 * 4),
              "fa_row_sgd: src rows");
  for (const at::Tensor* t : {static_cast<const at::Tensor*>(&W), &src, &Gr})
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "fa_row_sgd: 16-byte aligned rows");
  uint16_t* wb = nullptr;
  if (Wb.has_value() && Wb->defined()) {  // bf16 mirror rows of the same layout
    TORCH_CHECK(Wb->is_cuda() && Wb->scalar_type() == at::kBFloat16 && Wb->is_contiguous() &&
                    Wb->numel() >= rows * ld && reinterpret_cast<uintptr_t>(Wb->data_ptr()) % 8 == 0,
                "fa_row_sgd: Wb must be contiguous bf16 [rows, ld]");
    wb = reinterpret_cast<uint16_t*>(Wb->data_ptr());
  }
  c10::hip::HIPGuardMasqueradingAsCUDA guard(W.device());
  at::Tensor part;
  if (clip > 0) part = at::empty({rows * row_sgd_parts()}, W.options());
  launch_row_sgd(W.data_ptr<float>(), ld, src.data_ptr<float>(), sld, Gr.data_ptr<float>(), gld,
                 static_cast<int>(rows), d4, static_cast<float>(clip), static_cast<float>(lr),
                 static_cast<float>(wd), clip > 0 ? part.data_ptr<float>() : nullptr, wb, stream_now());
}

// out[j] += n sum_g (w0[j] - W[g*ld + j]), j < d
// (perm: rows / w0 in the engine's layout of D >= d positions, element j ->
// coordinate perm[j] of out, < 0: layout padding)
void fa_upload(at::Tensor out, const at::Tensor& w0, const at::Tensor& W, int64_t ld, int64_t rows, double n,
               const c10::optional<at::Tensor>& perm) {
  const int64_t dout = out.numel();
  const bool hp = perm.has_value() && perm->defined();
  const int64_t d = hp ? perm->numel() : dout;
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kFloat && out.is_contiguous() && w0.numel() >= d &&
                  w0.scalar_type() == at::kFloat && w0.is_contiguous() && d >= dout,
              "fa_upload: out / w0 fp32 [d]");
  check_rows(W, ld, rows, 0, d, "fa_upload: W");
  TORCH_CHECK(ld % 4 == 0 && reinterpret_cast<uintptr_t>(W.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(w0.data_ptr()) % 16 == 0,
              "fa_upload: rows of a multiple of 4 floats, 16-byte aligned");
  const int32_t* pp = nullptr;
  if (perm.has_value() && perm->defined()) {
    TORCH_CHECK(perm->is_cuda() && perm->scalar_type() == at::kInt && perm->is_contiguous(),
                "fa_upload: perm int32 [D]");
    pp = perm->data_ptr<int32_t>();
  }
  c10::hip::HIPGuardMasqueradingAsCUDA guard(out.device());
  launch_fedavg_upload(out.data_ptr<float>(), w0.data_ptr<float>(), W.data_ptr<float>(), ld,
                       static_cast<int>(rows), d, static_cast<float>(n), pp, stream_now(), dout);
}

// dst[j] = src[perm[j]], dstb = bf16(dst): the server weights in the engine's layout
void fa_gather_rows(at::Tensor dst, at::Tensor dstb, const at::Tensor& src, const at::Tensor& perm) {
  const int64_t d = perm.numel();
  TORCH_CHECK(perm.is_cuda() && perm.scalar_type() == at::kInt && perm.is_contiguous(), "fa_gather_rows: perm int32");
  TORCH_CHECK(dst.is_cuda() && dst.scalar_type() == at::kFloat && dst.is_contiguous() && dst.numel() >= d &&
                  dstb.scalar_type() == at::kBFloat16 && dstb.is_contiguous() && dstb.numel() >= d &&
                  src.scalar_type() == at::kFloat && src.is_contiguous() && src.numel() <= d,
              "fa_gather_rows: dst fp32, dstb bf16 >= D, src fp32 [<= D] (perm < 0: padding)");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(dst.device());
  launch_gather_rows(dst.data_ptr<float>(), bfw(dstb), src.data_ptr<float>(), perm.data_ptr<int32_t>(), d,
                     stream_now(), src.numel());
}

// W[g] = src for every row g < rows (d floats, 16-byte aligned rows)
void fa_bcast_rows(at::Tensor W, int64_t ld, const at::Tensor& src, int64_t rows, int64_t d) {
  const int64_t d4 = (d + 3) / 4;
  TORCH_CHECK(ld % 4 == 0 && d4 * 4 <= ld, "fa_bcast_rows: ld");
  check_rows(W, ld, rows, 0, d4 * 4, "fa_bcast_rows: W");
  TORCH_CHECK(src.is_cuda() && src.scalar_type() == at::kFloat && src.is_contiguous() && src.numel() >= d4 * 4 &&
                  reinterpret_cast<uintptr_t>(src.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(W.data_ptr()) % 16 == 0,
              "fa_bcast_rows: src fp32 >= d (padded to 4), aligned");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(W.device());
  launch_bcast_rows(W.data_ptr<float>(), ld, src.data_ptr<float>(), static_cast<int>(rows), d4, stream_now());
}

// Wb[g, off:off+n] = bf16(W[g, off:off+n]) for every row
void fa_cast_rows(at::Tensor Wb, const at::Tensor& W, int64_t ld, int64_t rows, int64_t off, int64_t n) {
  check_rows(W, ld, rows, off, n, "fa_cast_rows: W");
  TORCH_CHECK(Wb.is_cuda() && Wb.scalar_type() == at::kBFloat16 && Wb.is_contiguous() && Wb.numel() >= rows * ld,
              "fa_cast_rows: Wb bf16 [rows, ld]");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(W.device());
  launch_cast_rows(bfw(Wb), W.data_ptr<float>(), ld, static_cast<int>(rows), off, n, stream_now());
}

// [G*C, 3, 3, K] flipped / transposed dgrad image of 3x3 weights held as bf16
// (r, s, c)-ordered rows Wb[g*ld + off + (k*9 + t)*C + c] (ld 0: one image)
at::Tensor fa_dgrad_image(const at::Tensor& Wb, int64_t ld, int64_t G, int64_t off, int64_t K, int64_t C) {
  TORCH_CHECK(Wb.is_cuda() && Wb.scalar_type() == at::kBFloat16 && Wb.is_contiguous(), "fa_dgrad_image: Wb bf16");
  TORCH_CHECK(K % 64 == 0 && C % 64 == 0 && G >= 1 && off >= 0 && (ld == 0 || off + K * 9 * C <= ld) &&
                  (ld == 0 ? 0 : G - 1) * ld + off + K * 9 * C <= Wb.numel(),
              "fa_dgrad_image: 64 | K, C; rows in range");
  const int64_t Gi = ld == 0 ? 1 : G;
  c10::hip::HIPGuardMasqueradingAsCUDA guard(Wb.device());
  auto dst = at::empty({Gi * C, 3, 3, K}, Wb.options());
  launch_dgrad_image(bf(Wb) + off, ld, static_cast<int>(Gi), static_cast<int>(K), static_cast<int>(C), bfw(dst),
                     stream_now());
  return dst;
}

// grouped stride-1 3x3 conv of channel-stacked x whose group-g weights are the
// kg rows [kg][3][3][C] at w + off + g * ld (ld 0: every group the same rows)
at::Tensor conv3x3_fwd_rows(const at::Tensor& x, const at::Tensor& w, int64_t G, int64_t off, int64_t ld,
                            int64_t kg, const c10::optional<at::Tensor>& addend, bool bt) {
  check_cl_bf16(x, "conv3x3_fwd_rows: x");
  const int64_t N = x.size(0), GC = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(G >= 1 && GC % G == 0 && kg >= 1, "conv3x3_fwd_rows: channels not a multiple of G");
  const int64_t C = GC / G, K = G * kg;
  // bt: x is a conv's output gradient and w that conv's rows [C][3][3][kg]
  // (same element count per group as a [kg][3][3][C] image)
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kBFloat16 && w.is_contiguous() && off >= 0 && ld >= 0 &&
                  (ld == 0 || off + kg * 9 * C <= ld) && (ld == 0 ? 0 : G - 1) * ld + off + kg * 9 * C <= w.numel(),
              "conv3x3_fwd_rows: weight rows out of range");
  TORCH_CHECK(N * H * W * std::max(GC, K) < (int64_t{1} << 31), "conv3x3_fwd_rows: size");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  auto y = at::empty({N, K, H, W}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  const bool add = addend.has_value() && addend->defined();
  if (add) {  // y = conv + addend (fused in the epilogue)
    check_cl_bf16(*addend, "conv3x3_fwd_rows: addend");
    TORCH_CHECK(addend->sizes() == y.sizes(), "conv3x3_fwd_rows: addend shape");
  }
  ConvFwdArgs a;
  a.x = bf(x);
  a.w = bf(w) + off;
  a.y = bfw(y);
  a.mask = nullptr;
  a.addend = add ? bf(*addend) : nullptr;
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
  a.w_gs = ld > 0 ? ld : -1;
  a.w_bt = bt ? 1 : 0;
  if (a.P == 0) return y;
  if (!launch_conv3x3_fwd_grouped(a, stream_now())) return at::empty({0}, x.options());
  return y;
}

// x [n, G*C, h, w] channels_last -> (feat fp32 [G, n, 2C] = mean | max, codes uint8 [n, G*C])
std::tuple<at::Tensor, at::Tensor> fa_head_fwd(const at::Tensor& x, int64_t G) {
  check_cl_bf16(x, "fa_head_fwd: x");
  const int64_t n = x.size(0), GC = x.size(1), HW = x.size(2) * x.size(3);
  TORCH_CHECK(G >= 1 && GC % G == 0 && HW >= 1 && HW <= 256, "fa_head_fwd: G | channels, <= 256 pixels");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  const int64_t C = GC / G;
  auto feat = at::empty({G, n, 2 * C}, x.options().dtype(at::kFloat));
  auto codes = at::empty({n, GC}, x.options().dtype(at::kByte));
  launch_avgmax_head_fwd(bf(x), static_cast<int>(n), static_cast<int>(HW), static_cast<int>(G),
                         static_cast<int>(C), feat.data_ptr<float>(), codes.data_ptr<uint8_t>(), stream_now());
  return {feat, codes};
}

// the per-client classifier step (fedavg.hip fa_linear_ce_kernel): returns
// (loss [G n], correct [G n]); writes dfeat and the updated rows of dst
std::tuple<at::Tensor, at::Tensor> fa_linear_ce(const at::Tensor& feat, int64_t fsg, int64_t fsn, int64_t G,
                                                int64_t n, const at::Tensor& W, int64_t wld, int64_t woff,
                                                int64_t boff, int64_t C, int64_t F, double scale, const at::Tensor& y,
                                                at::Tensor dfeat, int64_t dsg, int64_t dsn, at::Tensor dst, int64_t dld,
                                                double beta, double alpha, const c10::optional<at::Tensor>& src,
                                                int64_t sld, const c10::optional<at::Tensor>& mirror, int64_t mld,
                                                int64_t dss, int64_t ccs) {
  TORCH_CHECK(feat.is_cuda() && (feat.scalar_type() == at::kFloat || feat.scalar_type() == at::kBFloat16) &&
                  (dfeat.scalar_type() == at::kFloat || dfeat.scalar_type() == at::kBFloat16),
              "fa_linear_ce: feat / dfeat fp32 or bf16");
  TORCH_CHECK(G >= 1 && n >= 1 && n <= kFaMaxN && C >= 1 && F >= 1 &&
                  fa_linear_lds_bytes(static_cast<int>(n), static_cast<int>(C), static_cast<int>(F)) <= kFaMaxLds,
              "fa_linear_ce: n <= ", kFaMaxN, " examples per client and n (F + C) floats of LDS");
  auto span_ok = [](const at::Tensor& t, int64_t sg, int64_t sn, int64_t G, int64_t n, int64_t F) {
    return t.is_contiguous() && sg >= 0 && sn >= 0 && (G - 1) * sg + (n - 1) * sn + F <= t.numel();
  };
  const int64_t S = ccs > 0 ? (C + ccs - 1) / ccs : 1;
  TORCH_CHECK(span_ok(feat, fsg, fsn, G, n, F) && span_ok(dfeat, dsg, dsn, G, n, F) &&
                  (S == 1 || (dss > 0 && (S - 1) * dss + (G - 1) * dsg + (n - 1) * dsn + F <= dfeat.numel())),
              "fa_linear_ce: feat / dfeat spans (S class-chunk slabs dss apart)");
  TORCH_CHECK(W.scalar_type() == at::kFloat && W.is_contiguous() && wld >= 0 && woff >= 0 &&
                  (G - 1) * wld + woff + C * F <= W.numel() && (boff < 0 || (G - 1) * wld + boff + C <= W.numel()),
              "fa_linear_ce: weight rows");
  TORCH_CHECK(dst.scalar_type() == at::kFloat && dst.is_contiguous() && dld >= 0 &&
                  (G - 1) * dld + woff + C * F <= dst.numel() && (boff < 0 || (G - 1) * dld + boff + C <= dst.numel()),
              "fa_linear_ce: dst rows");
  const bool hs = src.has_value() && src->defined();
  if (hs)
    TORCH_CHECK(src->scalar_type() == at::kFloat && src->is_contiguous() && sld >= 0 &&
                    (G - 1) * sld + woff + C * F <= src->numel() &&
                    (boff < 0 || (G - 1) * sld + boff + C <= src->numel()),
                "fa_linear_ce: src rows");
  const bool hm = mirror.has_value() && mirror->defined();
  if (hm)
    TORCH_CHECK(mirror->scalar_type() == at::kBFloat16 && mirror->is_contiguous() &&
                    (G - 1) * mld + woff + C * F <= mirror->numel(),
                "fa_linear_ce: mirror rows");
  TORCH_CHECK(y.scalar_type() == at::kLong && y.is_contiguous() && y.numel() == G * n, "fa_linear_ce: y int64 [G n]");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(feat.device());
  auto loss = at::empty({G * n}, feat.options().dtype(at::kFloat));
  auto correct = at::empty({G * n}, feat.options().dtype(at::kFloat));
  FaLinearArgs a{};
  a.feat = feat.data_ptr();
  a.fsg = fsg;
  a.fsn = fsn;
  a.W = W.data_ptr<float>();
  a.wld = wld;
  a.woff = woff;
  a.boff = boff;
  a.y = y.data_ptr<int64_t>();
  a.n = static_cast<int>(n);
  a.C = static_cast<int>(C);
  a.F = static_cast<int>(F);
  a.scale = static_cast<float>(scale);
  a.loss = loss.data_ptr<float>();
  a.correct = correct.data_ptr<float>();
  a.dfeat = dfeat.data_ptr();
  a.dsg = dsg;
  a.dsn = dsn;
  a.dss = dss;
  a.ccs = S == 1 ? 0 : static_cast<int>(ccs);
  a.dst = dst.data_ptr<float>();
  a.dld = dld;
  a.beta = static_cast<float>(beta);
  a.alpha = static_cast<float>(alpha);
  a.src = hs ? src->data_ptr<float>() : nullptr;
  a.sld = sld;
  a.mirror = hm ? reinterpret_cast<uint16_t*>(mirror->data_ptr()) : nullptr;
  a.mld = mld;
  auto logits = at::empty({G * n * C}, feat.options().dtype(at::kFloat));
  launch_fa_linear_ce(a, static_cast<int>(G), feat.scalar_type() == at::kBFloat16,
                      dfeat.scalar_type() == at::kBFloat16, logits.data_ptr<float>(), stream_now());
  return {loss, correct};
}

// ---- Fixup per-client scalars (fedavg.hip fa_affine*): x channel-stacked
// [n, G C, H, W] bf16 channels_last, or client-major (client_major: the
// stem's input [G n, C, H, W], any C)
static FaAffine affine_args(const at::Tensor& x, int64_t G, bool client_major, const at::Tensor& W, int64_t ld,
                            int64_t soff, int64_t boff, const char* what) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 4 && G >= 1, what, ": bf16 4-D x");
  TORCH_CHECK(W.scalar_type() == at::kFloat && W.is_contiguous() && ld >= 0 &&
                  (G - 1) * ld + std::max(soff, boff) < W.numel(),
              what, ": scalar rows");
  FaAffine a{};
  a.G = static_cast<int>(G);
  a.S = soff >= 0 ? W.data_ptr<float>() + soff : nullptr;
  a.B = boff >= 0 ? W.data_ptr<float>() + boff : nullptr;
  a.ld = ld;
  if (client_major) {
    TORCH_CHECK(x.is_contiguous(at::MemoryFormat::ChannelsLast) || x.is_contiguous(), what, ": dense x");
    TORCH_CHECK(x.numel() % (8 * G) == 0 && (x.numel() / G) % 8 == 0, what, ": 8-element client blocks");
    a.per = x.numel() / G;
    a.C = 0;
    a.GC = 0;
  } else {
    check_cl_bf16(x, what);
    const int64_t GC = x.size(1);
    TORCH_CHECK(GC % G == 0 && (GC / G) % 8 == 0, what, ": G | channels, 8 | channels per client");
    a.C = static_cast<int>(GC / G);
    a.GC = GC;
    a.per = x.numel() / G;
  }
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0, what, ": 16-byte aligned x");
  return a;
}

// y = relu?(x * s_g + b_g (+ add))
at::Tensor fa_affine(const at::Tensor& x, int64_t G, bool client_major, const at::Tensor& W, int64_t ld, int64_t soff,
                     int64_t boff, const c10::optional<at::Tensor>& add, bool relu) {
  FaAffine a = affine_args(x, G, client_major, W, ld, soff, boff, "fa_affine");
  auto y = at::empty_like(x);
  if (add.has_value() && add->defined()) {
    TORCH_CHECK(add->sizes() == x.sizes() && add->strides() == x.strides() && add->scalar_type() == at::kBFloat16,
                "fa_affine: add like x");
    a.add = bf(*add);
  }
  a.x = bf(x);
  a.y = bfw(y);
  a.relu = relu ? 1 : 0;
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  launch_fa_affine(a, stream_now());
  return y;
}

// (out1 = dpre * s (+ add2) or undefined, out2 = dpre or undefined, partial sums [chunks, G, 2])
std::tuple<at::Tensor, at::Tensor, at::Tensor> fa_affine_bwd(const at::Tensor& dy, int64_t G, bool client_major,
                                                             const at::Tensor& W, int64_t ld, int64_t soff,
                                                             const c10::optional<at::Tensor>& yrelu,
                                                             const c10::optional<at::Tensor>& xs,
                                                             const c10::optional<at::Tensor>& add2, bool want1,
                                                             bool want2) {
  FaAffine a = affine_args(dy, G, client_major, W, ld, soff, -1, "fa_affine_bwd");
  FaAffineBwd b{};
  b.dy = bf(dy);
  auto same = [&](const c10::optional<at::Tensor>& t, const char* nm) -> const uint16_t* {
    if (!t.has_value() || !t->defined()) return nullptr;
    TORCH_CHECK(t->sizes() == dy.sizes() && t->strides() == dy.strides() && t->scalar_type() == at::kBFloat16,
                "fa_affine_bwd: ", nm, " like dy");
    return bf(*t);
  };
  b.yrelu = same(yrelu, "y");
  b.xs = same(xs, "xs");
  b.add2 = same(add2, "add2");
  at::Tensor o1, o2;
  if (want1) {
    o1 = at::empty_like(dy);
    b.out1 = bfw(o1);
  }
  if (want2) {
    o2 = at::empty_like(dy);
    b.out2 = bfw(o2);
  }
  // chunks of ~8 K elements per block, at least one block per client
  b.chunk = 8192;
  const int64_t chunks = (a.per + b.chunk - 1) / b.chunk;
  auto part = at::empty({chunks, G, 2}, dy.options().dtype(at::kFloat));
  b.part = part.data_ptr<float>();
  c10::hip::HIPGuardMasqueradingAsCUDA guard(dy.device());
  launch_fa_affine_bwd(a, b, static_cast<int>(chunks), stream_now());
  return {o1, o2, part};
}

// ---- merged-batch Fixup scalars (ops/fixup.py): one scale / bias pair
// (fp32 [1] parameters) over a whole dense bf16 activation, any layout
static FaAffine fx_args(const at::Tensor& x, const c10::optional<at::Tensor>& s,
                        const c10::optional<at::Tensor>& b, const char* what) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.is_non_overlapping_and_dense() &&
                  x.numel() % 8 == 0 && x.numel() > 0 && reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0,
              what, ": dense 16-byte aligned bf16 x, 8 | numel");
  auto scalar = [&](const c10::optional<at::Tensor>& t, const char* nm) -> const float* {
    if (!t.has_value() || !t->defined()) return nullptr;
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->numel() == 1, what, ": fp32 scalar ", nm);
    return t->data_ptr<float>();
  };
  FaAffine a{};
  a.G = 1;
  a.S = scalar(s, "scale");
  a.B = scalar(b, "bias");
  a.ld = 0;
  a.per = x.numel();
  return a;
}

// y = relu?(x * s + b (+ add)), one bf16 rounding
at::Tensor fx_affine(const at::Tensor& x, const c10::optional<at::Tensor>& s, const c10::optional<at::Tensor>& b,
                     const c10::optional<at::Tensor>& add, bool relu, const c10::optional<at::Tensor>& post) {
  FaAffine a = fx_args(x, s, b, "fx_affine");
  if (post.has_value() && post->defined()) {
    TORCH_CHECK(relu && post->is_cuda() && post->scalar_type() == at::kFloat && post->numel() == 1,
                "fx_affine: fp32 scalar post bias after a relu");
    a.P = post->data_ptr<float>();
  }
  auto y = at::empty_like(x);
  if (add.has_value() && add->defined()) {
    TORCH_CHECK(add->sizes() == x.sizes() && add->strides() == x.strides() && add->scalar_type() == at::kBFloat16 &&
                    reinterpret_cast<uintptr_t>(add->data_ptr()) % 16 == 0,
                "fx_affine: add like x");
    a.add = bf(*add);
  }
  a.x = bf(x);
  a.y = bfw(y);
  a.relu = relu ? 1 : 0;
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  launch_fa_affine(a, stream_now());
  return y;
}

// (dx = dpre * s or undefined, dadd = dpre or undefined, sums fp32 [2] =
// {sum dpre, sum dpre xs -- without xs: sum dy unmasked}), dpre = dy masked
// by yrelu > 0; the sums in a fixed order (deterministic)
// mask_x: the relu mask recomputed from xs (x s + b > 0, b given), the second
// sum of dy unmasked (the post bias's gradient)
std::tuple<at::Tensor, at::Tensor, at::Tensor> fx_affine_bwd(const at::Tensor& dy, const c10::optional<at::Tensor>& s,
                                                             const c10::optional<at::Tensor>& yrelu,
                                                             const c10::optional<at::Tensor>& xs, bool want1,
                                                             bool want2, const c10::optional<at::Tensor>& bias,
                                                             bool mask_x, const c10::optional<at::Tensor>& add2) {
  FaAffine a = fx_args(dy, s, bias, "fx_affine_bwd");
  TORCH_CHECK(!mask_x || (xs.has_value() && xs->defined()), "fx_affine_bwd: mask_x needs xs");
  FaAffineBwd b{};
  b.dy = bf(dy);
  auto same = [&](const c10::optional<at::Tensor>& t, const char* nm) -> const uint16_t* {
    if (!t.has_value() || !t->defined()) return nullptr;
    TORCH_CHECK(t->sizes() == dy.sizes() && t->strides() == dy.strides() && t->scalar_type() == at::kBFloat16 &&
                    reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0,
                "fx_affine_bwd: ", nm, " like dy");
    return bf(*t);
  };
  b.yrelu = same(yrelu, "y");
  b.xs = same(xs, "xs");
  b.add2 = same(add2, "add2");  // out1 = dpre s + add2 (a second gradient of x)
  b.mask_x = mask_x ? 1 : 0;
  at::Tensor o1, o2;
  if (want1) {
    o1 = at::empty_like(dy);
    b.out1 = bfw(o1);
  }
  if (want2) {
    o2 = at::empty_like(dy);
    b.out2 = bfw(o2);
  }
  // at most ~2K blocks (then one block folds their partials), 2K-element multiples
  b.chunk = std::max<int64_t>(8192, ((a.per + 2047) / 2048 + 2047) / 2048 * 2048);
  const int64_t chunks = (a.per + b.chunk - 1) / b.chunk;
  auto part = at::empty({chunks, 1, 2}, dy.options().dtype(at::kFloat));
  auto sums = at::empty({2}, dy.options().dtype(at::kFloat));
  b.part = part.data_ptr<float>();
  c10::hip::HIPGuardMasqueradingAsCUDA guard(dy.device());
  launch_fa_affine_bwd(a, b, static_cast<int>(chunks), stream_now());
  launch_fx_part_sum(part.data_ptr<float>(), static_cast<int>(chunks), sums.data_ptr<float>(), stream_now());
  return {o1, o2, sums};
}

// dst[g ld + boff] / dst[g ld + soff] = beta src + alpha (sum of the partials' dpre / dpre x)
void fa_scalar_sgd(const at::Tensor& part, at::Tensor dst, int64_t ld, int64_t boff, int64_t soff, double beta,
                   double alpha, const c10::optional<at::Tensor>& src, int64_t sld) {
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat && part.is_contiguous() && part.dim() == 3 &&
                  part.size(2) == 2,
              "fa_scalar_sgd: part fp32 [chunks, G, 2]");
  const int64_t G = part.size(1);
  TORCH_CHECK(dst.scalar_type() == at::kFloat && dst.is_contiguous() && ld >= 0 &&
                  (G - 1) * ld + std::max(boff, soff) < dst.numel(),
              "fa_scalar_sgd: dst rows");
  const float* sp = nullptr;
  if (src.has_value() && src->defined()) {
    TORCH_CHECK(src->scalar_type() == at::kFloat && src->is_contiguous() && sld >= 0 &&
                    (G - 1) * sld + std::max(boff, soff) < src->numel(),
                "fa_scalar_sgd: src rows");
    sp = src->data_ptr<float>();
  }
  c10::hip::HIPGuardMasqueradingAsCUDA guard(part.device());
  launch_fa_scalar_sgd(part.data_ptr<float>(), static_cast<int>(part.size(0)), static_cast<int>(G),
                       dst.data_ptr<float>(), ld, boff, soff, static_cast<float>(beta), static_cast<float>(alpha), sp,
                       sld, stream_now());
}

at::Tensor fa_head_bwd(const at::Tensor& df, const at::Tensor& codes, int64_t H, int64_t W) {
  TORCH_CHECK(df.is_cuda() && df.scalar_type() == at::kFloat && df.is_contiguous() && df.dim() == 3 &&
                  df.size(2) % 2 == 0,
              "fa_head_bwd: df fp32 [S G, n, 2C] (S partial slabs, summed)");
  const int64_t n = df.size(1), C = df.size(2) / 2;
  TORCH_CHECK(codes.scalar_type() == at::kByte && codes.is_contiguous() && codes.dim() == 2 &&
                  codes.size(0) == n && C >= 1 && codes.size(1) % C == 0 && H * W >= 1 && H * W <= 256,
              "fa_head_bwd: codes uint8 [n, G*C]");
  const int64_t G = codes.size(1) / C, S = df.size(0) / (G > 0 ? G : 1);
  TORCH_CHECK(G >= 1 && S >= 1 && S * G == df.size(0), "fa_head_bwd: df rows a multiple of the clients");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(df.device());
  auto dx = at::empty({n, G * C, H, W}, df.options().dtype(at::kBFloat16).memory_format(at::MemoryFormat::ChannelsLast));
  launch_avgmax_head_bwd(df.data_ptr<float>(), codes.data_ptr<uint8_t>(), static_cast<int>(n),
                         static_cast<int>(H * W), static_cast<int>(G), static_cast<int>(C), bfw(dx), stream_now(),
                         static_cast<int>(S));
  return dx;
}

// mode 0: a + b, mode 1: relu(a) (bf16 channels_last, 8-element multiples)
at::Tensor fa_ew(const at::Tensor& a, const c10::optional<at::Tensor>& b, int64_t mode) {
  check_cl_bf16(a, "fa_ew: a");
  TORCH_CHECK(a.numel() % 8 == 0 && (mode == 0 || mode == 1), "fa_ew: numel % 8, mode 0 / 1");
  if (mode == 0) {
    TORCH_CHECK(b.has_value() && b->defined(), "fa_ew: add needs b");
    check_cl_bf16(*b, "fa_ew: b");
    TORCH_CHECK(b->sizes() == a.sizes(), "fa_ew: b shape");
  }
  c10::hip::HIPGuardMasqueradingAsCUDA guard(a.device());
  auto y = at::empty_like(a, a.options().memory_format(at::MemoryFormat::ChannelsLast));
  launch_ew_bf16(bf(a), mode == 0 ? bf(*b) : nullptr, bfw(y), a.numel() / 8, static_cast<int>(mode), stream_now());
  return y;
}

// grouped column image [P, G, Kc] (P = n*OH*OW): channel-stacked x [n, G*C, H, W]
// (client_major false) or client-major x [G*n, C, H, W] (true), channels_last
at::Tensor im2col_grouped(const at::Tensor& x, int64_t G, int64_t R, int64_t S, int64_t stride, int64_t pad,
                          int64_t Kc, bool client_major) {
  if (client_major) {  // the augmentation kernel's images: channels innermost, any pixel stride
    TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 4 && x.stride(1) == 1 &&
                    x.stride(3) >= x.size(1) && x.stride(2) >= x.stride(3) * x.size(3) &&
                    x.stride(0) >= x.stride(2) * x.size(2),
                "im2col_grouped: client-major x must be bf16 NCHW with channels innermost");
  } else {
    check_cl_bf16(x, "im2col_grouped: x");
  }
  const int64_t H = x.size(2), W = x.size(3);
  TORCH_CHECK(G >= 1, "im2col_grouped: G");
  const int64_t n = client_major ? x.size(0) / G : x.size(0);
  const int64_t C = client_major ? x.size(1) : x.size(1) / G;
  TORCH_CHECK(client_major ? x.size(0) % G == 0 : x.size(1) % G == 0, "im2col_grouped: G does not divide");
  TORCH_CHECK(R >= 1 && S >= 1 && stride >= 1 && pad >= 0 && pad < R && pad < S, "im2col_grouped: geometry");
  const int64_t OH = out_size(H, R, stride, pad), OW = out_size(W, S, stride, pad);
  TORCH_CHECK(OH > 0 && OW > 0 && Kc % 8 == 0 && Kc >= R * S * C, "im2col_grouped: Kc / output");
  const int64_t P = n * OH * OW;
  TORCH_CHECK(P * G * (Kc / 8) < (int64_t{1} << 32) && x.size(0) * x.stride(0) < (int64_t{1} << 40),
              "im2col_grouped: 32-bit range");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  auto col = at::empty({P, G, Kc}, x.options());
  Im2colArgs a{};
  a.x = bf(x);
  a.col = bfw(col);
  a.N = static_cast<int>(n); a.H = static_cast<int>(H); a.W = static_cast<int>(W);
  a.C = static_cast<int>(C); a.OH = static_cast<int>(OH); a.OW = static_cast<int>(OW);
  a.R = static_cast<int>(R); a.S = static_cast<int>(S);
  a.stride = static_cast<int>(stride); a.pad = static_cast<int>(pad); a.Kc = static_cast<int>(Kc);
  a.sN = x.stride(0); a.sH = x.stride(2); a.sW = x.stride(3);
  a.G = static_cast<int>(G);
  a.sG = client_major ? n * x.stride(0) : C;
  a.vec = C % 8 == 0 && a.sW % 8 == 0 && a.sH % 8 == 0 && a.sN % 8 == 0 && a.sG % 8 == 0 &&
          reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0;
  launch_im2col(a, stream_now());
  return col;
}

// gx [n, G*C, H, W] (channels_last, channel-stacked) of gcol [P, G, Kc]
at::Tensor col2im_grouped(const at::Tensor& gcol, int64_t G, int64_t n, int64_t H, int64_t W, int64_t C,
                          int64_t R, int64_t S, int64_t stride, int64_t pad) {
  TORCH_CHECK(gcol.is_cuda() && gcol.scalar_type() == at::kBFloat16 && gcol.dim() == 3 && gcol.is_contiguous(),
              "col2im_grouped: gcol must be a contiguous bf16 [P, G, Kc] tensor");
  TORCH_CHECK(C % 8 == 0 && R >= 1 && S >= 1 && stride >= 1 && pad >= 0 && pad < R && pad < S,
              "col2im_grouped: geometry (C % 8 == 0)");
  const int64_t OH = out_size(H, R, stride, pad), OW = out_size(W, S, stride, pad);
  const int64_t Kc = gcol.size(2);
  TORCH_CHECK(gcol.size(0) == n * OH * OW && gcol.size(1) == G && Kc % 8 == 0 && Kc >= R * S * C,
              "col2im_grouped: gcol shape");
  TORCH_CHECK(n * H * W * G * (C / 8) < (int64_t{1} << 32) && gcol.numel() < (int64_t{1} << 40),
              "col2im_grouped: index range");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(gcol.device());
  auto gx = at::empty({n, G * C, H, W}, gcol.options().memory_format(at::MemoryFormat::ChannelsLast));
  Im2colArgs a{};
  a.N = static_cast<int>(n); a.H = static_cast<int>(H); a.W = static_cast<int>(W);
  a.C = static_cast<int>(C); a.OH = static_cast<int>(OH); a.OW = static_cast<int>(OW);
  a.R = static_cast<int>(R); a.S = static_cast<int>(S);
  a.stride = static_cast<int>(stride); a.pad = static_cast<int>(pad); a.Kc = static_cast<int>(Kc);
  a.G = static_cast<int>(G);
  launch_col2im(a, bf(gcol), bfw(gx), stream_now());
  return gx;
}

// channel-stacked batch norm + ReLU: x [n, G*cg, h, w]; statistics per
// (client, channel) over the n*h*w pixels; affine parameters from the fp32
// rows prm[g*ld + woff / boff + c]; running statistics [G*cg] per client
std::tuple<at::Tensor, at::Tensor, at::Tensor> cs_bn_fwd(const at::Tensor& x, const at::Tensor& prm, int64_t ld,
                                                         int64_t woff, int64_t boff, int64_t G, double eps,
                                                         double momentum,
                                                         const c10::optional<at::Tensor>& run_mean,
                                                         const c10::optional<at::Tensor>& run_var,
                                                         const c10::optional<at::Tensor>& nbt,
                                                         const c10::optional<at::Tensor>& post_add) {
  check_cl_bf16(x, "cs_bn_fwd: x");
  const uint16_t* pa = nullptr;
  if (post_add.has_value() && post_add->defined()) {  // y = relu(bn(x)) + post_add
    check_cl_bf16(*post_add, "cs_bn_fwd: post_add");
    TORCH_CHECK(post_add->sizes() == x.sizes(), "cs_bn_fwd: post_add shape");
    pa = bf(*post_add);
  }
  const int64_t C = x.size(1), M = x.size(0) * x.size(2) * x.size(3);
  TORCH_CHECK(G >= 1 && C % G == 0 && (C / G) % 8 == 0 && M >= 1, "cs_bn_fwd: G | channels, 8 | channels per client");
  const int64_t cg = C / G;
  check_rows(prm, ld, G, std::min(woff, boff), std::max(woff, boff) - std::min(woff, boff) + cg, "cs_bn_fwd: prm");
  TORCH_CHECK(M * C / 8 < (int64_t{1} << 32), "cs_bn_fwd: tensor too large");
  float* rm = nullptr;
  float* rv = nullptr;
  if (run_mean.has_value() && run_mean->defined()) {
    TORCH_CHECK(run_var.has_value() && run_var->defined(), "cs_bn_fwd: running stats together");
    for (const auto* t : {&*run_mean, &*run_var})
      TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->is_contiguous() && t->numel() == C,
                  "cs_bn_fwd: running stats fp32 [G*cg]");
    rm = run_mean->data_ptr<float>();
    rv = run_var->data_ptr<float>();
  }
  int64_t* nb = nullptr;
  if (nbt.has_value() && nbt->defined()) {
    TORCH_CHECK(nbt->is_cuda() && nbt->scalar_type() == at::kLong && nbt->numel() == 1, "cs_bn_fwd: nbt int64 []");
    nb = nbt->data_ptr<int64_t>();
  }
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  auto fo = x.options().dtype(at::kFloat);
  auto part = at::empty({bn_cs_scratch_floats(static_cast<int>(M), static_cast<int>(C))}, fo);
  auto stat = at::empty({2, C}, fo);
  auto ab = at::empty({2, C}, fo);
  auto y = at::empty_like(x, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto bits = at::empty({x.numel() / 8}, x.options().dtype(at::kByte));
  launch_bn_cs_fwd(bf(x), prm.data_ptr<float>(), ld, woff, boff, static_cast<int>(cg), static_cast<int>(M),
                   static_cast<int>(C), static_cast<float>(eps), static_cast<float>(momentum), rm, rv, nb,
                   part.data_ptr<float>(), stat.data_ptr<float>(), ab.data_ptr<float>(), bfw(y),
                   bits.data_ptr<uint8_t>(), pa, stream_now());
  return {y, stat, bits};
}

// backward of cs_bn_fwd (ReLU through the forward's bits): returns dx; the
// per-client weight / bias gradients are written to grad[g*gld + gwoff / gboff + c]
at::Tensor cs_bn_bwd(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& stat, const at::Tensor& bits,
                     const at::Tensor& prm, int64_t ld, int64_t woff, int64_t G, at::Tensor grad, int64_t gld,
                     int64_t gwoff, int64_t gboff, double beta, double alpha,
                     const c10::optional<at::Tensor>& src, int64_t sld) {
  check_cl_bf16(x, "cs_bn_bwd: x");
  check_cl_bf16(dy, "cs_bn_bwd: dy");
  TORCH_CHECK(dy.sizes() == x.sizes(), "cs_bn_bwd: dy shape");
  const int64_t C = x.size(1), M = x.size(0) * x.size(2) * x.size(3);
  TORCH_CHECK(G >= 1 && C % G == 0 && (C / G) % 8 == 0, "cs_bn_bwd: G");
  const int64_t cg = C / G;
  TORCH_CHECK(stat.is_cuda() && stat.scalar_type() == at::kFloat && stat.is_contiguous() && stat.numel() == 2 * C,
              "cs_bn_bwd: stat fp32 [2, C]");
  TORCH_CHECK(bits.is_cuda() && bits.scalar_type() == at::kByte && bits.is_contiguous() && bits.numel() == x.numel() / 8,
              "cs_bn_bwd: bits uint8 [numel / 8]");
  check_rows(prm, ld, G, woff, cg, "cs_bn_bwd: prm");
  check_rows(grad, gld, G, std::min(gwoff, gboff), std::max(gwoff, gboff) - std::min(gwoff, gboff) + cg,
             "cs_bn_bwd: grad");
  const float* sp = src_rows(src, sld, G, std::min(gwoff, gboff),
                             std::max(gwoff, gboff) - std::min(gwoff, gboff) + cg, "cs_bn_bwd: src");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  auto fo = x.options().dtype(at::kFloat);
  auto part = at::empty({bn_cs_scratch_floats(static_cast<int>(M), static_cast<int>(C))}, fo);
  auto coef = at::empty({3 * C}, fo);
  auto dx = at::empty_like(x, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  launch_bn_cs_bwd(bf(x), bf(dy), bits.data_ptr<uint8_t>(), stat.data_ptr<float>(), prm.data_ptr<float>(), ld,
                   woff, static_cast<int>(cg), static_cast<int>(M), static_cast<int>(C), part.data_ptr<float>(),
                   coef.data_ptr<float>(), grad.data_ptr<float>(), gld, gwoff, gboff, bfw(dx), stream_now(),
                   static_cast<float>(beta), static_cast<float>(alpha), sp, sld);
  return dx;
}

// channel-stacked grouped 3x3 wgrad (halo kernel) written into the per-client
// gradient rows dst[g*ld + off + (k*C + c)*9 + t]; false (nothing written)
// where the geometry has no grouped halo tiling
bool conv3x3_wgrad_rows(const at::Tensor& dy, const at::Tensor& x, int64_t G, at::Tensor dst, int64_t ld,
                        int64_t off, bool rsc, double beta, double alpha, const c10::optional<at::Tensor>& mirror,
                        const c10::optional<at::Tensor>& src, int64_t sld) {
  check_cl_bf16(dy, "conv3x3_wgrad_rows: dy");
  check_cl_bf16(x, "conv3x3_wgrad_rows: x");
  const int64_t N = x.size(0), GC = x.size(1), H = x.size(2), W = x.size(3), K = dy.size(1);
  TORCH_CHECK(dy.size(0) == N && dy.size(2) == H && dy.size(3) == W && G >= 1 && GC % G == 0 && K % G == 0,
              "conv3x3_wgrad_rows: shapes");
  const int64_t C = GC / G, kg = K / G;
  // 64-channel clients (no 64-row grouped halo tiling): pairs of clients as
  // one 128-channel group, whose diagonal 64 x 64 blocks are the two clients'
  // weight gradients (twice the MFMA work, no column image)
  const bool pairs = kg == 64 && C == 64 && G % 2 == 0;
  const int64_t kC = pairs ? 128 : C, kK = pairs ? 128 : kg;
  if (!conv3x3_wgrad_grouped_supported(static_cast<int>(H), static_cast<int>(W), static_cast<int>(K),
                                       static_cast<int>(kC), static_cast<int>(kK)))
    return false;
  check_rows(dst, ld, G, off, kg * C * 9, "conv3x3_wgrad_rows: dst");
  const float* sp = src_rows(src, sld, G, off, kg * C * 9, "conv3x3_wgrad_rows: src");
  uint16_t* mp = nullptr;
  if (mirror.has_value() && mirror->defined()) {  // bf16 rows of dst's layout
    TORCH_CHECK(mirror->is_cuda() && mirror->scalar_type() == at::kBFloat16 && mirror->is_contiguous() &&
                    mirror->numel() >= dst.numel(),
                "conv3x3_wgrad_rows: mirror bf16 like dst");
    mp = reinterpret_cast<uint16_t*>(mirror->data_ptr()) + off;
  }
  TORCH_CHECK(N * H * W * std::max(GC, K) < (int64_t{1} << 31), "conv3x3_wgrad_rows: size");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  const int P = static_cast<int>(N * H * W);
  const int splits = conv3x3_wgrad_splits(P, static_cast<int>(H), static_cast<int>(W), static_cast<int>(K),
                                          static_cast<int>(kC));
  auto slab = at::empty({splits * K * 9 * kC}, x.options().dtype(at::kFloat));
  ConvWgradArgs a;
  a.dy = bf(dy);
  a.x = bf(x);
  a.slab = slab.data_ptr<float>();
  a.P = P;
  a.H = static_cast<int>(H);
  a.W = static_cast<int>(W);
  a.C = static_cast<int>(kC);
  a.K = static_cast<int>(K);
  a.splits = splits;
  a.x_stride = static_cast<int>(GC);
  a.kg = static_cast<int>(kK);
  launch_conv3x3_wgrad_rows(a, dst.data_ptr<float>() + off, static_cast<int>(kK), ld, rsc, stream_now(),
                            pairs ? 64 : 0, static_cast<float>(beta), static_cast<float>(alpha), mp,
                            sp != nullptr ? sp + off : nullptr, sld);
  return true;
}

// rows_g[off + k*N + j] = beta rows_g + alpha sum_p A[g][k][p] B[g][p][j] with
// A [G, K, P] (unit stride along K: the channel-stacked output gradient seen
// as [G, K, P]) and B [G, P, N] (unit stride along N: a grouped column image)
// on the TN MFMA GEMM (gemm_tn.hip), the bf16 mirror of the updated rows
// written in its epilogue -- hipBLASLt's baddbmm + a cast pass re-reading the
// rows otherwise.  false (nothing written): a layout the kernel cannot read.
bool fa_bmm_rows(const at::Tensor& A, const at::Tensor& B, at::Tensor dst, int64_t ld, int64_t off, double beta,
                 double alpha, const c10::optional<at::Tensor>& mirror, int64_t small,
                 const c10::optional<at::Tensor>& src, int64_t sld, const c10::optional<at::Tensor>& ximp,
                 int64_t R, int64_t stride, int64_t pad) {
  int64_t OH = 0, OW = 0;
  if (ximp.has_value() && ximp->defined()) {
    // B = the implicit R x R / stride / pad column image of the
    // channel-stacked ximp [n, G*C, H, W] (B itself is only a [G, P, R*R*C]
    // shape carrier: any tensor of those sizes, e.g. an expanded view)
    check_cl_bf16(*ximp, "fa_bmm_rows: ximp");
    TORCH_CHECK(R >= 1 && stride >= 1 && pad >= 0, "fa_bmm_rows: geometry");
    OH = (ximp->size(2) + 2 * pad - R) / stride + 1;
    OW = (ximp->size(3) + 2 * pad - R) / stride + 1;
    const int64_t G = A.size(0), C = ximp->size(1) / G, P = ximp->size(0) * OH * OW;
    TORCH_CHECK(ximp->size(1) == G * C && B.size(0) == G && B.size(1) == P && B.size(2) == R * R * C &&
                    A.size(2) == P,
                "fa_bmm_rows: ximp shapes");
    if (C % 8 || A.stride(1) != 1 || A.size(1) % 8 || A.stride(2) % 8 || A.stride(0) % 8 ||
        reinterpret_cast<uintptr_t>(A.data_ptr()) % 16 || ld % 4 || off % 4)
      return false;
  }
  TORCH_CHECK(A.is_cuda() && B.is_cuda() && A.scalar_type() == at::kBFloat16 && B.scalar_type() == at::kBFloat16 &&
                  A.dim() == 3 && B.dim() == 3 && A.size(0) == B.size(0) && A.size(2) == B.size(1),
              "fa_bmm_rows: A [G, K, P], B [G, P, N] bf16");
  const int64_t G = A.size(0), K = A.size(1), P = A.size(2), N = B.size(2);
  const auto a16 = [](const at::Tensor& t) { return reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0; };
  // N % 8 != 0 (the stem's 27 columns): the 16-byte chunk loads read up to
  // round8(N) columns, which must stay inside the operand row (its padding:
  // products of the columns past N are never stored)
  const int64_t N8 = (N + 7) / 8 * 8;
  const bool imp = ximp.has_value() && ximp->defined();
  if (A.stride(1) != 1 || K % 8 || A.stride(2) % 8 || A.stride(0) % 8 || !a16(A) || ld % 4 || off % 4 ||
      (!imp && (B.stride(2) != 1 || B.stride(1) % 8 || B.stride(0) % 8 || !a16(B) ||
                (N % 8 && (N8 > B.stride(1) || N8 > B.stride(0))))))
    return false;
  check_rows(dst, ld, G, off, K * N, "fa_bmm_rows: dst");
  TORCH_CHECK(ld > 0, "fa_bmm_rows: per-client rows");
  const float* sp = src_rows(src, sld, G, off, K * N, "fa_bmm_rows: src");
  if (sp != nullptr && (sld % 4 || reinterpret_cast<uintptr_t>(sp + off) % 16)) return false;
  uint16_t* mp = nullptr;
  if (mirror.has_value() && mirror->defined()) {
    TORCH_CHECK(mirror->is_cuda() && mirror->scalar_type() == at::kBFloat16 && mirror->is_contiguous() &&
                    mirror->numel() >= dst.numel(),
                "fa_bmm_rows: mirror bf16 like dst");
    mp = reinterpret_cast<uint16_t*>(mirror->data_ptr()) + off;
  }
  TORCH_CHECK(P < (int64_t{1} << 31) && K * N < (int64_t{1} << 31), "fa_bmm_rows: size");
  if (G == 0 || K == 0 || N == 0) return true;
  if (P == 0) return false;  // (the launcher skips T = 0: the decay alone is the caller's)
  c10::hip::HIPGuardMasqueradingAsCUDA guard(A.device());
  GemmTnArgs g{};
  g.A = bf(A);
  g.lda = A.stride(2);
  g.sa = A.stride(0);
  g.B = bf(B);
  g.ldb = B.stride(1);
  g.sb = B.stride(0);
  g.C = dst.data_ptr<float>() + off;
  g.ldc = N;
  g.cg = ld;
  g.M = static_cast<int>(K);
  g.N = static_cast<int>(N);
  g.T = static_cast<int>(P);
  g.G = static_cast<int>(G);
  g.splits = 1;  // G clients x tiles: the chip is usually full without split-K
  g.beta = static_cast<float>(beta);
  g.alpha = static_cast<float>(alpha);
  g.mirror = mp;
  g.mcg = ld;
  g.src = sp != nullptr ? sp + off : nullptr;
  g.scg = sld;
  if (ximp.has_value() && ximp->defined()) {
    g.B = bf(*ximp);
    g.ldb = ximp->size(1);  // G * C channels per pixel row
    g.sb = ximp->size(1) / G;
    g.imp_C = static_cast<int>(ximp->size(1) / G);
    g.imp_H = static_cast<int>(ximp->size(2));
    g.imp_W = static_cast<int>(ximp->size(3));
    g.imp_OH = static_cast<int>(OH);
    g.imp_OW = static_cast<int>(OW);
    g.imp_R = static_cast<int>(R);
    g.imp_s = static_cast<int>(stride);
    g.imp_pad = static_cast<int>(pad);
  }
  g.small = static_cast<int>(small);
  g.stage = (small == 1 || small == -2) ? 1 : 0;
  if (small == -2) g.small = 1;
  g.nt = 1;  // (streamed rows: nontemporal stores, 30.55 vs 30.64 ms per round, same-box A/B)
  if (N % 4) {  // the staged epilogue moves 16-byte row pieces: the MFMA-layout one
    g.stage = 0;
    g.small = 1;
  }
  // few tiles over long K (the stem's [64 x 27] per client over 5,120 pixels:
  // G one-tile blocks of 80 K-steps): split K over the free slots, fp32 slabs,
  // then the reduction applies the SGD step (src / beta / alpha) and the mirror
  at::Tensor slab;
  {
    static int cus = 0;
    if (cus == 0) {
      hipDeviceProp_t prop;
      int dev = 0;
      cus = 256;
      if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
        cus = prop.multiProcessorCount;
    }
    const bool sm = g.small > 0 || (g.small < 0 && (K % 256 != 0 || N % 256 != 0));
    const int64_t t = sm ? 128 : 256, slots = static_cast<int64_t>(cus) * (sm ? 2 : 1);
    const int64_t blocks = G * ((K + t - 1) / t) * ((N + t - 1) / t);
    const int64_t steps = (P + 63) / 64;
    if (2 * blocks <= slots && (N * K) % 4 == 0 && (ld % 4) == 0) {
      int64_t s = slots / blocks;
      if (s > steps / 4) s = steps / 4;
      if (s > 1) {
        slab = at::empty({G * s, K, N}, A.options().dtype(at::kFloat));
        g.slab = slab.data_ptr<float>();
        g.splits = static_cast<int>(s);
      }
    }
  }
  launch_gemm_tn_acc(g, stream_now());  // (slab: stream-ordered reuse after this call)
  return true;
}

// out_g (bf16) = A_g op(B_g) (+ beta out_g) for the G clients on the native
// MFMA GEMM (gemm.hip, group strides): A [G, M, K], B [G, N, K] (nt) or
// [G, K, N] (nn), out [G, M, N], each with unit stride along its last dim (the
// channel-stacked activations / column images and the weight rows as strided
// views).  false (nothing written): a shape or layout the kernel does not take.
bool fa_gemm(const at::Tensor& A, const at::Tensor& B, at::Tensor out, bool nn, double beta,
             const c10::optional<at::Tensor>& ximp, int64_t R, int64_t stride, int64_t pad) {
  TORCH_CHECK(A.is_cuda() && B.is_cuda() && out.is_cuda() && A.scalar_type() == at::kBFloat16 &&
                  B.scalar_type() == at::kBFloat16 && out.scalar_type() == at::kBFloat16 && A.dim() == 3 &&
                  B.dim() == 3 && out.dim() == 3,
              "fa_gemm: bf16 [G, ., .] operands");
  const int64_t G = A.size(0), M = A.size(1), K = A.size(2), N = nn ? B.size(2) : B.size(1);
  TORCH_CHECK(B.size(0) == G && out.size(0) == G && (nn ? B.size(1) : B.size(2)) == K && out.size(1) == M &&
                  out.size(2) == N,
              "fa_gemm: shapes");
  const auto a16 = [](const at::Tensor& t) { return reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0; };
  // ximp (NT only): A is the implicit R x R / stride / pad column image of the
  // channel-stacked ximp [n, G*C, H, W] (A: a [G, M, R*R*C] shape carrier)
  const bool imp = ximp.has_value() && ximp->defined();
  int64_t iC = 0, iOH = 0, iOW = 0;
  if (imp) {
    check_cl_bf16(*ximp, "fa_gemm: ximp");
    iC = ximp->size(1) / G;
    iOH = (ximp->size(2) + 2 * pad - R) / stride + 1;
    iOW = (ximp->size(3) + 2 * pad - R) / stride + 1;
    TORCH_CHECK(!nn && ximp->size(1) == G * iC && K == R * R * iC && M == ximp->size(0) * iOH * iOW,
                "fa_gemm: ximp geometry");
    if (iC % 64 || !a16(*ximp)) return false;
  }
  if ((!imp && (A.stride(2) != 1 || !a16(A) || A.stride(1) % 8 || A.stride(0) % 8)) || B.stride(2) != 1 ||
      out.stride(2) != 1 || !a16(B) || !a16(out) || B.stride(1) % 8 || B.stride(0) % 8 || out.stride(1) % 8 ||
      out.stride(0) % 8 || !gemm_supported(static_cast<int>(M), static_cast<int>(N), static_cast<int>(K), nn) ||
      M >= (int64_t{1} << 31))  // (element offsets are 64-bit in the kernel)
    return false;
  if (G == 0 || M == 0) return true;
  c10::hip::HIPGuardMasqueradingAsCUDA guard(A.device());
  GemmArgs g{};
  g.A = bf(A);
  g.lda = A.stride(1);
  g.B = bf(B);
  g.ldb = B.stride(1);
  g.C = out.data_ptr();
  g.ldc = out.stride(1);
  g.C2 = nullptr;
  g.bias = nullptr;
  g.M = static_cast<int>(M);
  g.N = static_cast<int>(N);
  g.K = static_cast<int>(K);
  g.beta = static_cast<float>(beta);
  g.G = static_cast<int>(G);
  g.sa = A.stride(0);
  g.sb = B.stride(0);
  g.sc = out.stride(0);
  if (imp) {
    g.A = bf(*ximp);
    g.lda = ximp->size(1);  // pixel row: G * C channels
    g.sa = iC;
    g.imp_C = static_cast<int>(iC);
    g.imp_H = static_cast<int>(ximp->size(2));
    g.imp_W = static_cast<int>(ximp->size(3));
    g.imp_OH = static_cast<int>(iOH);
    g.imp_OW = static_cast<int>(iOW);
    g.imp_R = static_cast<int>(R);
    g.imp_s = static_cast<int>(stride);
    g.imp_pad = static_cast<int>(pad);
  }
  launch_gemm(g, nn, 0, false, stream_now());
  return true;
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(commeff, m) {
  m.def("fa_gemm(Tensor A, Tensor B, Tensor(a!) out, bool nn, float beta=0., Tensor? ximp=None, int R=3, "
        "int stride=1, int pad=1) -> bool");
  m.def("fa_bmm_rows(Tensor A, Tensor B, Tensor(a!) dst, int ld, int off, float beta=1., float alpha=1., "
        "Tensor(b!)? mirror=None, int small=-1, Tensor? src=None, int sld=0, Tensor? ximp=None, int R=3, "
        "int stride=1, int pad=1) -> bool");
  m.def("fa_weight_image(Tensor W, int ld, int G, int off, int K, int C, int R, int Kc, int kind) -> Tensor");
  m.def("fa_row_sgd(Tensor(a!) W, int ld, Tensor src, int sld, Tensor G, int gld, int rows, int d, float clip, "
        "float lr, float wd, Tensor(b!)? Wb=None) -> ()");
  m.def("fa_upload(Tensor(a!) out, Tensor w0, Tensor W, int ld, int rows, float n, Tensor? perm=None) -> ()");
  m.def("fa_gather_rows(Tensor(a!) dst, Tensor(b!) dstb, Tensor src, Tensor perm) -> ()");
  m.def("fa_dgrad_image(Tensor Wb, int ld, int G, int off, int K, int C) -> Tensor");
  m.def("conv3x3_fwd_rows(Tensor x, Tensor w, int G, int off, int ld, int kg, Tensor? addend=None, "
        "bool bt=False) -> Tensor");
  m.def("fa_linear_ce(Tensor feat, int fsg, int fsn, int G, int n, Tensor W, int wld, int woff, int boff, int C, "
        "int F, float scale, Tensor y, Tensor(a!) dfeat, int dsg, int dsn, Tensor(b!) dst, int dld, float beta, "
        "float alpha, Tensor? src, int sld, Tensor(c!)? mirror, int mld, int dss=0, int ccs=0) -> (Tensor, Tensor)");
  m.def("fx_affine(Tensor x, Tensor? s, Tensor? b, Tensor? add, bool relu, Tensor? post) -> Tensor");
  m.def("fx_affine_bwd(Tensor dy, Tensor? s, Tensor? yrelu, Tensor? xs, bool want1, bool want2, Tensor? b, "
        "bool mask_x, Tensor? add2=None) -> (Tensor, Tensor, Tensor)");
  m.def("fa_affine(Tensor x, int G, bool client_major, Tensor W, int ld, int soff, int boff, Tensor? add, "
        "bool relu) -> Tensor");
  m.def("fa_affine_bwd(Tensor dy, int G, bool client_major, Tensor W, int ld, int soff, Tensor? yrelu, "
        "Tensor? xs, Tensor? add2, bool want1, bool want2) -> (Tensor, Tensor, Tensor)");
  m.def("fa_scalar_sgd(Tensor part, Tensor(a!) dst, int ld, int boff, int soff, float beta, float alpha, "
        "Tensor? src, int sld) -> ()");
  m.def("fa_head_fwd(Tensor x, int G) -> (Tensor, Tensor)");
  m.def("fa_head_bwd(Tensor df, Tensor codes, int H, int W) -> Tensor");
  m.def("fa_ew(Tensor a, Tensor? b, int mode) -> Tensor");
  m.def("im2col_grouped(Tensor x, int G, int R, int S, int stride, int pad, int Kc, bool client_major) -> Tensor");
  m.def("col2im_grouped(Tensor gcol, int G, int n, int H, int W, int C, int R, int S, int stride, int pad) -> Tensor");
  m.def("cs_bn_fwd(Tensor x, Tensor prm, int ld, int woff, int boff, int G, float eps, float momentum, "
        "Tensor(a!)? run_mean, Tensor(b!)? run_var, Tensor(c!)? nbt, Tensor? post_add=None) "
        "-> (Tensor, Tensor, Tensor)");
  m.def("cs_bn_bwd(Tensor dy, Tensor x, Tensor stat, Tensor bits, Tensor prm, int ld, int woff, int G, "
        "Tensor(a!) grad, int gld, int gwoff, int gboff, float beta=0., float alpha=1., Tensor? src=None, "
        "int sld=0) -> Tensor");
  m.def("conv3x3_wgrad_rows(Tensor dy, Tensor x, int G, Tensor(a!) dst, int ld, int off, bool rsc=False, "
        "float beta=0., float alpha=1., Tensor(b!)? mirror=None, Tensor? src=None, int sld=0) -> bool");
  m.def("fa_bcast_rows(Tensor(a!) W, int ld, Tensor src, int rows, int d) -> ()");
  m.def("fa_cast_rows(Tensor(a!) Wb, Tensor W, int ld, int rows, int off, int n) -> ()");
}

TORCH_LIBRARY_IMPL(commeff, CUDA, m) {
  m.impl("fa_weight_image", &fa_weight_image);
  m.impl("fa_bmm_rows", &fa_bmm_rows);
  m.impl("fa_gemm", &fa_gemm);
  m.impl("fa_row_sgd", &fa_row_sgd);
  m.impl("fa_upload", &fa_upload);
  m.impl("fa_gather_rows", &fa_gather_rows);
  m.impl("fa_bcast_rows", &fa_bcast_rows);
  m.impl("fa_cast_rows", &fa_cast_rows);
  m.impl("fa_linear_ce", &fa_linear_ce);
  m.impl("fx_affine", &fx_affine);
  m.impl("fx_affine_bwd", &fx_affine_bwd);
  m.impl("fa_affine", &fa_affine);
  m.impl("fa_affine_bwd", &fa_affine_bwd);
  m.impl("fa_scalar_sgd", &fa_scalar_sgd);
  m.impl("fa_dgrad_image", &fa_dgrad_image);
  m.impl("conv3x3_fwd_rows", &conv3x3_fwd_rows);
  m.impl("fa_head_fwd", &fa_head_fwd);
  m.impl("fa_head_bwd", &fa_head_bwd);
  m.impl("fa_ew", &fa_ew);
  m.impl("im2col_grouped", &im2col_grouped);
  m.impl("col2im_grouped", &col2im_grouped);
  m.impl("cs_bn_fwd", &cs_bn_fwd);
  m.impl("cs_bn_bwd", &cs_bn_bwd);
  m.impl("conv3x3_wgrad_rows", &conv3x3_wgrad_rows);
}

}  // namespace commeff
