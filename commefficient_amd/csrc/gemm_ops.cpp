// torch.ops.commeff.mm_nt / mm_nn: the native MFMA GEMMs of csrc/gemm.hip
// (GPU) and an fp32 ATen reference with the same rounding points (CPU).
//   mm_nt(a [M,K], b [N,K]) = a b^T        mm_nn(a [M,K], b [K,N]) = a b
//   + bias[N] (fp32), + beta * out (in place into ``out``), act 1: tanh-GELU
//   with the bf16 pre-activation written to ``pre``.
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <torch/library.h>

#include <algorithm>

#include "kernels.h"

namespace commeff {
namespace {

at::Tensor mm_impl(const at::Tensor& a, const at::Tensor& b, bool nn, const c10::optional<at::Tensor>& bias,
                   const c10::optional<at::Tensor>& out, double beta, int64_t act,
                   const c10::optional<at::Tensor>& pre) {
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && a.scalar_type() == at::kBFloat16 && b.scalar_type() == at::kBFloat16,
              "mm: bf16 matrices");
  TORCH_CHECK(a.stride(1) == 1 && b.stride(1) == 1, "mm: unit column stride");
  const int64_t M = a.size(0), K = a.size(1), N = nn ? b.size(1) : b.size(0);
  TORCH_CHECK((nn ? b.size(0) : b.size(1)) == K, "mm: inner dimensions differ");
  const bool has_out = out.has_value() && out->defined();
  const bool f32 = has_out && out->scalar_type() == at::kFloat;
  if (has_out)
    TORCH_CHECK(out->dim() == 2 && out->size(0) == M && out->size(1) == N && out->stride(1) == 1 &&
                    (f32 || out->scalar_type() == at::kBFloat16),
                "mm: out must be [M, N] bf16 / fp32 with unit column stride");
  if (bias.has_value() && bias->defined())
    TORCH_CHECK((bias->scalar_type() == at::kFloat || bias->scalar_type() == at::kBFloat16) &&
                    bias->is_contiguous() && bias->numel() == N,
                "mm: bias f32 / bf16 [N]");
  TORCH_CHECK(act == 0 || (act == 1 && !f32 && pre.has_value() && pre->defined() && pre->sizes() == at::IntArrayRef({M, N}) &&
                           pre->is_contiguous() && pre->scalar_type() == at::kBFloat16),
              "mm: act 1 (GELU) needs a bf16 [M, N] pre tensor and a bf16 output");
  at::Tensor C = has_out ? *out : at::empty({M, N}, a.options());
  if (!a.is_cuda()) {  // fp32 reference: one rounding at the end, as the kernel
    auto r = nn ? at::mm(a.to(at::kFloat), b.to(at::kFloat)) : at::mm(a.to(at::kFloat), b.to(at::kFloat).t());
    if (bias.has_value() && bias->defined()) r = r + bias->to(at::kFloat);
    if (beta != 0.0) r = r + beta * C.to(at::kFloat);
    if (act == 1) {
      auto p = r.to(at::kBFloat16);
      pre->copy_(p);
      r = at::gelu(p.to(at::kFloat), "tanh");
    }
    C.copy_(r);
    return C;
  }
  // NT with N not a multiple of 64 (the tied LM head): C's rows must hold the
  // 8-column chunk past N (a padded buffer), no bias / activation / beta
  const bool nedge = !nn && N % 64 != 0 && act == 0 && !(bias.has_value() && bias->defined()) && beta == 0.0 &&
                     C.stride(0) >= (N + 7) / 8 * 8 &&
                     gemm_supported_nedge(static_cast<int>(M), static_cast<int>(N), static_cast<int>(K));
  TORCH_CHECK(nedge || gemm_supported(static_cast<int>(M), static_cast<int>(N), static_cast<int>(K), nn),
              "mm: native GEMM needs N % 64 == 0 (NT: or an output whose rows hold the chunk past N) and "
              "K % 64 == 0");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(a.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(b.data_ptr()) % 16 == 0 &&
                  a.stride(0) % 8 == 0 && b.stride(0) % 8 == 0 &&
                  reinterpret_cast<uintptr_t>(C.data_ptr()) % 16 == 0 && C.stride(0) % 8 == 0 &&
                  (!bias.has_value() || !bias->defined() || reinterpret_cast<uintptr_t>(bias->data_ptr()) % 16 == 0),
              "mm: 16-byte aligned operands and row strides");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(a.device());
  GemmArgs g;
  g.A = reinterpret_cast<const uint16_t*>(a.data_ptr());
  g.lda = a.stride(0);
  g.B = reinterpret_cast<const uint16_t*>(b.data_ptr());
  g.ldb = b.stride(0);
  g.C = C.data_ptr();
  g.ldc = C.stride(0);
  g.C2 = act == 1 ? pre->data_ptr() : nullptr;
  const bool hb = bias.has_value() && bias->defined();
  g.bias = hb && bias->scalar_type() == at::kFloat ? bias->data_ptr<float>() : nullptr;
  g.bias16 = hb && bias->scalar_type() == at::kBFloat16 ? reinterpret_cast<const uint16_t*>(bias->data_ptr()) : nullptr;
  g.M = static_cast<int>(M);
  g.N = static_cast<int>(N);
  g.K = static_cast<int>(K);
  g.beta = static_cast<float>(beta);
  launch_gemm(g, nn, static_cast<int>(act), f32, c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream());
  return C;
}

at::Tensor mm_nt(const at::Tensor& a, const at::Tensor& b, const c10::optional<at::Tensor>& bias,
                 const c10::optional<at::Tensor>& out, double beta, int64_t act, const c10::optional<at::Tensor>& pre) {
  return mm_impl(a, b, false, bias, out, beta, act, pre);
}

at::Tensor mm_nn(const at::Tensor& a, const at::Tensor& b, const c10::optional<at::Tensor>& bias,
                 const c10::optional<at::Tensor>& out, double beta, int64_t act, const c10::optional<at::Tensor>& pre) {
  return mm_impl(a, b, true, bias, out, beta, act, pre);
}

// a [M, K] b [K, N] -> bf16 [M, N] for a long K and few output tiles (the tied
// LM head's dh = g W, K = 50,257, M x N = T x 768: 30 tiles): S groups of Kc
// K-steps on the grouped NN GEMM into fp32 partials (splits ~ one wave of
// 512 block slots, >= 16 K-steps each; the K tail past S Kc -- any K -- is
// folded into the reduction kernel), then one fixed-order reduction.  Only a's
// first K columns and b's first K rows are read.  CPU: the fp32 reference.
at::Tensor mm_nn_splitk(const at::Tensor& a, const at::Tensor& b, int64_t splits) {
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && a.scalar_type() == at::kBFloat16 && b.scalar_type() == at::kBFloat16 &&
                  a.stride(1) == 1 && b.stride(1) == 1 && a.size(1) == b.size(0),
              "mm_nn_splitk: bf16 a [M, K], b [K, N] with unit column strides");
  const int64_t M = a.size(0), K = a.size(1), N = b.size(1);
  if (!a.is_cuda()) return at::mm(a.to(at::kFloat), b.to(at::kFloat)).to(at::kBFloat16);
  TORCH_CHECK(N % 64 == 0 && N >= 64 && K >= 64 && M >= 1 && a.stride(0) % 8 == 0 && b.stride(0) % 8 == 0 &&
                  reinterpret_cast<uintptr_t>(a.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(b.data_ptr()) % 16 == 0,
              "mm_nn_splitk: N % 64 == 0, K >= 64, 16-byte aligned operands and row strides");
  const int64_t steps = K / 64;
  const int64_t tiles = ((M + 127) / 128) * ((N + 127) / 128);
  int64_t S = splits > 0 ? splits : std::max<int64_t>(1, std::min<int64_t>(16, 512 / tiles));
  S = std::max<int64_t>(1, std::min<int64_t>(S, steps / 16 > 0 ? steps / 16 : 1));
  const int64_t Kc = (steps / S) * 64, Kmain = S * Kc;
  c10::hip::HIPGuardMasqueradingAsCUDA guard(a.device());
  const hipStream_t st = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
  auto part = at::empty({S, M, N}, a.options().dtype(at::kFloat));
  auto out = at::empty({M, N}, a.options());
  GemmArgs g{};
  g.A = reinterpret_cast<const uint16_t*>(a.data_ptr());
  g.lda = a.stride(0);
  g.B = reinterpret_cast<const uint16_t*>(b.data_ptr());
  g.ldb = b.stride(0);
  g.C = part.data_ptr();
  g.ldc = N;
  g.M = static_cast<int>(M);
  g.N = static_cast<int>(N);
  g.K = static_cast<int>(Kc);
  g.beta = 0.f;
  g.G = static_cast<int>(S);
  g.sa = Kc;
  g.sb = Kc * b.stride(0);
  g.sc = M * N;
  launch_gemm(g, true, 0, true, st);
  launch_splitk_tail(part.data_ptr<float>(), static_cast<int>(S), static_cast<int>(M), static_cast<int>(N),
                     g.A, a.stride(0), g.B, b.stride(0), static_cast<int>(Kmain), static_cast<int>(K),
                     reinterpret_cast<uint16_t*>(out.data_ptr()), N, st);
  return out;
}

// (a b^T bf16 [M, N], tile moments fp32 [ceil(M / 128), 4, N]): the forward
// of a conv feeding a ghost batch norm of G groups of M / G rows, with the
// norm's per-128-row-tile mean / M2 (split at group boundaries) written by the
// GEMM epilogue (GemmArgs::stats).  CPU: the same quantities from the fp32
// reference's bf16-rounded output.
std::tuple<at::Tensor, at::Tensor> mm_nt_bnstats(const at::Tensor& a, const at::Tensor& b, int64_t G) {
  const int64_t M = a.size(0), N = b.size(0);
  TORCH_CHECK(G >= 1 && M % G == 0 && M / G >= kBnStatTile, "mm_nt_bnstats: G | M with >= 128 rows per group");
  const int64_t Mg = M / G, T = (M + kBnStatTile - 1) / kBnStatTile;
  // every tile writes all four rows of its statistics (slot 1 zero when it
  // holds one group)
  auto stats = a.is_cuda() ? at::empty({T, 4, N}, a.options().dtype(at::kFloat))
                           : at::zeros({T, 4, N}, a.options().dtype(at::kFloat));
  if (!a.is_cuda()) {
    auto y = mm_impl(a, b, false, c10::nullopt, c10::nullopt, 0.0, 0, c10::nullopt);
    auto yf = y.to(at::kFloat);
    for (int64_t t = 0; t < T; ++t) {
      const int64_t r0 = t * kBnStatTile, r1 = std::min(M, r0 + kBnStatTile);
      const int64_t rb = std::min(r1, (r0 / Mg + 1) * Mg);
      const int64_t bounds[3] = {r0, rb, r1};
      for (int slot = 0; slot < 2; ++slot) {
        if (bounds[slot + 1] <= bounds[slot]) continue;
        auto blk = yf.slice(0, bounds[slot], bounds[slot + 1]);
        auto mean = blk.mean(0);
        stats[t][2 * slot].copy_(mean);
        stats[t][2 * slot + 1].copy_((blk - mean).pow(2).sum(0));
      }
    }
    return {y, stats};
  }
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && a.scalar_type() == at::kBFloat16 && b.scalar_type() == at::kBFloat16 &&
                  a.stride(1) == 1 && b.stride(1) == 1 && b.size(1) == a.size(1),
              "mm_nt_bnstats: bf16 [M, K] x [N, K] with unit column stride");
  const int64_t K = a.size(1);
  TORCH_CHECK(gemm_supported(static_cast<int>(M), static_cast<int>(N), static_cast<int>(K), false),
              "mm_nt_bnstats: native GEMM needs N % 64 == 0 and K % 64 == 0");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(a.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(b.data_ptr()) % 16 == 0 &&
                  a.stride(0) % 8 == 0 && b.stride(0) % 8 == 0,
              "mm_nt_bnstats: 16-byte aligned operands and row strides");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(a.device());
  auto C = at::empty({M, N}, a.options());
  GemmArgs g;
  g.A = reinterpret_cast<const uint16_t*>(a.data_ptr());
  g.lda = a.stride(0);
  g.B = reinterpret_cast<const uint16_t*>(b.data_ptr());
  g.ldb = b.stride(0);
  g.C = C.data_ptr();
  g.ldc = C.stride(0);
  g.C2 = nullptr;
  g.bias = nullptr;
  g.M = static_cast<int>(M);
  g.N = static_cast<int>(N);
  g.K = static_cast<int>(K);
  g.beta = 0.f;
  g.stats = stats.data_ptr<float>();
  g.stats_mg = static_cast<int>(Mg);
  launch_gemm(g, false, 0, false, c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream());
  return {C, stats};
}

// (y bf16 [n OH OW, K], tile moments fp32 [ceil(M / 128), 4, K] or empty when
// G == 0): the R x R / stride / pad conv of the channels-last bf16 x [n, C, H,
// W] against its (r, s, c) weight image w [K, R R C] as the native NT GEMM
// with the column image gathered per tap from x (GemmArgs::imp_*, no im2col
// pass), the BN moments of mm_nt_bnstats in the epilogue when G >= 1.
std::tuple<at::Tensor, at::Tensor> conv_nt_imp(const at::Tensor& x, const at::Tensor& w, int64_t R, int64_t stride,
                                               int64_t pad, int64_t G) {
  TORCH_CHECK(x.is_cuda() && w.is_cuda() && x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16 &&
                  x.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast) && w.dim() == 2 &&
                  w.stride(1) == 1,
              "conv_nt_imp: channels-last bf16 x, bf16 [K, R R C] w");
  const int64_t n = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3), K = w.size(0);
  TORCH_CHECK(R >= 1 && stride >= 1 && pad >= 0 && pad < R && C % 64 == 0 && w.size(1) == R * R * C,
              "conv_nt_imp: geometry (C % 64 == 0, w [K, R R C])");
  const int64_t OH = (H + 2 * pad - R) / stride + 1, OW = (W + 2 * pad - R) / stride + 1, M = n * OH * OW;
  TORCH_CHECK(OH >= 1 && OW >= 1 && M < (int64_t{1} << 31), "conv_nt_imp: output size");
  TORCH_CHECK(gemm_supported(static_cast<int>(M), static_cast<int>(K), static_cast<int>(R * R * C), false),
              "conv_nt_imp: native GEMM needs K % 64 == 0");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(w.data_ptr()) % 16 == 0 &&
                  w.stride(0) % 8 == 0,
              "conv_nt_imp: 16-byte aligned operands and row strides");
  TORCH_CHECK(G == 0 || (M % G == 0 && M / G >= kBnStatTile), "conv_nt_imp: G | M with >= 128 rows per group");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  auto y = at::empty({M, K}, x.options());
  at::Tensor stats;
  GemmArgs g{};
  g.A = reinterpret_cast<const uint16_t*>(x.data_ptr());
  g.lda = C;  // pixel row
  g.B = reinterpret_cast<const uint16_t*>(w.data_ptr());
  g.ldb = w.stride(0);
  g.C = y.data_ptr();
  g.ldc = K;
  g.C2 = nullptr;
  g.bias = nullptr;
  g.M = static_cast<int>(M);
  g.N = static_cast<int>(K);
  g.K = static_cast<int>(R * R * C);
  g.beta = 0.f;
  g.imp_C = static_cast<int>(C);
  g.imp_H = static_cast<int>(H);
  g.imp_W = static_cast<int>(W);
  g.imp_OH = static_cast<int>(OH);
  g.imp_OW = static_cast<int>(OW);
  g.imp_R = static_cast<int>(R);
  g.imp_s = static_cast<int>(stride);
  g.imp_pad = static_cast<int>(pad);
  if (G >= 1) {
    stats = at::empty({(M + kBnStatTile - 1) / kBnStatTile, 4, K}, x.options().dtype(at::kFloat));
    g.stats = stats.data_ptr<float>();
    g.stats_mg = static_cast<int>(M / G);
  } else {
    stats = at::empty({0}, x.options().dtype(at::kFloat));
  }
  launch_gemm(g, false, 0, false, c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream());
  return {y, stats};
}

}  // namespace
}  // namespace commeff

TORCH_LIBRARY_FRAGMENT(commeff, m) {
  m.def("mm_nt(Tensor a, Tensor b, Tensor? bias=None, Tensor(c!)? out=None, float beta=0.0, int act=0, "
        "Tensor(d!)? pre=None) -> Tensor");
  m.def("mm_nn(Tensor a, Tensor b, Tensor? bias=None, Tensor(c!)? out=None, float beta=0.0, int act=0, "
        "Tensor(d!)? pre=None) -> Tensor");
  m.def("mm_nt_bnstats(Tensor a, Tensor b, int G) -> (Tensor, Tensor)");
  m.def("mm_nn_splitk(Tensor a, Tensor b, int splits=0) -> Tensor");
  m.def("conv_nt_imp(Tensor x, Tensor w, int R, int stride, int pad, int G) -> (Tensor, Tensor)");
}

TORCH_LIBRARY_IMPL(commeff, CPU, m) {
  m.impl("mm_nt", &commeff::mm_nt);
  m.impl("mm_nn", &commeff::mm_nn);
  m.impl("mm_nt_bnstats", &commeff::mm_nt_bnstats);
  m.impl("mm_nn_splitk", &commeff::mm_nn_splitk);
}

TORCH_LIBRARY_IMPL(commeff, CUDA, m) {
  m.impl("mm_nt", &commeff::mm_nt);
  m.impl("mm_nn", &commeff::mm_nn);
  m.impl("mm_nt_bnstats", &commeff::mm_nt_bnstats);
  m.impl("mm_nn_splitk", &commeff::mm_nn_splitk);
  m.impl("conv_nt_imp", &commeff::conv_nt_imp);
}
