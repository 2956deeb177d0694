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
  TORCH_CHECK(gemm_supported(static_cast<int>(M), static_cast<int>(N), static_cast<int>(K), nn),
              "mm: native GEMM needs N % 64 == 0 and K % 64 == 0");
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

}  // namespace
}  // namespace commeff

TORCH_LIBRARY_FRAGMENT(commeff, m) {
  m.def("mm_nt(Tensor a, Tensor b, Tensor? bias=None, Tensor(c!)? out=None, float beta=0.0, int act=0, "
        "Tensor(d!)? pre=None) -> Tensor");
  m.def("mm_nn(Tensor a, Tensor b, Tensor? bias=None, Tensor(c!)? out=None, float beta=0.0, int act=0, "
        "Tensor(d!)? pre=None) -> Tensor");
  m.def("mm_nt_bnstats(Tensor a, Tensor b, int G) -> (Tensor, Tensor)");
}

TORCH_LIBRARY_IMPL(commeff, CPU, m) {
  m.impl("mm_nt", &commeff::mm_nt);
  m.impl("mm_nn", &commeff::mm_nn);
  m.impl("mm_nt_bnstats", &commeff::mm_nt_bnstats);
}

TORCH_LIBRARY_IMPL(commeff, CUDA, m) {
  m.impl("mm_nt", &commeff::mm_nt);
  m.impl("mm_nn", &commeff::mm_nn);
  m.impl("mm_nt_bnstats", &commeff::mm_nt_bnstats);
}
