// torch.ops.commeff.mm_nt / mm_nn: the native MFMA GEMMs of csrc/gemm.hip
// (GPU) and an fp32 ATen reference with the same rounding points (CPU).
//   mm_nt(a [M,K], b [N,K]) = a b^T        mm_nn(a [M,K], b [K,N]) = a b
//   + bias[N] (fp32), + beta * out (in place into ``out``), act 1: tanh-GELU
//   with the bf16 pre-activation written to ``pre``.
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <torch/library.h>

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

}  // namespace
}  // namespace commeff

TORCH_LIBRARY_FRAGMENT(commeff, m) {
  m.def("mm_nt(Tensor a, Tensor b, Tensor? bias=None, Tensor(c!)? out=None, float beta=0.0, int act=0, "
        "Tensor(d!)? pre=None) -> Tensor");
  m.def("mm_nn(Tensor a, Tensor b, Tensor? bias=None, Tensor(c!)? out=None, float beta=0.0, int act=0, "
        "Tensor(d!)? pre=None) -> Tensor");
}

TORCH_LIBRARY_IMPL(commeff, CPU, m) {
  m.impl("mm_nt", &commeff::mm_nt);
  m.impl("mm_nn", &commeff::mm_nn);
}

TORCH_LIBRARY_IMPL(commeff, CUDA, m) {
  m.impl("mm_nt", &commeff::mm_nt);
  m.impl("mm_nn", &commeff::mm_nn);
}
