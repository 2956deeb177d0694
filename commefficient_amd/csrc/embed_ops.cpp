// torch.ops.commeff registrations of the GPT-2 input embedding
// (csrc/embed.hip, ops/transformer.py _Embed).  GPU only: the CPU path is the
// HF modules' own embedding.
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <torch/library.h>

#include "kernels.h"

namespace commeff {

void launch_embed_fwd(const int64_t* ids, const int64_t* tt, const int32_t* tok, int L, const uint16_t* wte,
                      const uint16_t* wpe, uint16_t* out, int Mr, int H, hipStream_t stream);
void launch_embed_bwd(const uint16_t* de, const int64_t* ids, const int64_t* tt, const int32_t* tok, int L,
                      int pos, unsigned long long* acc, float* spill, int32_t* cnt, int32_t* lst, int V, int H,
                      float* sink, int64_t ld, int Mr, hipStream_t stream);

namespace {

hipStream_t stream_now() { return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

void check_ids(const at::Tensor& t, int64_t M, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kLong && t.is_contiguous() && t.numel() == M, name,
              " must be contiguous int64 [M] on the device");
}

const int32_t* tok_ptr(const c10::optional<at::Tensor>& tok, int64_t M, int64_t* Mr) {
  if (!tok.has_value() || !tok->defined()) {
    *Mr = M;
    return nullptr;
  }
  TORCH_CHECK(tok->is_cuda() && tok->scalar_type() == at::kInt && tok->is_contiguous() && tok->numel() <= M,
              "embed: tok must be contiguous int32 [Mr <= M] real-token positions");
  *Mr = tok->numel();
  return tok->data_ptr<int32_t>();
}

// e [Mr, H] bf16 = wte[ids[t]] + wpe[t % L] (+ wte[tt[t]]), t = tok[r] (or r)
at::Tensor embed_fwd(const at::Tensor& ids, const c10::optional<at::Tensor>& tt, const c10::optional<at::Tensor>& tok,
                     int64_t L, const at::Tensor& wte, const at::Tensor& wpe) {
  const int64_t M = ids.numel();
  check_ids(ids, M, "embed_fwd: ids");
  if (tt.has_value() && tt->defined()) check_ids(*tt, M, "embed_fwd: tt");
  TORCH_CHECK(wte.scalar_type() == at::kBFloat16 && wpe.scalar_type() == at::kBFloat16 && wte.is_contiguous() &&
                  wpe.is_contiguous() && wte.dim() == 2 && wpe.dim() == 2 && wte.size(1) == wpe.size(1) &&
                  L >= 1 && L <= wpe.size(0),
              "embed_fwd: wte [V, H], wpe [>= L, H] contiguous bf16");
  int64_t Mr = 0;
  const int32_t* tp = tok_ptr(tok, M, &Mr);
  const int64_t H = wte.size(1);
  c10::hip::HIPGuardMasqueradingAsCUDA guard(ids.device());
  auto out = at::empty({Mr, H}, wte.options());
  launch_embed_fwd(ids.data_ptr<int64_t>(), (tt.has_value() && tt->defined()) ? tt->data_ptr<int64_t>() : nullptr,
                   tp, static_cast<int>(L), reinterpret_cast<const uint16_t*>(wte.data_ptr()),
                   reinterpret_cast<const uint16_t*>(wpe.data_ptr()), reinterpret_cast<uint16_t*>(out.data_ptr()),
                   static_cast<int>(Mr), static_cast<int>(H), stream_now());
  return out;
}

// sink [V, H] fp32 (row stride ld) += the table gradient of de [Mr, H]: keys
// ids[t] (+ tt[t]) (pos false) or t % L (pos true).  acc int64 [V*H], spill fp32
// [V*H], cnt int32 [V], lst int32 [V + 1]: the persistent fixed-point workspace
// and its out-of-range / non-finite spill (zero on entry, zero again on exit)
void embed_bwd(const at::Tensor& de, const at::Tensor& ids, const c10::optional<at::Tensor>& tt,
               const c10::optional<at::Tensor>& tok, int64_t L, bool pos, at::Tensor acc, at::Tensor spill,
               at::Tensor cnt, at::Tensor lst, at::Tensor sink) {
  const int64_t M = ids.numel();
  check_ids(ids, M, "embed_bwd: ids");
  const bool has_tt = !pos && tt.has_value() && tt->defined();
  if (has_tt) check_ids(*tt, M, "embed_bwd: tt");
  int64_t Mr = 0;
  const int32_t* tp = tok_ptr(tok, M, &Mr);
  TORCH_CHECK(de.is_cuda() && de.scalar_type() == at::kBFloat16 && de.is_contiguous() && de.dim() == 2 &&
                  de.size(0) == Mr,
              "embed_bwd: de must be contiguous bf16 [Mr, H]");
  const int64_t H = de.size(1);
  TORCH_CHECK(sink.is_cuda() && sink.scalar_type() == at::kFloat && sink.dim() == 2 && sink.size(1) == H &&
                  sink.stride(1) == 1,
              "embed_bwd: sink fp32 [V, H] with unit column stride");
  const int64_t V = sink.size(0);
  TORCH_CHECK(acc.scalar_type() == at::kLong && acc.is_contiguous() && acc.numel() == V * H &&
                  spill.scalar_type() == at::kFloat && spill.is_contiguous() && spill.numel() == V * H &&
                  cnt.scalar_type() == at::kInt && cnt.is_contiguous() && cnt.numel() == V &&
                  lst.scalar_type() == at::kInt && lst.is_contiguous() && lst.numel() == V + 1,
              "embed_bwd: workspace acc int64 [V*H], spill fp32 [V*H], cnt int32 [V], lst int32 [V+1]");
  TORCH_CHECK(pos ? L >= 1 && L <= V : true, "embed_bwd: positions past the table");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(de.device());
  launch_embed_bwd(reinterpret_cast<const uint16_t*>(de.data_ptr()), ids.data_ptr<int64_t>(),
                   has_tt ? tt->data_ptr<int64_t>() : nullptr, tp, static_cast<int>(L), pos ? 1 : 0,
                   reinterpret_cast<unsigned long long*>(acc.data_ptr<int64_t>()), spill.data_ptr<float>(),
                   cnt.data_ptr<int32_t>(),
                   lst.data_ptr<int32_t>(), static_cast<int>(V), static_cast<int>(H), sink.data_ptr<float>(),
                   sink.stride(0), static_cast<int>(Mr), stream_now());
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(commeff, m) {
  m.def("embed_fwd(Tensor ids, Tensor? tt, Tensor? tok, int L, Tensor wte, Tensor wpe) -> Tensor");
  m.def("embed_bwd(Tensor de, Tensor ids, Tensor? tt, Tensor? tok, int L, bool pos, Tensor(a!) acc, "
        "Tensor(b!) spill, Tensor(c!) cnt, Tensor(d!) lst, Tensor(e!) sink) -> ()");
}

TORCH_LIBRARY_IMPL(commeff, CUDA, m) {
  m.impl("embed_fwd", &embed_fwd);
  m.impl("embed_bwd", &embed_bwd);
}

}  // namespace commeff
