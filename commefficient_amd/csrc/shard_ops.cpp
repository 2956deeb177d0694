// torch.ops.commeff registrations of the sharded-server k-list helpers
// (csrc/shard.hip): topk_pack, merge_packed, gather_i64 -- HIP kernels on the
// GPU, the same semantics in plain ATen on the CPU (the gloo rehearsal) -- and
// the per-round host staging copy host_read_copy (csrc/hostcopy.hip).
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <torch/library.h>

#include "kernels.h"

namespace commeff {
namespace {

hipStream_t stream_now() { return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

void check_pack_args(const at::Tensor& idx, const at::Tensor& vals) {
  TORCH_CHECK(idx.scalar_type() == at::kLong && idx.is_contiguous() && vals.scalar_type() == at::kFloat &&
                  vals.is_contiguous() && idx.numel() == vals.numel() && idx.device() == vals.device(),
              "topk_pack: idx int64 and vals f32 of one length");
}

at::Tensor topk_pack_cpu(const at::Tensor& idx, const at::Tensor& vals, const c10::optional<at::Tensor>& cmap,
                         int64_t m) {
  check_pack_args(idx, vals);
  auto g = idx;
  if (cmap.has_value() && cmap->defined()) {
    auto q = idx.div(m, "floor");
    g = cmap->to(at::kLong).index_select(0, q).mul(m).add(idx - q * m);
  }
  auto bits = vals.view(at::kInt).to(at::kLong).bitwise_and(0xffffffffLL);
  return g.bitwise_left_shift(32).bitwise_or(bits);
}

at::Tensor topk_pack_hip(const at::Tensor& idx, const at::Tensor& vals, const c10::optional<at::Tensor>& cmap,
                         int64_t m) {
  check_pack_args(idx, vals);
  const int32_t* cm = nullptr;
  if (cmap.has_value() && cmap->defined()) {
    TORCH_CHECK(cmap->scalar_type() == at::kInt && cmap->is_contiguous() && cmap->device() == idx.device() && m >= 1,
                "topk_pack: cmap must be int32 on the device, m >= 1");
    cm = cmap->data_ptr<int32_t>();
  }
  c10::hip::HIPGuardMasqueradingAsCUDA guard(idx.device());
  auto out = at::empty_like(idx);
  launch_topk_pack(idx.data_ptr<int64_t>(), vals.data_ptr<float>(), idx.numel(), cm, m, out.data_ptr<int64_t>(),
                   stream_now());
  return out;
}

void check_merge_args(const at::Tensor& allp, int64_t nl, int64_t k) {
  TORCH_CHECK(allp.scalar_type() == at::kLong && allp.is_contiguous() && allp.numel() == nl * k && nl >= 1,
              "merge_packed: allp must be int64 [nl * k]");
}

std::tuple<at::Tensor, at::Tensor> merge_packed_cpu(const at::Tensor& allp, int64_t nl, int64_t k) {
  check_merge_args(allp, nl, k);
  auto key = allp.bitwise_right_shift(32).bitwise_and(0xffffffffLL);
  auto order = std::get<1>(key.sort(/*stable=*/true, /*dim=*/0, /*descending=*/false));
  auto sp = allp.index_select(0, order);
  auto vals = sp.bitwise_and(0xffffffffLL).to(at::kInt).view(at::kFloat).contiguous();
  return {vals, key.index_select(0, order)};
}

std::tuple<at::Tensor, at::Tensor> merge_packed_hip(const at::Tensor& allp, int64_t nl, int64_t k) {
  check_merge_args(allp, nl, k);
  TORCH_CHECK(merge_packed_supported(static_cast<int>(nl)), "merge_packed: at most 64 lists");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(allp.device());
  auto vals = at::empty({nl * k}, allp.options().dtype(at::kFloat));
  auto idx = at::empty({nl * k}, allp.options());
  launch_merge_packed(allp.data_ptr<int64_t>(), static_cast<int>(nl), k, vals.data_ptr<float>(),
                      idx.data_ptr<int64_t>(), stream_now());
  return {vals, idx};
}

at::Tensor gather_i64_cpu(const at::Tensor& src, const at::Tensor& pos) { return src.index_select(0, pos); }

at::Tensor gather_i64_hip(const at::Tensor& src, const at::Tensor& pos) {
  TORCH_CHECK(src.scalar_type() == at::kLong && pos.scalar_type() == at::kLong && src.is_contiguous() &&
                  pos.is_contiguous() && src.device() == pos.device(),
              "gather_i64: int64 tensors on one device");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(src.device());
  auto out = at::empty_like(pos);
  launch_gather_i64(src.data_ptr<int64_t>(), pos.data_ptr<int64_t>(), pos.numel(), out.data_ptr<int64_t>(),
                    stream_now());
  return out;
}

// dst (device) <- src (pinned host), read by a kernel on the current stream
// (csrc/hostcopy.hip); alignment or an unpinned source: a stream-ordered copy
void host_read_copy_hip(at::Tensor dst, const at::Tensor& src) {
  TORCH_CHECK(dst.is_cuda() && !src.is_cuda() && dst.is_contiguous() && src.is_contiguous() &&
                  dst.nbytes() == src.nbytes(),
              "host_read_copy: contiguous device dst and host src of one size");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(dst.device());
  void* dptr = nullptr;
  const bool mapped = src.is_pinned() &&
                      hipHostGetDevicePointer(&dptr, const_cast<void*>(src.data_ptr()), 0) == hipSuccess &&
                      dptr != nullptr;
  if (!mapped || reinterpret_cast<uintptr_t>(dptr) % 16 != 0 ||
      reinterpret_cast<uintptr_t>(dst.data_ptr()) % 16 != 0) {
    (void)hipGetLastError();
    dst.copy_(src, /*non_blocking=*/true);
    return;
  }
  launch_host_read_copy(dptr, dst.data_ptr(), static_cast<int64_t>(dst.nbytes()), stream_now());
}

// launch-status probe (launch.h): a launch the runtime rejects -- here more
// dynamic LDS than a CU has -- raises a RuntimeError naming the kernel, grid,
// block and LDS bytes
void launch_probe_hip(at::Tensor out, int64_t lds_bytes) {
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kInt && out.numel() >= 1, "launch_probe: int32 device out");
  launch_probe(out.data_ptr<int32_t>(), static_cast<uint32_t>(lds_bytes), stream_now());
}

// CPU tensor: only on a machine without a HIP device, where the launch itself
// must fail -- the same checked path, observable in the CPU test suite
void launch_probe_cpu(at::Tensor out, int64_t lds_bytes) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  (void)hipGetLastError();
  TORCH_CHECK(n == 0, "launch_probe: pass a device tensor on a machine with a GPU");
  launch_probe(nullptr, static_cast<uint32_t>(lds_bytes), nullptr);
}

}  // namespace
}  // namespace commeff

TORCH_LIBRARY_FRAGMENT(commeff, m) {
  m.def("launch_probe(Tensor(a!) out, int lds_bytes) -> ()");
  m.def("host_read_copy(Tensor(a!) dst, Tensor src) -> ()");
  m.def("topk_pack(Tensor idx, Tensor vals, Tensor? cmap=None, int m=1) -> Tensor");
  m.def("merge_packed(Tensor allp, int nl, int k) -> (Tensor, Tensor)");
  m.def("gather_i64(Tensor src, Tensor pos) -> Tensor");
}

TORCH_LIBRARY_IMPL(commeff, CPU, m) {
  m.impl("topk_pack", &commeff::topk_pack_cpu);
  m.impl("merge_packed", &commeff::merge_packed_cpu);
  m.impl("gather_i64", &commeff::gather_i64_cpu);
  m.impl("host_read_copy", [](at::Tensor dst, const at::Tensor& src) { dst.copy_(src); });
  m.impl("launch_probe", &commeff::launch_probe_cpu);
}

TORCH_LIBRARY_IMPL(commeff, CUDA, m) {
  m.impl("topk_pack", &commeff::topk_pack_hip);
  m.impl("merge_packed", &commeff::merge_packed_hip);
  m.impl("gather_i64", &commeff::gather_i64_hip);
  m.impl("host_read_copy", &commeff::host_read_copy_hip);
  m.impl("launch_probe", &commeff::launch_probe_hip);
}
