// Launch tapes (csrc/launch.h): record the native kernel launches of one
// federated round and replay them from C++ (parallel/tape.py drives this).
//
//   tape_begin()             start recording (every COMMEFF_LAUNCH / tape_memset
//                            is appended to a new tape; launches still execute,
//                            or are captured when the stream is capturing)
//   tape_end() -> id         stop recording, keep the tape
//   tape_replay(id, side)    re-issue the recorded launches on the current stream
//                            (lane-1 launches on stream ``side``, see launch.h)
//   tape_fork(side), tape_join()
//                            record a fork onto / a join from the side stream
//   tape_forks(id)           forks in a tape
//   tape_size(id), tape_free(id)
//   graph_node_counts(g)     [kernel, memcpy, memset, other] nodes of a captured
//                            hipGraph_t (torch.cuda.CUDAGraph.raw_cuda_graph()):
//                            the completeness check of a tape recorded under
//                            stream capture; then [roots, max dependencies,
//                            max dependents] (a single chain: <= 1 each)
//
// Replaces the per-round Python enqueue of the reference's worker loop
// (/root/reference/CommEfficient/fed_worker.py:26-138) and server step
// (fed_aggregator.py:429-613) for rounds of fixed geometry.
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <hip/hip_runtime_api.h>
#include <torch/library.h>

#include <algorithm>
#include <atomic>
#include <map>
#include <memory>
#include <mutex>
#include <vector>

#include "launch.h"

namespace commeff {

namespace {
std::atomic<LaunchTape*> g_active{nullptr};
std::atomic<hipStream_t> g_side{nullptr};
std::mutex g_mu;
std::map<int64_t, std::unique_ptr<LaunchTape>> g_tapes;
int64_t g_next = 1;
std::unique_ptr<LaunchTape> g_recording;

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }
}  // namespace

LaunchTape* tape_active() { return g_active.load(std::memory_order_acquire); }
hipStream_t tape_side_stream() { return g_side.load(std::memory_order_acquire); }

namespace {

void tape_begin() {
  std::lock_guard<std::mutex> lk(g_mu);
  TORCH_CHECK(!g_recording, "tape_begin: a tape is already recording");
  g_recording = std::make_unique<LaunchTape>();
  g_active.store(g_recording.get(), std::memory_order_release);
}

int64_t tape_end() {
  std::lock_guard<std::mutex> lk(g_mu);
  TORCH_CHECK(g_recording, "tape_end: no tape is recording");
  TORCH_CHECK(!g_recording->open, "tape_end: a fork onto the side stream was not joined");
  g_active.store(nullptr, std::memory_order_release);
  g_side.store(nullptr, std::memory_order_release);
  const int64_t id = g_next++;
  g_tapes[id] = std::move(g_recording);
  return id;
}

LaunchTape* get(int64_t id) {
  auto it = g_tapes.find(id);
  TORCH_CHECK(it != g_tapes.end(), "unknown launch tape ", id);
  return it->second.get();
}

// (recording only; the eager fork / join is the caller's stream wait)
void tape_fork(int64_t side) {
  LaunchTape* t = tape_active();
  if (t == nullptr) return;
  TORCH_CHECK(side != 0, "tape_fork: no side stream");
  const hipStream_t hs = reinterpret_cast<hipStream_t>(static_cast<intptr_t>(side));
  const hipStream_t prev = g_side.load(std::memory_order_acquire);
  TORCH_CHECK(prev == nullptr || prev == hs, "tape_fork: one side stream per tape");
  g_side.store(hs, std::memory_order_release);
  t->ops.emplace_back([](hipStream_t) {});
  t->lane.push_back(2);
  t->forks += 1;
  t->open = true;
}

void tape_join() {
  LaunchTape* t = tape_active();
  if (t == nullptr || !t->open) return;
  t->ops.emplace_back([](hipStream_t) {});
  t->lane.push_back(3);
  t->open = false;
}

void tape_replay(int64_t id, int64_t side) {
  LaunchTape* t;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    t = get(id);
  }
  const hipStream_t s = cur_stream();
  if (t->forks == 0) {
    for (auto& op : t->ops) op(s);
    return;
  }
  TORCH_CHECK(side != 0, "tape_replay: the tape forks onto a side stream; pass one");
  const hipStream_t ss = reinterpret_cast<hipStream_t>(static_cast<intptr_t>(side));
  TORCH_CHECK(ss != s, "tape_replay: the side stream is the replaying stream");
  if (t->events.empty()) {
    size_t n = 0;
    for (uint8_t l : t->lane) n += l >= 2;
    t->events.assign(n, nullptr);
    for (auto& e : t->events)
      TORCH_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess, "hipEventCreate failed");
  }
  size_t ev = 0;
  for (size_t i = 0; i < t->ops.size(); ++i) {
    switch (t->lane[i]) {
      case 0: t->ops[i](s); break;
      case 1: t->ops[i](ss); break;
      default: {
        const bool fork = t->lane[i] == 2;
        hipEvent_t e = t->events[ev++];
        TORCH_CHECK(hipEventRecord(e, fork ? s : ss) == hipSuccess, "tape_replay: hipEventRecord failed");
        TORCH_CHECK(hipStreamWaitEvent(fork ? ss : s, e, 0) == hipSuccess, "tape_replay: hipStreamWaitEvent failed");
      }
    }
  }
}

int64_t tape_forks(int64_t id) {
  std::lock_guard<std::mutex> lk(g_mu);
  return get(id)->forks;
}

int64_t tape_size(int64_t id) {  // launches + memsets (not forks / joins)
  std::lock_guard<std::mutex> lk(g_mu);
  const LaunchTape* t = get(id);
  int64_t n = 0;
  for (uint8_t l : t->lane) n += l < 2;
  return n;
}

void tape_free(int64_t id) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_tapes.erase(id);
}

std::vector<int64_t> graph_node_counts(int64_t graph) {
  hipGraph_t g = reinterpret_cast<hipGraph_t>(static_cast<intptr_t>(graph));
  size_t n = 0;
  TORCH_CHECK(hipGraphGetNodes(g, nullptr, &n) == hipSuccess, "hipGraphGetNodes failed");
  std::vector<hipGraphNode_t> nodes(n);
  if (n > 0) TORCH_CHECK(hipGraphGetNodes(g, nodes.data(), &n) == hipSuccess, "hipGraphGetNodes failed");
  std::vector<int64_t> cnt(4, 0);
  for (size_t i = 0; i < n; ++i) {
    hipGraphNodeType ty;
    TORCH_CHECK(hipGraphNodeGetType(nodes[i], &ty) == hipSuccess, "hipGraphNodeGetType failed");
    switch (ty) {
      case hipGraphNodeTypeKernel: ++cnt[0]; break;
      case hipGraphNodeTypeMemcpy: ++cnt[1]; break;
      case hipGraphNodeTypeMemset: ++cnt[2]; break;
      case hipGraphNodeTypeEmpty: break;  // capture joins / forks
      default: ++cnt[3]; break;
    }
  }
  // the dependency shape: a tape replays its launches in order on the streams
  // they were recorded on, without cross-stream waits, so only a single chain
  // (one root, no node with two dependencies or two dependents) replays the
  // captured order exactly
  int64_t roots = 0, max_in = 0, max_out = 0;
  for (size_t i = 0; i < n; ++i) {
    size_t din = 0, dout = 0;
    TORCH_CHECK(hipGraphNodeGetDependencies(nodes[i], nullptr, &din) == hipSuccess,
                "hipGraphNodeGetDependencies failed");
    TORCH_CHECK(hipGraphNodeGetDependentNodes(nodes[i], nullptr, &dout) == hipSuccess,
                "hipGraphNodeGetDependentNodes failed");
    roots += din == 0;
    max_in = std::max<int64_t>(max_in, static_cast<int64_t>(din));
    max_out = std::max<int64_t>(max_out, static_cast<int64_t>(dout));
  }
  cnt.push_back(roots);
  cnt.push_back(max_in);
  cnt.push_back(max_out);
  return cnt;
}

// t.zero_() through the tape (a recorded round may clear buffers)
void zero_(at::Tensor t) {
  TORCH_CHECK(t.is_contiguous(), "zero_: contiguous tensors only");
  if (t.numel() == 0) return;
  if (t.is_cuda()) {
    tape_memset(t.data_ptr(), 0, t.numel() * t.element_size(), cur_stream());
  } else {
    t.zero_();
  }
}

}  // namespace
}  // namespace commeff

TORCH_LIBRARY_FRAGMENT(commeff, m) {
  m.def("zero_(Tensor(a!) t) -> ()", &commeff::zero_);
  m.def("tape_begin() -> ()", &commeff::tape_begin);
  m.def("tape_end() -> int", &commeff::tape_end);
  m.def("tape_replay(int id, int side=0) -> ()", &commeff::tape_replay);
  m.def("tape_fork(int side) -> ()", &commeff::tape_fork);
  m.def("tape_join() -> ()", &commeff::tape_join);
  m.def("tape_forks(int id) -> int", &commeff::tape_forks);
  m.def("tape_size(int id) -> int", &commeff::tape_size);
  m.def("tape_free(int id) -> ()", &commeff::tape_free);
  m.def("graph_node_counts(int graph) -> int[]", &commeff::graph_node_counts);
}
