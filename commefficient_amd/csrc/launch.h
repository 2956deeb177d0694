// Kernel launches of the native extension, with an optional launch tape.
//
// Every launcher in csrc/*.hip launches through COMMEFF_LAUNCH (and clears
// memory through tape_memset).  Normally that is a plain hipLaunchKernel.
// While a launch tape is recording (tape_begin .. tape_end, driven by
// parallel/tape.py), each launch is also appended to the tape as a closure
// holding a by-value copy of the kernel's arguments (device pointers, scalars,
// argument structs), its grid, block and dynamic LDS size.  Replaying the tape
// re-issues exactly those launches, in recording order, on the caller's
// stream: a whole federated round (~45 kernels) costs the host ~45
// hipLaunchKernel calls instead of a Python pass through autograd, the
// dispatcher and the engine's bookkeeping.
//
// A tape is only valid while every buffer it points at stays where it was at
// recording time; parallel/tape.py records under a PyTorch graph-capture
// private memory pool (so intermediates keep their addresses) and checks that
// the captured HIP graph holds exactly as many kernel / memset nodes as the
// tape (no launch that bypassed COMMEFF_LAUNCH, e.g. a PyTorch kernel).
// Per-round scalars (learning rate, round index) must therefore reach the
// recorded kernels through device memory, never as launch arguments.
//
// Every launch and memset status is checked (eager, recorded and replayed
// alike): a failure raises (std::runtime_error -> Python RuntimeError through
// the op bindings) naming the kernel, its grid, block and dynamic LDS bytes,
// instead of leaving the outputs unwritten.  hipLaunchKernel's return value
// costs nothing extra; the sticky error is also cleared so a later PyTorch
// check does not report it against an unrelated op.
#pragma once
#include <hip/hip_runtime_api.h>
#include <cstdint>
#include <cstdio>
#include <functional>
#include <stdexcept>
#include <tuple>
#include <type_traits>
#include <utility>
#include <vector>

namespace commeff {

// Two lanes: a tape may fork work onto a side stream (ops/lanes.py: the conv
// weight gradients, which nothing in the backward waits for) and join it back.
// lane[i]: 0 = the replaying stream, 1 = the side stream, 2 = fork (the side
// stream waits for everything issued so far on the main one), 3 = join (the
// main stream waits for the side one); forks / joins replay as event record +
// stream wait pairs, on events created at the first replay.
struct LaunchTape {
  std::vector<std::function<void(hipStream_t)>> ops;
  std::vector<uint8_t> lane;
  std::vector<hipEvent_t> events;  // one per fork / join, lazily created
  int forks = 0;
  bool open = false;  // a fork not yet joined (recording)
  ~LaunchTape() {
    for (hipEvent_t e : events)
      if (e != nullptr) (void)hipEventDestroy(e);
  }
};

// non-null while a tape records (set/cleared by the bindings, tape.cpp)
LaunchTape* tape_active();
// the side stream of the recording (nullptr: none); a launch issued on it is
// recorded on lane 1
hipStream_t tape_side_stream();

inline void tape_push(LaunchTape* t, std::function<void(hipStream_t)> op, hipStream_t s) {
  const hipStream_t side = tape_side_stream();
  t->ops.emplace_back(std::move(op));
  t->lane.push_back(side != nullptr && s == side ? 1 : 0);
}

[[noreturn]] inline void launch_failed(const char* name, hipError_t e, dim3 g, dim3 b, uint32_t sh) {
  (void)hipGetLastError();  // clear the sticky status
  char msg[512];
  std::snprintf(msg, sizeof(msg),
                "commeff: launch of %s failed: %s (%d); grid (%u, %u, %u), block (%u, %u, %u), "
                "dynamic LDS %u bytes",
                name, hipGetErrorString(e), static_cast<int>(e), g.x, g.y, g.z, b.x, b.y, b.z, sh);
  throw std::runtime_error(msg);
}

template <typename F, typename T, size_t... I>
inline void launch_from_tuple(const char* name, F k, dim3 g, dim3 b, uint32_t sh, hipStream_t s,
                              T& args, std::index_sequence<I...>) {
  void* argv[sizeof...(I) > 0 ? sizeof...(I) : 1] = {static_cast<void*>(&std::get<I>(args))...};
  const hipError_t e = hipLaunchKernel(reinterpret_cast<const void*>(k), g, b, argv, sh, s);
  if (e != hipSuccess) launch_failed(name, e, g, b, sh);
}

template <typename... P, typename... A>
inline void tape_launch(const char* name, void (*k)(P...), dim3 g, dim3 b, uint32_t sh,
                        hipStream_t s, A&&... a) {
  static_assert(sizeof...(P) == sizeof...(A), "kernel argument count");
  using Tup = std::tuple<std::decay_t<P>...>;
  Tup args(static_cast<std::decay_t<P>>(std::forward<A>(a))...);
  if (LaunchTape* t = tape_active()) {
    tape_push(
        t,
        [name, k, g, b, sh, args](hipStream_t st) mutable {
          launch_from_tuple(name, k, g, b, sh, st, args, std::index_sequence_for<P...>{});
        },
        s);
  }
  launch_from_tuple(name, k, g, b, sh, s, args, std::index_sequence_for<P...>{});
}

inline void memset_checked(void* p, int v, size_t n, hipStream_t s) {
  const hipError_t e = hipMemsetAsync(p, v, n, s);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    char msg[256];
    std::snprintf(msg, sizeof(msg), "commeff: hipMemsetAsync of %zu bytes at %p failed: %s (%d)", n,
                  p, hipGetErrorString(e), static_cast<int>(e));
    throw std::runtime_error(msg);
  }
}

inline void tape_memset(void* p, int v, size_t n, hipStream_t s) {
  if (LaunchTape* t = tape_active()) {
    tape_push(t, [p, v, n](hipStream_t st) { memset_checked(p, v, n, st); }, s);
  }
  memset_checked(p, v, n, s);
}

}  // namespace commeff

#define COMMEFF_LAUNCH(kernel, grid, block, shmem, stream, ...) \
  ::commeff::tape_launch(#kernel, kernel, grid, block, shmem, stream, ##__VA_ARGS__)
