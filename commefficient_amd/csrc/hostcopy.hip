// Per-round host -> device staging without a copy engine or blit.
//
// The engine stages each round's small host arrays (sample positions, client
// slots, accounting metadata, the server's lr / round word: a few KB) into
// device buffers.  Through hipMemcpyAsync from pinned memory every copy is a
// runtime blit (__amd_rocclr_copyBuffer) whose dispatch waits for the queue
// to drain and for system-scope cache maintenance on both sides: 20-40 us of
// idle GPU per round in the ResNet-9 bench trace (profiles/r4_experiments.md).
// Here the compute queue's own kernel reads the pinned host slot through its
// device mapping (kernels are dispatched with a system-scope acquire, so the
// host's writes before the launch are visible) and writes the device buffer:
// one ordinary dispatch in the round's stream.
#include <hip/hip_runtime.h>
#include <cstdint>
#include "kernels.h"

namespace commeff {
namespace {

struct alignas(16) U4 {
  uint32_t w[4];
};

// 16-byte words, grid-stride; the byte tail (n % 16) by the first lanes
__global__ void __launch_bounds__(256) host_read_copy_kernel(const unsigned char* __restrict__ src,
                                                             unsigned char* __restrict__ dst, int64_t n) {
  const int64_t nw = n >> 4;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * 256;
  const int64_t t0 = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  const U4* s4 = reinterpret_cast<const U4*>(src);
  U4* d4 = reinterpret_cast<U4*>(dst);
  for (int64_t i = t0; i < nw; i += stride) d4[i] = s4[i];
  const int64_t tail = n - (nw << 4);
  if (t0 < tail) dst[(nw << 4) + t0] = src[(nw << 4) + t0];
}

// launch-status probe: writes its dynamic LDS size (checked launches, launch.h)
__global__ void __launch_bounds__(64) launch_probe_kernel(int32_t* out) {
  extern __shared__ int32_t probe_lds[];
  probe_lds[threadIdx.x] = static_cast<int32_t>(threadIdx.x);
  __syncthreads();
  if (threadIdx.x == 0) out[0] = probe_lds[63] + 1;
}

}  // namespace

void launch_probe(int32_t* out, uint32_t lds_bytes, hipStream_t stream) {
  COMMEFF_LAUNCH(launch_probe_kernel, dim3(1), dim3(64), lds_bytes, stream, out);
}

void launch_host_read_copy(const void* host_src, void* dst, int64_t n, hipStream_t stream) {
  if (n <= 0) return;
  const int64_t words = (n + 15) / 16;
  int64_t blocks = (words + 255) / 256;
  if (blocks > 64) blocks = 64;  // a few KB per round: PCIe-latency bound, not bandwidth
  COMMEFF_LAUNCH(host_read_copy_kernel, dim3(static_cast<uint32_t>(blocks)), dim3(256), 0, stream,
                 static_cast<const unsigned char*>(host_src), static_cast<unsigned char*>(dst), n);
}

}  // namespace commeff
