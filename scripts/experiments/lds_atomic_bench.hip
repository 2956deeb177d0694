// LDS atomic-add throughput on gfx950: f32 vs u32 vs u64 (fixed point) at
// random addresses in an 8192-entry tile (the dense sketch encode P2 pattern).
// hipcc -O3 --offload-arch=gfx950 scripts/experiments/lds_atomic_bench.hip -o /tmp/lab
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <typename T>
__global__ void __launch_bounds__(1024) k_atomic(T* out, int iters, uint32_t seed) {
  __shared__ T tab[8192];
  for (int i = threadIdx.x; i < 8192; i += blockDim.x) tab[i] = T(0);
  __syncthreads();
  uint32_t x = seed ^ (blockIdx.x * 1024 + threadIdx.x) * 2654435761u;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      x = x * 1664525u + 1013904223u;
      atomicAdd(&tab[(x >> 8) & 8191], T(1));
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 8192; i += blockDim.x) out[blockIdx.x * 8192 + i] = tab[i];
}

template <typename T>
float run(const char* name, int blocks, int iters) {
  T* out;
  hipMalloc(&out, sizeof(T) * 8192 * blocks);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(k_atomic<T>, dim3(blocks), dim3(1024), 0, 0, out, iters, 1u);
  hipEventRecord(a);
  hipLaunchKernelGGL(k_atomic<T>, dim3(blocks), dim3(1024), 0, 0, out, iters, 7u);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  const double n = double(blocks) * 1024 * iters * 8;
  printf("%-4s %8.3f ms  %7.2f G atomics/s  %5.3f lanes/clk/CU @2.4GHz\n", name, ms, n / ms / 1e6,
         n / (ms * 1e-3) / 256 / 2.4e9);
  hipFree(out);
  return ms;
}

int main() {
  const int blocks = 256 * 4, iters = 256;
  run<float>("f32", blocks, iters);
  run<uint32_t>("u32", blocks, iters);
  run<unsigned long long>("u64", blocks, iters);
  run<float>("f32", blocks, iters);
  return 0;
}
