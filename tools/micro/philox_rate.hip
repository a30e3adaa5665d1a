// Microbenchmark (diagnostic only): Philox4x32-10 throughput on gfx950
// (wave-cycles per evaluation for a full wave), 64-bit-product form.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include "../../cloud-haskell-paxos_amd/csrc/paxos_device.h"

__global__ __launch_bounds__(64) void bench(uint32_t* out, uint32_t seed, int iters) {
  uint32_t acc = threadIdx.x;
  for (int i = 0; i < iters; ++i) {
    uint4 w = pxb::philox(acc, blockIdx.x, (uint32_t)i, seed, 0x1234u, 0x5678u);
    acc ^= w.x + w.y;
  }
  out[blockIdx.x * 64 + threadIdx.x] = acc;
}

int main() {
  uint32_t* d;
  const int waves = 256 * 4 * 8, iters = 4096;
  hipMalloc(&d, (size_t)waves * 64 * 4);
  hipLaunchKernelGGL(bench, dim3(waves), dim3(64), 0, 0, d, 1u, 16);
  hipDeviceSynchronize();
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(bench, dim3(waves), dim3(64), 0, 0, d, 1u, iters);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  double evals = (double)waves * iters;             // wave-level evaluations
  double simd_cycles = ms * 1e-3 * 2.4e9 * 1024;    // 1024 SIMDs
  printf("philox: %.1f SIMD-cycles per wave-evaluation (%.3f ms)\n", simd_cycles / evals, ms);
  return 0;
}
