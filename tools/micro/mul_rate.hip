// Microbenchmark (diagnostic only): issue cost of the integer multiplies the
// Philox rounds use (v_mad_u64_u32 vs v_mul_hi_u32 / v_mul_lo_u32) against
// plain VALU, on gfx950: 8 independent chains per wave, 1..8 waves per SIMD.
// Prints wall cycles per wave-instruction per SIMD.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

template <int MODE>
__global__ __launch_bounds__(64) void k(uint32_t* out, uint32_t m, int iters) {
  uint32_t x[8];
  uint64_t y[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { x[j] = threadIdx.x * (j + 3); y[j] = x[j]; }
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (MODE == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[j]) : "v"(m));
      if (MODE == 1) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x[j]) : "v"(m));
      if (MODE == 2) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x[j]) : "v"(m));
      if (MODE == 3) asm volatile("v_mad_u64_u32 %0, s[40:41], %1, %2, %0" : "+v"(y[j]) : "v"(x[j]), "v"(m) : "s40", "s41");
      if (MODE == 4) asm volatile("v_bitop3_b32 %0, %0, %1, %1 bitop3:0x96" : "+v"(x[j]) : "v"(m));
    }
  }
  uint32_t r = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) r ^= x[j] ^ (uint32_t)y[j] ^ (uint32_t)(y[j] >> 32);
  out[blockIdx.x * 64 + threadIdx.x] = r;
}

int main() {
  uint32_t* d;
  hipMalloc(&d, (size_t)256 * 4 * 8 * 64 * 4);
  const char* names[] = {"v_add_u32", "v_mul_hi_u32", "v_mul_lo_u32", "v_mad_u64_u32", "v_bitop3_b32"};
  void (*ks[])(uint32_t*, uint32_t, int) = {k<0>, k<1>, k<2>, k<3>, k<4>};
  const int iters = 4096;
  for (int mode = 0; mode < 5; ++mode)
    for (int wps : {1, 2, 4, 8}) {
      const int grid = 256 * 4 * wps;
      hipLaunchKernelGGL(ks[mode], dim3(grid), dim3(64), 0, 0, d, 0x9E3779B9u, 16);
      hipDeviceSynchronize();
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      hipEventRecord(e0);
      hipLaunchKernelGGL(ks[mode], dim3(grid), dim3(64), 0, 0, d, 0x9E3779B9u, iters);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double cyc = ms * 1e-3 * 2.4e9 / ((double)iters * 8 * wps);
      printf("%-14s waves/SIMD %d: %.2f cycles per wave-instruction per SIMD\n", names[mode], wps, cyc);
      fflush(stdout);
    }
  return 0;
}
