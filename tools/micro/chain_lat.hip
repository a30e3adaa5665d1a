// Microbenchmark (diagnostic only): issue latency of dependent instruction
// chains on gfx950, one wave per SIMD vs several.  Prints cycles per link.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

template <int MODE>
__global__ void chain(uint64_t* out, uint32_t seed, int iters) {
  uint32_t x = threadIdx.x ^ seed, y = seed * 7u;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    if (MODE == 0) {          // VALU -> VALU
      asm volatile("v_add_u32 %0, %0, %1\n v_xor_b32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(y));
    } else if (MODE == 1) {   // VALU cmp -> SALU and -> VALU cndmask (x4)
      asm volatile(
        "v_cmp_gt_u32 s[20:21], %0, %1\n s_and_b64 s[20:21], s[20:21], exec\n v_cndmask_b32 %0, %1, %0, s[20:21]\n"
        "v_cmp_gt_u32 s[20:21], %0, %1\n s_and_b64 s[20:21], s[20:21], exec\n v_cndmask_b32 %0, %1, %0, s[20:21]\n"
        : "+v"(x) : "v"(y) : "s20", "s21");
    } else if (MODE == 2) {   // VALU cmp -> VALU cndmask (vcc, no SALU) x4
      asm volatile(
        "v_cmp_gt_u32 vcc, %0, %1\n v_cndmask_b32 %0, %1, %0, vcc\n"
        "v_cmp_gt_u32 vcc, %0, %1\n v_cndmask_b32 %0, %1, %0, vcc\n"
        : "+v"(x) : "v"(y) : "vcc");
    } else if (MODE == 3) {   // VALU cmp -> SALU bcnt -> VALU add (x2)
      asm volatile(
        "v_cmp_gt_u32 s[20:21], %0, %1\n s_bcnt1_i32_b64 s22, s[20:21]\n v_add_u32 %0, s22, %0\n"
        "v_cmp_gt_u32 s[20:21], %0, %1\n s_bcnt1_i32_b64 s22, s[20:21]\n v_add_u32 %0, s22, %0\n"
        : "+v"(x) : "v"(y) : "s20", "s21", "s22");
    }
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
  if (x == 0x12345678u) out[0] = 0;   // keep x live
}

int main() {
  uint64_t* d;
  hipMalloc(&d, 4096 * 8);
  const char* names[] = {"valu x4", "cmp-sand-cndmask x2", "cmp-cndmask(vcc) x2", "cmp-sbcnt-vadd x2", "cmp-scmp-cbranch-vadd x2"};
  const int iters = 1024;
  for (int mode = 0; mode < 4; ++mode) {
    for (int wps : {1, 4, 8}) {
      // blocks of 64 threads; grid = 256 CUs * 4 SIMDs * wps waves
      int grid = 256 * 4 * wps;
      void (*k)(uint64_t*, uint32_t, int) = mode == 0 ? chain<0> : mode == 1 ? chain<1> : mode == 2 ? chain<2> : chain<3>;
      hipLaunchKernelGGL(k, dim3(grid), dim3(64), 0, 0, d, 5u, iters);
      hipDeviceSynchronize();
      hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
      hipEventRecord(e0);
      hipLaunchKernelGGL(k, dim3(grid), dim3(64), 0, 0, d, 5u, iters);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      uint64_t h[1]; hipMemcpy(h, d, 8, hipMemcpyDeviceToHost);
      // per-wave memtime delta per iteration; plus wall-clock per iteration per SIMD
      double wall_cyc = ms * 1e-3 * 2.4e9 / iters;
      printf("%-28s waves/SIMD %d: wave memtime/iter %.1f  wall cycles/iter %.1f (%.2f per wave-iter)\n",
             names[mode], wps, (double)h[0] / iters, wall_cyc, wall_cyc / wps);
      fflush(stdout);
    }
  }
  return 0;
}
