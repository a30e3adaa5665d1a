// valu_peak.hip — empirical wave64 integer-VALU issue ceiling of the chip, the
// roofline the batch kernel is measured against (tools/valu_roofline.py).
// Eight independent add/xor/select chains per lane, 8 waves per SIMD, so issue
// (not dependency latency) is the limit.  Reports wave-instructions per second
// counted from the loop body (16 x 8 VALU ops per iteration, checked in the
// disassembly by the caller) and per CU-cycle at the clock given on the
// command line.
//   hipcc --offload-arch=gfx950 -O3 -o valu_peak valu_peak.hip && ./valu_peak
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHK(x)                                                        \
  do {                                                                \
    hipError_t e_ = (x);                                              \
    if (e_ != hipSuccess) {                                           \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));         \
      return 1;                                                       \
    }                                                                 \
  } while (0)

template <int SEL>
__global__ __launch_bounds__(256) void valu_chains(uint32_t* out, int iters) {
  uint32_t a = threadIdx.x, b = a * 3u + 1u, c = a ^ 0x55u, d = a + 7u;
  uint32_t e = a * 5u, f = a ^ 0x99u, g = a + 11u, h = a * 9u + 3u;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      if (SEL) {   // the batch kernel's idiom: compare-free selects on a lane bit
        a = (b & 1u) ? a + c : a;
        b = (c & 2u) ? b ^ d : b;
        c = (d & 4u) ? c + e : c;
        d = (e & 8u) ? d ^ f : d;
        e = (f & 1u) ? e + g : e;
        f = (g & 2u) ? f ^ h : f;
        g = (h & 4u) ? g + a : g;
        h = (a & 8u) ? h ^ b : h;
      } else {
        a += b; b ^= c; c += d; d ^= e; e += f; f ^= g; g += h; h ^= a;
      }
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a ^ b ^ c ^ d ^ e ^ f ^ g ^ h;
}

int main(int argc, char** argv) {
  int dev = 0, cus = 0;
  CHK(hipGetDevice(&dev));
  CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const double clock_ghz = argc > 1 ? atof(argv[1]) : 2.4;
  const int blocks = cus * 8;   // 8 x 4 waves per CU = 8 waves per SIMD
  const int iters = 4000;
  uint32_t* out = nullptr;
  CHK(hipMalloc(&out, (size_t)blocks * 256 * sizeof(uint32_t)));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  for (int sel = 0; sel < 2; ++sel) {
    auto k = sel ? valu_chains<1> : valu_chains<0>;
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, 10);
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, iters);
    CHK(hipEventRecord(e1, 0));
    CHK(hipEventSynchronize(e1));
    float ms = 0.f;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    // VALU instructions per loop iteration and wave, from the gfx950
    // disassembly: add/xor 16 x 8 x 1 = 128; select 16 x 8 x 3 = 384
    // (v_bfe_i32 + v_and/v_bitop3 + v_add/v_xor per select)
    const double insts = (double)blocks * 4 * iters * (sel ? 384 : 128);
    printf("{\"kernel\": \"%s\", \"ms\": %.3f, \"G_wave_valu_insts_per_s\": %.1f, "
           "\"wave_valu_insts_per_CU_cycle\": %.3f, \"clock_GHz_assumed\": %.2f}\n",
           sel ? "select chains" : "add/xor chains", ms, insts / (ms * 1e-3) / 1e9,
           insts / (ms * 1e-3) / (cus * clock_ghz * 1e9), clock_ghz);
  }
  CHK(hipFree(out));
  return 0;
}
