// Microbenchmark: cost of a wave64 VALU instruction kind at 4 waves/SIMD (throughput, 8
// independent chains per iteration, inline asm so nothing folds).  Prints ns per
// wave-instruction per SIMD.  Used to choose the ring placement's byte-shift instruction.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#define ITERS 4096
template <int OP>
__global__ void __launch_bounds__(256) kb(uint32_t* out, uint32_t seed) {
  uint32_t a[16];
  for (int i = 0; i < 16; i++) a[i] = seed * (i + 3) + threadIdx.x;
  uint32_t s = (threadIdx.x & 3) * 8;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int k = 0; k < 8; k++) {
      if (OP == 0) asm volatile("v_lshlrev_b64 %0, %1, %0" : "+v"(*(uint64_t*)&a[2 * k]) : "v"(s));
      if (OP == 1) asm volatile("v_perm_b32 %0, %1, %0, %2" : "+v"(a[2 * k]) : "v"(a[2 * k + 1]), "v"(s));
      if (OP == 2) asm volatile("v_add_u32 %0, %1, %0" : "+v"(a[2 * k]) : "v"(a[2 * k + 1]));
      if (OP == 3) asm volatile("v_alignbit_b32 %0, %1, %0, %2" : "+v"(a[2 * k]) : "v"(a[2 * k + 1]), "v"(s));
      if (OP == 4) asm volatile("v_lshl_or_b32 %0, %1, %2, %0" : "+v"(a[2 * k]) : "v"(a[2 * k + 1]), "v"(s));
      if (OP == 5) asm volatile("v_lshrrev_b64 %0, %1, %0" : "+v"(*(uint64_t*)&a[2 * k]) : "v"(s));
      if (OP == 6) asm volatile("v_bfe_u32 %0, %1, %2, 8" : "+v"(a[2 * k]) : "v"(a[2 * k + 1]), "v"(s));
      if (OP == 7) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[2 * k]) : "v"(a[2 * k + 1]));
    }
  }
  uint32_t x = 0;
  for (int i = 0; i < 16; i++) x ^= a[i];
  if (x == 0x12345678u) out[0] = x;
}
template <int OP>
static float run(uint32_t* d, const char* name) {
  const int grid = 256 * 4;  // 4 workgroups of 4 waves per CU -> 4 waves/SIMD
  hipLaunchKernelGGL(kb<OP>, dim3(grid), dim3(256), 0, 0, d, 7u);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  for (int r = 0; r < 5; r++) hipLaunchKernelGGL(kb<OP>, dim3(grid), dim3(256), 0, 0, d, 7u + r);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  // wave-instructions per SIMD: waves per SIMD (grid*4 waves / 1024 SIMDs) * ITERS * 8 * 5 runs
  const double wi = (double)grid * 4 / 1024 * ITERS * 8 * 5;
  printf("%-16s %.3f ns per wave-instruction per SIMD\n", name, ms * 1e6 / wi);
  return ms;
}
int main() {
  uint32_t* d;
  hipMalloc(&d, 64);
  run<2>(d, "v_add_u32");
  run<1>(d, "v_perm_b32");
  run<3>(d, "v_alignbit_b32");
  run<0>(d, "v_lshlrev_b64");
  run<5>(d, "v_lshrrev_b64");
  run<4>(d, "v_lshl_or_b32");
  run<6>(d, "v_bfe_u32");
  run<7>(d, "v_cndmask_b32");
  return 0;
}
