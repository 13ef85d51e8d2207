// mb_addtid.hip -- where does ds_write_addtid_b32 write on gfx950?  (M0 base + offset + 4 lane?)
// Build: hipcc --offload-arch=gfx950 -O3 tools/mb_addtid.hip -o tools/mb_addtid
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k(unsigned* out, unsigned m0v) {
  __shared__ unsigned s[1024];
  for (int i = threadIdx.x; i < 1024; i += 64) s[i] = 0xFFFFFFFFu;
  __syncthreads();
  unsigned base = (unsigned)(uintptr_t)(__attribute__((address_space(3))) void*)s;
  unsigned v = 1000u + threadIdx.x, save;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\tds_write_addtid_b32 %2 offset:16\n\ts_mov_b32 m0, %0\n\ts_waitcnt lgkmcnt(0)"
               : "=&s"(save) : "s"(base + m0v), "v"(v) : "memory");
  __syncthreads();
  for (int i = threadIdx.x; i < 1024; i += 64) out[i] = s[i];
  if (threadIdx.x == 0) out[1024] = base;
}
int main() {
  unsigned* d; hipMalloc(&d, 1025 * 4);
  unsigned h[1025];
  for (unsigned m0v : {0u, 256u}) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, m0v);
    hipMemcpy(h, d, 1025 * 4, hipMemcpyDeviceToHost);
    printf("m0 = base(%u) + %u:", h[1024], m0v);
    int shown = 0;
    for (int i = 0; i < 1024 && shown < 6; i++) if (h[i] != 0xFFFFFFFFu) { printf(" s[%d]=%u", i, h[i]); shown++; }
    int cnt = 0; for (int i = 0; i < 1024; i++) cnt += h[i] != 0xFFFFFFFFu;
    printf("  (%d dwords written)\n", cnt);
  }
  return 0;
}
