// microbench_lds.hip -- throughput of the LDS primitives the expansion kernel uses,
// with its access pattern (lane l touches dword l*STRIDE + i, i.e. ~16-byte
// candidates per lane).  Build: hipcc --offload-arch=gfx950 -O3 tools/microbench_lds.hip -o mb
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

template <int KIND>
__global__ void __launch_bounds__(256) k_lds(int iters, int stride, unsigned* sink) {
  __shared__ unsigned lds[4 * 1024 * 4];  // 64 KB per block
  const unsigned lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  unsigned* my = lds + wv * 4096;
  for (int i = threadIdx.x; i < 4 * 1024 * 4; i += blockDim.x) lds[i] = 0;
  __syncthreads();
  unsigned acc = lane;
  for (int it = 0; it < iters; it++) {
    const unsigned a = (lane * stride + it) & 4095u;
    if (KIND == 0) atomicOr(&my[a], acc);                         // ds_or_b32
    if (KIND == 1) my[a] = acc;                                  // ds_write_b32
    if (KIND == 2) ((unsigned char*)my)[(lane * stride * 4 + it) & 16383u] = (unsigned char)acc;  // ds_write_b8
    if (KIND == 3) acc = (unsigned)__shfl((int)acc, (lane + it) & 63);  // ds_bpermute chain
    if (KIND == 4) acc += my[a];                                 // ds_read_b32 chain-free
    if (KIND == 5) atomicOr(&my[(lane * 4 + (it & 3)) & 4095u], acc);   // ds_or, lanes 4 dwords apart fixed
    acc = acc * 1664525u + 1013904223u;
  }
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(sink, acc + my[lane]);
}

int main() {
  unsigned* sink;
  CHECK(hipMalloc(&sink, 64));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  const char* names[] = {"ds_or_b32   ", "ds_write_b32", "ds_write_b8 ", "ds_bpermute ", "ds_read_b32 ", "ds_or fixed4"};
  const int iters = 4096;
  for (int kind = 0; kind < 6; kind++) {
    for (int stride : {1, 4, 5}) {
      for (int bpc : {1, 2}) {  // blocks per CU (4 waves each)
        const int blocks = cus * bpc;
        auto launch = [&]() {
          switch (kind) {
            case 0: hipLaunchKernelGGL(k_lds<0>, dim3(blocks), dim3(256), 0, 0, iters, stride, sink); break;
            case 1: hipLaunchKernelGGL(k_lds<1>, dim3(blocks), dim3(256), 0, 0, iters, stride, sink); break;
            case 2: hipLaunchKernelGGL(k_lds<2>, dim3(blocks), dim3(256), 0, 0, iters, stride, sink); break;
            case 3: hipLaunchKernelGGL(k_lds<3>, dim3(blocks), dim3(256), 0, 0, iters, stride, sink); break;
            case 4: hipLaunchKernelGGL(k_lds<4>, dim3(blocks), dim3(256), 0, 0, iters, stride, sink); break;
            case 5: hipLaunchKernelGGL(k_lds<5>, dim3(blocks), dim3(256), 0, 0, iters, stride, sink); break;
          }
        };
        launch();
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(a));
        for (int r = 0; r < 5; r++) launch();
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms;
        CHECK(hipEventElapsedTime(&ms, a, b));
        ms /= 5;
        // wave-instructions per CU
        const double winst = (double)bpc * 4 * iters;
        const double cyc = ms * 1e-3 * 2.4e9;
        printf("%s stride %d  waves/CU %2d: %.3f ms  %.2f cycles per wave-instruction per CU\n", names[kind], stride,
               bpc * 4, ms, cyc / winst);
      }
    }
  }
  return 0;
}
