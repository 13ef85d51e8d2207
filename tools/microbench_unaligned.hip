// microbench_unaligned.hip -- does gfx950 LDS take unaligned ds_write_b32/b64 (and
// ds_read_b64/b128) at byte offsets, and at what rate?  The expansion kernel wants
// to write <= 8-byte pieces at arbitrary byte offsets.
// Build: hipcc --offload-arch=gfx950 -O3 tools/microbench_unaligned.hip -o tools/mb_unaligned
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

typedef uint64_t u64;
typedef uint32_t u32;

// correctness: lane l writes the 8 bytes (l*8+k) at byte offset 3 + 11*l (unaligned),
// in increasing lane order by rounds so there is no intra-instruction overlap.
__global__ void k_check(uint8_t* out, u32 b3, u32 b11, u32 b1) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[2048];
  const u32 l = threadIdx.x;
  for (u32 i = l; i < 2048; i += 64) lds[i] = 0xee;
  __syncthreads();
  u64 v = 0;
  for (u32 k = 0; k < 8; k++) v |= (u64)(uint8_t)(l * 8 + k) << (8 * k);
  const u32 off = b3 + b11 * l;  // 11 > 8: no overlap
  *(u64*)(lds + off) = v;
  if (l < 36) *(uint4*)(lds + 1400 + 17 * l + b1) = make_uint4(l * 4 + 0x01010101u, l * 4 + 0x02020202u, l, ~l);  // 16 B at stride 17
  const u32 off2 = 1024 + 5 * l + b1;  // 4-byte writes at stride 5
  *(u32*)(lds + off2) = (u32)v;
  __syncthreads();
  // unaligned reads back
  const u64 r = *(u64*)(lds + off);
  const u32 r2 = *(u32*)(lds + off2);
  for (u32 i = l; i < 2048; i += 64) out[i] = lds[i];
  ((u64*)(out + 2048))[l] = r;
  ((u32*)(out + 2048 + 512))[l] = r2;
}

// rate: each wave writes KIND pieces per lane per iteration at offsets o += len (len 1..8)
template <int KIND>
__global__ void __launch_bounds__(256) k_rate(int iters, u32* sink) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[4 * 8192 + 64];
  const u32 lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint8_t* my = lds + wv * 8192;
  u32 o = lane * 16 + (lane * 7 & 3);
  u64 v = 0x0102030405060708ull * (lane + 1);
  u32 acc = 0;
  for (int it = 0; it < iters; it++) {
    const u32 len = 1 + ((lane + it) & 7);
    if (KIND == 0) *(u64*)(my + (o & 8191u)) = v;                       // unaligned ds_write_b64
    if (KIND == 1) *(u32*)(my + (o & 8191u)) = (u32)v;                  // unaligned ds_write_b32
    if (KIND == 2) *(u64*)(my + (o & 8191u & ~7u)) = v;                 // aligned ds_write_b64
    if (KIND == 3) atomicOr((u32*)(my + (o & 8191u & ~3u)), (u32)v);    // aligned ds_or_b32
    if (KIND == 4) acc += *(const u32*)(my + ((o * 5) & 8191u));        // unaligned ds_read_b32
    if (KIND == 5) { const uint4 q = *(const uint4*)(my + ((o * 3) & 8191u & ~15u)); acc += q.x ^ q.w; }  // b128 aligned
    if (KIND == 6) atomicOr((unsigned long long*)(my + (o & 8191u & ~7u)), (unsigned long long)v);  // ds_or_b64
    if (KIND == 7) my[o & 8191u] = (uint8_t)v;                                                       // ds_write_b8
    if (KIND == 8) *(uint16_t*)(my + (o & 8191u)) = (uint16_t)v;                                     // b16 unaligned
    if (KIND == 9) *(uint4*)(my + (o & 8191u & ~15u)) = make_uint4((u32)v, (u32)(v >> 32), 1u, 2u);  // b128 aligned
    if (KIND == 10) *(uint4*)(my + (o & 8191u)) = make_uint4((u32)v, (u32)(v >> 32), 1u, 2u);        // b128 unaligned
    if (KIND == 11) *(uint2*)(my + (o & 8191u)) = make_uint2((u32)v, (u32)(v >> 32));               // b64 unaligned (uint2)
    o += len * 8;  // lanes ~ stride 16 B apart, moving on
    v = v * 0x9E3779B97F4A7C15ull + 1;
  }
  __syncthreads();
  if (lane == 0) atomicAdd(sink, acc + my[lane] + (u32)v);
}

int main() {
  uint8_t* d;
  CHECK(hipMalloc(&d, 4096));
  CHECK(hipMemset(d, 0, 4096));
  hipLaunchKernelGGL(k_check, dim3(1), dim3(64), 0, 0, d, 3u, 11u, 1u);
  CHECK(hipDeviceSynchronize());
  uint8_t h[4096];
  CHECK(hipMemcpy(h, d, 4096, hipMemcpyDeviceToHost));
  int bad = 0;
  for (u32 l = 0; l < 64; l++) {
    for (u32 k = 0; k < 8; k++) if (h[3 + 11 * l + k] != (uint8_t)(l * 8 + k)) bad++;
    u64 r;
    memcpy(&r, h + 2048 + 8 * l, 8);
    for (u32 k = 0; k < 8; k++) if ((uint8_t)(r >> (8 * k)) != (uint8_t)(l * 8 + k)) bad++;
  }
  // the 4-byte stride-5 writes: byte 1024+5l+1+k = (l*8+k) for k<4, later lanes don't overlap (5>4)
  for (u32 l = 0; l < 64; l++)
    for (u32 k = 0; k < 4; k++) if (h[1024 + 5 * l + 1 + k] != (uint8_t)(l * 8 + k)) bad++;
  for (u32 l = 0; l < 22; l++) {  // 1400 + 17*l + 1 .. +16 within the 2048 dump for l < 38
    u32 x[4] = {l * 4 + 0x01010101u, l * 4 + 0x02020202u, l, ~l};
    if (memcmp(h + 1400 + 17 * l + 1, x, 16)) bad++;
  }
  // gaps untouched
  if (h[0] != 0xee || h[1] != 0xee || h[2] != 0xee || h[11] != 0xee || h[13] != 0xee) bad++;
  printf("unaligned LDS check: %s (%d bad bytes)\n", bad ? "FAIL" : "OK", bad);

  u32* sink;
  CHECK(hipMalloc(&sink, 64));
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  const char* names[] = {"ds_write_b64 unaligned", "ds_write_b32 unaligned", "ds_write_b64 aligned  ",
                         "ds_or_b32 aligned     ", "ds_read_b32 unaligned ", "ds_read_b128 aligned  ",
                         "ds_or_b64 aligned     ", "ds_write_b8           ", "ds_write_b16 unaligned", "ds_write_b128 aligned ",
                         "ds_write_b128 unalign ", "ds_write_b64 unal (u2)"};
  const int iters = 8192;
  for (int kind = 0; kind < 12; kind++) {
    for (int bpc : {2, 4}) {
      const int blocks = cus * bpc;
      auto launch = [&]() {
        switch (kind) {
          case 0: hipLaunchKernelGGL(k_rate<0>, dim3(blocks), dim3(256), 0, 0, iters, sink); break;
          case 1: hipLaunchKernelGGL(k_rate<1>, dim3(blocks), dim3(256), 0, 0, iters, sink); break;
          case 2: hipLaunchKernelGGL(k_rate<2>, dim3(blocks), dim3(256), 0, 0, iters, sink); break;
          case 3: hipLaunchKernelGGL(k_rate<3>, dim3(blocks), dim3(256), 0, 0, iters, sink); break;
          case 4: hipLaunchKernelGGL(k_rate<4>, dim3(blocks), dim3(256), 0, 0, iters, sink); break;
          case 5: hipLaunchKernelGGL(k_rate<5>, dim3(blocks), dim3(256), 0, 0, iters, sink); break;
          case 6: hipLaunchKernelGGL(k_rate<6>, dim3(blocks), dim3(256), 0, 0, iters, sink); break;
          case 7: hipLaunchKernelGGL(k_rate<7>, dim3(blocks), dim3(256), 0, 0, iters, sink); break;
          case 8: hipLaunchKernelGGL(k_rate<8>, dim3(blocks), dim3(256), 0, 0, iters, sink); break;
          case 9: hipLaunchKernelGGL(k_rate<9>, dim3(blocks), dim3(256), 0, 0, iters, sink); break;
          case 10: hipLaunchKernelGGL(k_rate<10>, dim3(blocks), dim3(256), 0, 0, iters, sink); break;
          case 11: hipLaunchKernelGGL(k_rate<11>, dim3(blocks), dim3(256), 0, 0, iters, sink); break;
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
      const double winst = (double)bpc * 4 * iters;
      printf("%s waves/CU %2d: %.3f ms  %.2f CU-cycles per wave-instruction\n", names[kind], bpc * 4, ms,
             ms * 1e-3 * 2.4e9 / winst);
    }
  }
  return bad ? 1 : 0;
}
