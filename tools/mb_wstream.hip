// mb_wstream.hip -- what HBM write rate does MI355X give a pure store stream, by access
// pattern?  Bounds k_expand_fast (one wave per 8192-candidate chunk = ~140 KB of
// contiguous output, 1 KiB per wave store instruction).  Variants: per-wave regions of
// several sizes vs a grid-stride sweep, nontemporal vs plain stores, occupancy.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mb_wstream.hip -o tools/mb_wstream
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)
typedef uint32_t u32;
typedef uint64_t u64;
typedef u32 v4u __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ void st16(uint8_t* p, v4u v) {
  if (NT) __builtin_nontemporal_store(v, (v4u*)p);
  else *(v4u*)p = v;
}

// one wave per region of R bytes (contiguous), 1 KiB per store instruction; U stores per
// loop iteration
template <bool NT, int U>
__global__ void __launch_bounds__(256) k_region(uint8_t* out, u64 total, u64 R) {
  const u32 lane = threadIdx.x & 63;
  const u64 wv = blockIdx.x * 4ull + threadIdx.x / 64;
  const u64 b0 = wv * R, b1 = min(total, b0 + R);
  for (u64 b = b0 + 16ull * lane; b < b1; b += 1024ull * U) {
#pragma unroll
    for (int u = 0; u < U; u++)
      if (b + 1024ull * u < b1) st16<NT>(out + b + 1024ull * u, (v4u){(u32)b, (u32)u, 1u, 2u});
  }
}

// one wave per region of R bytes, store instructions on the 1 KiB-aligned address grid
// (the region's first instruction partial): are misaligned 1 KiB instructions the cost?
template <bool NT>
__global__ void __launch_bounds__(256) k_region_grid(uint8_t* out, u64 total, u64 R, u64 G) {
  const u32 lane = threadIdx.x & 63;
  const u64 wv = blockIdx.x * 4ull + threadIdx.x / 64;
  const u64 b0 = wv * R, b1 = min(total, b0 + R);
  for (u64 b = (b0 & ~(G - 1)) + 16ull * lane; b < b1; b += 1024ull)
    if (b >= b0) st16<NT>(out + b, (v4u){(u32)b, 0u, 1u, 2u});
}

// grid-stride sweep: wave-instruction i of wave w writes KiB (i * nwaves + w)
template <bool NT>
__global__ void __launch_bounds__(256) k_sweep(uint8_t* out, u64 total) {
  const u32 lane = threadIdx.x & 63;
  const u64 wv = blockIdx.x * 4ull + threadIdx.x / 64, nwv = gridDim.x * 4ull;
  for (u64 b = wv * 1024ull + 16ull * lane; b < total; b += nwv * 1024ull) st16<NT>(out + b, (v4u){(u32)b, 0u, 1u, 2u});
}

// per-wave regions with static LDS that limits occupancy to OCC waves per SIMD
template <bool NT, int LDSB>
__global__ void __launch_bounds__(256) k_region_lds(uint8_t* out, u64 total, u64 R) {
  __shared__ u32 pad[LDSB / 4];
  const u32 lane = threadIdx.x & 63;
  const u64 wv = blockIdx.x * 4ull + threadIdx.x / 64;
  const u64 b0 = wv * R, b1 = min(total, b0 + R);
  if (lane == 0) pad[(threadIdx.x / 64) & (LDSB / 4 - 1)] = (u32)wv;
  for (u64 b = b0 + 16ull * lane; b < b1; b += 1024ull) st16<NT>(out + b, (v4u){(u32)b, pad[0], 1u, 2u});
}

int main(int argc, char** argv) {
  const u64 total = argc > 1 ? strtoull(argv[1], 0, 10) : 30600000000ull;
  uint8_t* out;
  CHK(hipMalloc(&out, total + 4096));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  auto run = [&](const char* name, auto launch) {
    float best = 1e30f;
    for (int rep = 0; rep < 3; rep++) {
      CHK(hipEventRecord(e0));
      launch();
      CHK(hipEventRecord(e1));
      CHK(hipEventSynchronize(e1));
      float ms;
      CHK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    printf("%-44s %8.3f ms  %7.0f GB/s  frac %.3f\n", name, best, total / (best * 1e-3) / 1e9, total / (best * 1e-3) / 8e12);
  };
  if (argc > 2) {  // alignment study only
    for (u64 R : {140000ull, 140032ull, 140288ull, 139264ull}) {
      const u64 nw = (total + R - 1) / R, nb = (nw + 3) / 4;
      char nm[96];
      snprintf(nm, sizeof nm, "region %llu B nt", (unsigned long long)R);
      run(nm, [&] { hipLaunchKernelGGL((k_region<true, 1>), dim3(nb), dim3(256), 0, 0, out, total, R); });
      for (u64 G : {128ull, 1024ull}) {
        snprintf(nm, sizeof nm, "region %llu B nt, %llu-B instr grid", (unsigned long long)R, (unsigned long long)G);
        run(nm, [&] { hipLaunchKernelGGL((k_region_grid<true>), dim3(nb), dim3(256), 0, 0, out, total, R, G); });
        snprintf(nm, sizeof nm, "region %llu B plain, %llu-B instr grid", (unsigned long long)R, (unsigned long long)G);
        run(nm, [&] { hipLaunchKernelGGL((k_region_grid<false>), dim3(nb), dim3(256), 0, 0, out, total, R, G); });
      }
    }
    return 0;
  }
  const u64 Rs[] = {140000, 32768, 8192, 524288};
  for (u64 R : Rs) {
    const u64 nw = (total + R - 1) / R, nb = (nw + 3) / 4;
    char nm[96];
    snprintf(nm, sizeof nm, "region %llu B nt", (unsigned long long)R);
    run(nm, [&] { hipLaunchKernelGGL((k_region<true, 1>), dim3(nb), dim3(256), 0, 0, out, total, R); });
    snprintf(nm, sizeof nm, "region %llu B plain", (unsigned long long)R);
    run(nm, [&] { hipLaunchKernelGGL((k_region<false, 1>), dim3(nb), dim3(256), 0, 0, out, total, R); });
    snprintf(nm, sizeof nm, "region %llu B nt x4 unroll", (unsigned long long)R);
    run(nm, [&] { hipLaunchKernelGGL((k_region<true, 4>), dim3(nb), dim3(256), 0, 0, out, total, R); });
  }
  {
    const u64 R = 140000, nw = (total + R - 1) / R, nb = (nw + 3) / 4;
    run("region 140000 nt, 4 waves/CU (160 KiB LDS/WG)",
        [&] { hipLaunchKernelGGL((k_region_lds<true, 163840>), dim3(nb), dim3(256), 0, 0, out, total, R); });
    run("region 140000 nt, 8 waves/CU (80 KiB LDS/WG)",
        [&] { hipLaunchKernelGGL((k_region_lds<true, 81920>), dim3(nb), dim3(256), 0, 0, out, total, R); });
    run("region 140000 nt, 16 waves/CU (40 KiB LDS/WG)",
        [&] { hipLaunchKernelGGL((k_region_lds<true, 40960>), dim3(nb), dim3(256), 0, 0, out, total, R); });
    run("region 140000 nt, 32 waves/CU (20 KiB LDS/WG)",
        [&] { hipLaunchKernelGGL((k_region_lds<true, 20480>), dim3(nb), dim3(256), 0, 0, out, total, R); });
  }
  for (int g : {1024, 2048, 4096, 8192}) {
    char nm[96];
    snprintf(nm, sizeof nm, "sweep nt, %d WGs", g);
    run(nm, [&] { hipLaunchKernelGGL((k_sweep<true>), dim3(g), dim3(256), 0, 0, out, total); });
    snprintf(nm, sizeof nm, "sweep plain, %d WGs", g);
    run(nm, [&] { hipLaunchKernelGGL((k_sweep<false>), dim3(g), dim3(256), 0, 0, out, total); });
  }
  run("hipMemsetD32", [&] { CHK(hipMemsetD32((hipDeviceptr_t)out, 0x0a0a0a0a, total / 4)); });
  return 0;
}
