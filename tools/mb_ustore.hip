// mb_ustore.hip -- can the expansion write its candidate stream straight from registers
// with UNALIGNED global stores (no LDS ring)?  A lane holding a byte run [o, o + n),
// n >= 16, writes it exactly with 16-B stores at o, o + 16, ..., and o + n - 16 (the last
// one overlaps the previous; every byte written belongs to the run, so lanes never race).
// Measures the store path at the C3 shape (candidates 8..26 B, runs of 4 per lane, 8192
// candidates per wave, ~30 GB) against the aligned coalesced stream, and checks bytes.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mb_ustore.hip -o tools/mb_ustore
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)
typedef uint32_t u32;
typedef uint64_t u64;
typedef u32 v4u __attribute__((ext_vector_type(4)));
typedef v4u v4ua __attribute__((aligned(1)));
typedef u32 u32a __attribute__((aligned(1)));

#ifndef CH
#define CH 16384u  // candidates per wave (k_expand_fast's chunk, A5X_CHUNK default)
#endif
#define K 4u

__device__ __forceinline__ u32 clen(u64 c) {  // 8..26 bytes, mean 17
  u64 x = c * 0x9E3779B97F4A7C15ull;
  x ^= x >> 29;
  return 8u + (u32)((x >> 40) % 19u);
}
// content byte at global position x
__device__ __forceinline__ u32 fb(u64 x) { return (u32)((x ^ (x >> 8) ^ (x >> 16)) & 255u); }
__device__ __forceinline__ u32 fdw(u64 x) { return fb(x) | (fb(x + 1) << 8) | (fb(x + 2) << 16) | (fb(x + 3) << 24); }

__global__ void k_sums(u64 n, u64* sums) {
  const u64 ch = blockIdx.x * 4ull + threadIdx.x / 64;
  const u32 lane = threadIdx.x & 63;
  u64 s = 0;
  for (u32 i = lane; i < CH; i += 64) {
    const u64 c = ch * CH + i;
    if (c < n) s += clen(c);
  }
  for (int m = 32; m; m >>= 1) s += __shfl_xor(s, m);
  if (lane == 0) sums[ch] = s;
}

__device__ __forceinline__ u32 incl_scan(u32 x) {
  const u32 lane = threadIdx.x & 63;
  for (int d = 1; d < 64; d <<= 1) {
    const u32 y = __shfl_up(x, d);
    if (lane >= (u32)d) x += y;
  }
  return x;
}

// MODE 0: aligned coalesced nontemporal dwordx4 over the chunk's range (the ceiling)
// MODE 1: runs of K candidates per lane, content computed in registers, unaligned stores
// MODE 2: as 1, constant content (store path only)
// MODE 3: as 1 with nontemporal unaligned stores
// MODE 4: runs assembled in a per-lane LDS slot (two unaligned ds_write_b128 pieces per
//         candidate), read back with unaligned ds_read_b128, unaligned global stores
// MODE 5: as 0 with plain (write-back) stores
// MODE 6 / 7: as 0 (nt) / 5 (plain) with the store instructions on the 128-B line grid
// MODE 8 / 9: k_expand_fast's flush pattern: per round of 64 runs of K candidates, the
//         complete 16-B blocks written so far (nt), instructions from the round's first
//         block (8) or on the 128-B line grid (9); the partial block waits for the next round
// MODE 10 / 11: as 8 / 9 with plain stores
// MODE 12 / 13: as 8 / 9 with sc1 (write-through) stores
// MODE 14..18: as 8 with the cache-policy bits sc0 / sc0 nt / sc1 nt / sc0 sc1 / sc0 sc1 nt
template <int MODE>
__global__ void __launch_bounds__(256) k_store(uint8_t* out, const u64* boff, u64 n) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[4 * 64 * 144];
  const u32 lane = threadIdx.x & 63, wv = threadIdx.x / 64;
  const u64 ch = blockIdx.x * 4ull + wv;
  if (ch * CH >= n) return;
  const u64 c0 = ch * CH, c1 = min(n, c0 + CH);
  u64 pos = boff[ch];
  if (MODE == 0 || MODE == 5 || MODE == 6 || MODE == 7) {
    const u64 end = boff[ch + 1];
    const u64 b0 = (MODE == 6 || MODE == 7) ? (pos & ~127ull) : (pos & ~15ull);
    for (u64 b = b0 + 16ull * lane; b < end; b += 1024) {
      if (b + 16 <= (pos & ~15ull)) continue;
      v4u v = {(u32)b, (u32)(b >> 32), 0x0a0a0a0au, (u32)ch};
      if (MODE == 0 || MODE == 6) __builtin_nontemporal_store(v, (v4u*)(out + b));
      else *(v4u*)(out + b) = v;
    }
    return;
  }
  if (MODE >= 8) {
    constexpr bool NT = MODE == 8 || MODE == 9, GRID = MODE == 9 || MODE == 11 || MODE == 13;
    constexpr bool SC1 = MODE == 12 || MODE == 13;
    u64 B = pos & ~15ull;  // first unwritten block
    for (u64 c = c0; c < c1; c += 64 * K) {
      const u64 cs = c + (u64)lane * K;
      u32 rl = 0;
#pragma unroll
      for (u32 i = 0; i < K; i++) rl += cs + i < c1 ? clen(cs + i) : 0u;
      const u32 inc = incl_scan(rl);
      pos += __shfl(inc, 63);
      const u64 E = (c + 64 * K >= c1) ? ((pos + 15) & ~15ull) : (pos & ~15ull);  // complete blocks (all at the end)
      const u64 G = GRID ? (B & ~127ull) : B;
      for (u64 b = G + 16ull * lane; b < E; b += 1024) {
        if (b < B) continue;
        v4u v = {(u32)b, (u32)(b >> 32), 0x0a0a0a0au, (u32)ch};
        if (MODE == 14) asm volatile("global_store_dwordx4 %0, %1, off sc0" ::"v"(out + b), "v"(v) : "memory");
        else if (MODE == 15) asm volatile("global_store_dwordx4 %0, %1, off sc0 nt" ::"v"(out + b), "v"(v) : "memory");
        else if (MODE == 16) asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" ::"v"(out + b), "v"(v) : "memory");
        else if (MODE == 17) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(out + b), "v"(v) : "memory");
        else if (MODE == 18) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt" ::"v"(out + b), "v"(v) : "memory");
        else if (SC1) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(out + b), "v"(v) : "memory");
        else if (NT) __builtin_nontemporal_store(v, (v4u*)(out + b));
        else *(v4u*)(out + b) = v;
      }
      B = E;
    }
    return;
  }
  uint8_t* slot = lds + (wv * 64 + lane) * 144;
  for (u64 c = c0; c < c1; c += 64 * K) {
    const u64 cs = c + (u64)lane * K;
    u32 l[K], rl = 0;
#pragma unroll
    for (u32 i = 0; i < K; i++) { l[i] = cs + i < c1 ? clen(cs + i) : 0u; rl += l[i]; }
    const u32 inc = incl_scan(rl);
    const u64 o = pos + inc - rl;
    pos += __shfl(inc, 63);
    if (MODE == 4) {
      // two pieces per candidate, 16-B unaligned LDS writes, later ones over earlier tails
      u32 p = 0;
#pragma unroll
      for (u32 i = 0; i < K; i++) {
        const u32 l0 = l[i] / 2, l1 = l[i] - l0;
        v4u a = {fdw(o + p), fdw(o + p + 4), fdw(o + p + 8), fdw(o + p + 12)};
        *(v4ua*)(slot + p) = a;
        p += l0;
        v4u b = {fdw(o + p), fdw(o + p + 4), fdw(o + p + 8), fdw(o + p + 12)};
        *(v4ua*)(slot + p) = b;
        p += l1;
      }
      __builtin_amdgcn_wave_barrier();
    }
    if (rl < 16) continue;  // (never at these lengths)
    const u32 nst = (rl + 15) / 16;
    for (u32 k = 0; k < (K * 26 + 15) / 16; k++) {
      if (k < nst) {
        const u32 r = min(16u * k, rl - 16u);
        v4u v;
        if (MODE == 2) v = (v4u){r, 1u, 2u, 3u};
        else if (MODE == 4) v = *(const v4ua*)(slot + r);
        else v = (v4u){fdw(o + r), fdw(o + r + 4), fdw(o + r + 8), fdw(o + r + 12)};
        if (MODE == 3) __builtin_nontemporal_store(v, (v4ua*)(out + o + r));
        else *(v4ua*)(out + o + r) = v;
      }
    }
  }
}

__global__ void k_check(const uint8_t* out, u64 total, u64* bad) {
  u64 nb = 0;
  for (u64 x = (blockIdx.x * 256ull + threadIdx.x) * 4; x < total; x += gridDim.x * 256ull * 4) {
    const u32 got = *(const u32*)(out + x);
    for (u32 b = 0; b < 4 && x + b < total; b++) nb += ((got >> (8 * b)) & 255u) != fb(x + b);
  }
  if (nb) atomicAdd((unsigned long long*)bad, (unsigned long long)nb);
}

int main(int argc, char** argv) {
  const u64 n = argc > 1 ? strtoull(argv[1], 0, 10) : 1800000000ull;
  const u64 nch = (n + CH - 1) / CH;
  u64 *dsum, *dboff, *dbad;
  CHK(hipMalloc(&dsum, nch * 8));
  CHK(hipMalloc(&dboff, (nch + 1) * 8));
  CHK(hipMalloc(&dbad, 8));
  hipLaunchKernelGGL(k_sums, dim3((nch + 3) / 4), dim3(256), 0, 0, n, dsum);
  std::vector<u64> s(nch), bo(nch + 1);
  CHK(hipMemcpy(s.data(), dsum, nch * 8, hipMemcpyDeviceToHost));
  bo[0] = 0;
  for (u64 i = 0; i < nch; i++) bo[i + 1] = bo[i] + s[i];
  const u64 total = bo[nch];
  CHK(hipMemcpy(dboff, bo.data(), (nch + 1) * 8, hipMemcpyHostToDevice));
  uint8_t* out;
  CHK(hipMalloc(&out, total + 64));
  printf("candidates %llu, bytes %.3f GB, chunks %llu (%u candidates per wave)\n", (unsigned long long)n, total / 1e9, (unsigned long long)nch, CH);
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  const char* names[] = {"aligned nt dwordx4 (ceiling)", "unaligned runs, reg content", "unaligned runs, const content",
                         "unaligned runs, nt", "LDS-slot runs, unaligned", "aligned plain dwordx4",
                         "aligned nt, 128-B instr grid", "aligned plain, 128-B instr grid",
                         "round flushes nt (kernel pattern)", "round flushes nt, 128-B grid",
                         "round flushes plain", "round flushes plain, 128-B grid",
                         "round flushes sc1", "round flushes sc1, 128-B grid", "round flushes sc0", "round flushes sc0 nt",
                         "round flushes sc1 nt", "round flushes sc0 sc1", "round flushes sc0 sc1 nt"};
  const int only = argc > 2 ? atoi(argv[2]) : 0;  // 1: the aligned / flush-pattern modes only
  for (int m = 0; m < 19; m++) {
    if (only && (m >= 1 && m <= 4)) continue;
    if (only == 2 && m < 8) continue;
    for (int rep = 0; rep < 3; rep++) {
      CHK(hipMemset(out, 0, total + 64));
      CHK(hipEventRecord(e0));
      switch (m) {
        case 0: hipLaunchKernelGGL(k_store<0>, dim3((nch + 3) / 4), dim3(256), 0, 0, out, dboff, n); break;
        case 1: hipLaunchKernelGGL(k_store<1>, dim3((nch + 3) / 4), dim3(256), 0, 0, out, dboff, n); break;
        case 2: hipLaunchKernelGGL(k_store<2>, dim3((nch + 3) / 4), dim3(256), 0, 0, out, dboff, n); break;
        case 3: hipLaunchKernelGGL(k_store<3>, dim3((nch + 3) / 4), dim3(256), 0, 0, out, dboff, n); break;
        case 4: hipLaunchKernelGGL(k_store<4>, dim3((nch + 3) / 4), dim3(256), 0, 0, out, dboff, n); break;
        case 5: hipLaunchKernelGGL(k_store<5>, dim3((nch + 3) / 4), dim3(256), 0, 0, out, dboff, n); break;
        case 6: hipLaunchKernelGGL(k_store<6>, dim3((nch + 3) / 4), dim3(256), 0, 0, out, dboff, n); break;
        case 7: hipLaunchKernelGGL(k_store<7>, dim3((nch + 3) / 4), dim3(256), 0, 0, out, dboff, n); break;
        case 8: hipLaunchKernelGGL(k_store<8>, dim3((nch + 3) / 4), dim3(256), 0, 0, out, dboff, n); break;
        case 9: hipLaunchKernelGGL(k_store<9>, dim3((nch + 3) / 4), dim3(256), 0, 0, out, dboff, n); break;
        case 10: hipLaunchKernelGGL(k_store<10>, dim3((nch + 3) / 4), dim3(256), 0, 0, out, dboff, n); break;
        case 11: hipLaunchKernelGGL(k_store<11>, dim3((nch + 3) / 4), dim3(256), 0, 0, out, dboff, n); break;
        case 12: hipLaunchKernelGGL(k_store<12>, dim3((nch + 3) / 4), dim3(256), 0, 0, out, dboff, n); break;
        case 13: hipLaunchKernelGGL(k_store<13>, dim3((nch + 3) / 4), dim3(256), 0, 0, out, dboff, n); break;
        case 14: hipLaunchKernelGGL(k_store<14>, dim3((nch + 3) / 4), dim3(256), 0, 0, out, dboff, n); break;
        case 15: hipLaunchKernelGGL(k_store<15>, dim3((nch + 3) / 4), dim3(256), 0, 0, out, dboff, n); break;
        case 16: hipLaunchKernelGGL(k_store<16>, dim3((nch + 3) / 4), dim3(256), 0, 0, out, dboff, n); break;
        case 17: hipLaunchKernelGGL(k_store<17>, dim3((nch + 3) / 4), dim3(256), 0, 0, out, dboff, n); break;
        case 18: hipLaunchKernelGGL(k_store<18>, dim3((nch + 3) / 4), dim3(256), 0, 0, out, dboff, n); break;
      }
      CHK(hipEventRecord(e1));
      CHK(hipEventSynchronize(e1));
      float ms;
      CHK(hipEventElapsedTime(&ms, e0, e1));
      u64 bad = 0;
      if (rep == 2 && (m == 1 || m == 3 || m == 4)) {
        CHK(hipMemset(dbad, 0, 8));
        hipLaunchKernelGGL(k_check, dim3(4096), dim3(256), 0, 0, out, total, dbad);
        CHK(hipMemcpy(&bad, dbad, 8, hipMemcpyDeviceToHost));
      }
      printf("%-34s %8.3f ms  %7.0f GB/s  frac %.3f%s%llu\n", names[m], ms, total / (ms * 1e-3) / 1e9,
             total / (ms * 1e-3) / 8e12, rep == 2 && m != 0 && m != 2 ? "  bad bytes " : "  ",
             (unsigned long long)bad);
    }
  }
  return 0;
}
