// mb_valu.hip -- SIMD issue cost of the integer VALU instructions the fused digests are made of
// (MD5 / MD4 rounds: v_add3_u32, v_bitop3_b32, v_alignbit_b32, v_bfi_b32, v_alignbit_b32, ...; the expansion: v_perm_b32,
// v_alignbyte_b32, v_lshl_or_b32), at 1 / 2 / 4 / 8 waves per SIMD.
//
// Every instruction is an inline-asm statement (the opcode cannot be changed or folded), its
// operands come from memory (no compile-time values) and every chain ends in the output, so no
// line is dead code.  Eight independent chains per wave (ILP 8).  The shader clock f comes from the
// 1-wave-per-SIMD run (each wave's s_memtime ticks over the kernel's event time: the wave spans the
// kernel); at W waves per SIMD the cost is
//   SIMD cycles per wave-instruction = event time x f / (instructions per wave x W),
// every wave of the grid resident at once (256-thread blocks, 256 x W of them, one wave per SIMD
// each).  A line under 1 cycle is impossible (the check prints IMPOSSIBLE) -- dead code or waves not
// co-resident.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mb_valu.hip -o tools/mb_valu
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <vector>
#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s\n", hipGetErrorString(e_)); return 1; } } while (0)
typedef uint32_t u32;

#define OP3(op) asm volatile(op " %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(y), "v"(z))
#define OP2(op) asm volatile(op " %0, %1, %2" : "=v"(r) : "v"(x), "v"(y))

template <int OP>
__device__ __forceinline__ u32 op(u32 x, u32 y, u32 z) {
  u32 r;
  if constexpr (OP == 0) OP2("v_add_u32");
  else if constexpr (OP == 1) OP2("v_xor_b32");
  else if constexpr (OP == 2) OP3("v_add3_u32");
  else if constexpr (OP == 3) OP3("v_xad_u32");  // (gfx950 has no v_xor3_b32)
  else if constexpr (OP == 4) OP3("v_bfi_b32");
  else if constexpr (OP == 5) OP3("v_alignbit_b32");
  else if constexpr (OP == 6) OP3("v_perm_b32");
  else if constexpr (OP == 7) OP3("v_alignbyte_b32");
  else if constexpr (OP == 8) OP3("v_lshl_or_b32");
  else if constexpr (OP == 9) OP3("v_lshl_add_u32");
  else if constexpr (OP == 10) OP2("v_mul_hi_u32");
  else if constexpr (OP == 12) asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(x), "v"(y), "v"(z));
  else if constexpr (OP == 13) OP2("v_add_u32_e64");  // a VOP2 opcode in the VOP3 encoding
  else if constexpr (OP == 14) OP2("v_lshlrev_b32_e64");
  else if constexpr (OP == 15) asm volatile("v_add3_u32 %0, %1, %2, 7" : "=v"(r) : "v"(x), "v"(y));  // 2 VGPR operands
  return r;
}

template <int OP>
__global__ void __launch_bounds__(256) k_valu(const u32* in, u32* out, unsigned long long* ticks, int iters) {
  const u32 t = blockIdx.x * blockDim.x + threadIdx.x;
  u32 a = in[t & 1023], b = in[(t + 1) & 1023], c = in[(t + 2) & 1023], d = in[(t + 3) & 1023];
  u32 e = in[(t + 4) & 1023], f = in[(t + 5) & 1023], g = in[(t + 6) & 1023], h = in[(t + 7) & 1023];
  const u32 s = in[1024 + (t & 3)];  // shift / selector operand, also from memory
  __builtin_amdgcn_s_waitcnt(0);
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int k = 0; k < 16; k++) {
      if constexpr (OP == 11) {  // v_cmp + v_cndmask (VCC): 2 instructions per step
        a = a > s ? b : c; b = b > s ? c : d; c = c > s ? d : e; d = d > s ? e : f;
        e = e > s ? f : g; f = f > s ? g : h; g = g > s ? h : a; h = h > s ? a : b;
        asm volatile("" : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h));
      } else {
        a = op<OP>(a, b, s); b = op<OP>(b, c, s); c = op<OP>(c, d, s); d = op<OP>(d, e, s);
        e = op<OP>(e, f, s); f = op<OP>(f, g, s); g = op<OP>(g, h, s); h = op<OP>(h, a, s);
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[t] = a ^ b ^ c ^ d ^ e ^ f ^ g ^ h;
  if ((threadIdx.x & 63) == 0) ticks[t / 64] = t1 - t0;
}

typedef void (*KFn)(const u32*, u32*, unsigned long long*, int);
int main() {
  u32 *in, *out;
  unsigned long long* ticks;
  CHK(hipMalloc(&in, 2048 * 4));
  CHK(hipMalloc(&out, 8 * 256 * 256 * 4));
  CHK(hipMalloc(&ticks, 8 * 256 * 4 * 8));
  std::vector<u32> h(2048);
  for (int i = 0; i < 2048; i++) h[i] = 0x9E3779B9u * (i + 1) ^ (i << 7);
  h[1024] = 0x05040100; h[1025] = 0x06050401; h[1026] = 0x07060502; h[1027] = 0x03020100;  // perm selectors / small shifts
  CHK(hipMemcpy(in, h.data(), 2048 * 4, hipMemcpyHostToDevice));
  const char* names[] = {"v_add_u32 (VOP2)", "v_xor_b32 (VOP2)", "v_add3_u32", "v_xad_u32", "v_bfi_b32", "v_alignbit_b32",
                         "v_perm_b32", "v_alignbyte_b32", "v_lshl_or_b32", "v_lshl_add_u32", "v_mul_hi_u32",
                         "v_cmp + v_cndmask (2 instr)", "v_bitop3_b32 (CDNA4)", "v_add_u32_e64", "v_lshlrev_b32_e64",
                         "v_add3_u32 (2 VGPR + imm)"};
  KFn fns[] = {k_valu<0>, k_valu<1>, k_valu<2>, k_valu<3>, k_valu<4>, k_valu<5>, k_valu<6>, k_valu<7>,
               k_valu<8>, k_valu<9>, k_valu<10>, k_valu<11>, k_valu<12>, k_valu<13>, k_valu<14>, k_valu<15>};
  const int iters = 4000;
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  printf("%-28s %s\n", "instruction", "SIMD cycles per wave-instruction at 1 / 2 / 4 / 8 waves per SIMD");
  double fclk = 0;
  for (int o = 0; o < 16; o++) {
    printf("%-28s", names[o]);
    for (int wps : {1, 2, 4, 8}) {
      const int blocks = 256 * wps;  // 256-thread blocks: one wave per SIMD each
      double best = 1e30;
      for (int rep = 0; rep < 3; rep++) {
        CHK(hipEventRecord(e0));
        hipLaunchKernelGGL(fns[o], dim3(blocks), dim3(256), 0, 0, in, out, ticks, iters);
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        float ms;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        std::vector<unsigned long long> tk(blocks * 4);
        CHK(hipMemcpy(tk.data(), ticks, tk.size() * 8, hipMemcpyDeviceToHost));
        double mean = 0;
        for (auto v : tk) mean += (double)v;
        mean /= tk.size();
        if (o == 0 && wps == 1 && rep == 2) fclk = mean / (ms * 1e-3);
        const double instr = (double)iters * 16 * 8 * (o == 11 ? 2 : 1);
        const double t = ms * 1e-3;
        best = t < best ? t : best;
        if (rep == 2 && fclk > 0) best = best * fclk / (instr * wps);
        else if (rep == 2) best = -1;
      }
      printf("  %6.2f%s", best, best > 0 && best < 1.0 ? " IMPOSSIBLE" : "");
    }
    printf("\n");
  }
  printf("shader clock from the 1-wave run: %.3f GHz\n", fclk / 1e9);
  return 0;
}
