// mb_valu.hip -- VALU issue rate of integer ops (v_perm_b32, v_add_u32, v_cndmask) at
// 1..4 waves per SIMD: cycles per wave-instruction per SIMD.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s\n", hipGetErrorString(e_)); return 1; } } while (0)
template <int OP>
__global__ void __launch_bounds__(256) k_valu(uint32_t* out, int iters) {
  uint32_t a = threadIdx.x, b = a * 3 + 1, c = a ^ 0x55, d = a + 7, e = a * 5, f = a + 11, g = a ^ 0x33, h = a * 9;
  const uint32_t s = 0x05040100 + (threadIdx.x & 3);
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int k = 0; k < 16; k++) {
      if (OP == 2) {
        a = __builtin_amdgcn_alignbyte(a, b, s); b = __builtin_amdgcn_alignbyte(b, c, s); c = __builtin_amdgcn_alignbyte(c, d, s);
        d = __builtin_amdgcn_alignbyte(d, e, s); e = __builtin_amdgcn_alignbyte(e, f, s); f = __builtin_amdgcn_alignbyte(f, g, s);
        g = __builtin_amdgcn_alignbyte(g, h, s); h = __builtin_amdgcn_alignbyte(h, a, s);
      } else if (OP == 3) {
        a = (a << (s & 31)) | b; b = (b << (s & 31)) | c; c = (c << (s & 31)) | d; d = (d << (s & 31)) | e;
        e = (e << (s & 31)) | f; f = (f << (s & 31)) | g; g = (g << (s & 31)) | h; h = (h << (s & 31)) | a;
      } else if (OP == 4) {
        a = a > s ? b : c; b = b > s ? c : d; c = c > s ? d : e; d = d > s ? e : f;
        e = e > s ? f : g; f = f > s ? g : h; g = g > s ? h : a; h = h > s ? a : b;
      } else if (OP == 5) {
        a = __umulhi(a, b); b = __umulhi(b, c); c = __umulhi(c, d); d = __umulhi(d, e);
        e = __umulhi(e, f); f = __umulhi(f, g); g = __umulhi(g, h); h = __umulhi(h, a | 1);
      } else if (OP == 6) {
        a = (uint32_t)(((uint64_t)a << (b & 31)) >> 32) ^ c; b = (uint32_t)(((uint64_t)b << (c & 31)) >> 32) ^ d;
        c = (uint32_t)(((uint64_t)c << (d & 31)) >> 32) ^ e; d = (uint32_t)(((uint64_t)d << (e & 31)) >> 32) ^ f;
        e = (uint32_t)(((uint64_t)e << (f & 31)) >> 32) ^ g; f = (uint32_t)(((uint64_t)f << (g & 31)) >> 32) ^ h;
        g = (uint32_t)(((uint64_t)g << (h & 31)) >> 32) ^ a; h = (uint32_t)(((uint64_t)h << (a & 31)) >> 32) ^ b;
      } else if (OP == 0) {
        a = __builtin_amdgcn_perm(a, b, s); b = __builtin_amdgcn_perm(b, c, s); c = __builtin_amdgcn_perm(c, d, s);
        d = __builtin_amdgcn_perm(d, e, s); e = __builtin_amdgcn_perm(e, f, s); f = __builtin_amdgcn_perm(f, g, s);
        g = __builtin_amdgcn_perm(g, h, s); h = __builtin_amdgcn_perm(h, a, s);
      } else {
        a += b; b += c; c += d; d += e; e += f; f += g; g += h; h += a;
      }
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a ^ b ^ c ^ d ^ e ^ f ^ g ^ h;
}
int main() {
  uint32_t* o;
  CHK(hipMalloc(&o, 64 << 20));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  const int iters = 2000;
  const char* names[] = {"v_perm", "v_add ", "alignbyte", "lshl_or", "cmp+cndmask", "mul_hi", "shl64+xor"};
  for (int op = 0; op < 7; op++)
    for (int wps : {4}) {  // waves per SIMD: 256-thread blocks = 1 wave per SIMD each
      const int blocks = 256 * wps;
      for (int rep = 0; rep < 2; rep++) {
        CHK(hipEventRecord(e0));
        switch (op) {
          case 0: hipLaunchKernelGGL(k_valu<0>, dim3(blocks), dim3(256), 0, 0, o, iters); break;
          case 1: hipLaunchKernelGGL(k_valu<1>, dim3(blocks), dim3(256), 0, 0, o, iters); break;
          case 2: hipLaunchKernelGGL(k_valu<2>, dim3(blocks), dim3(256), 0, 0, o, iters); break;
          case 3: hipLaunchKernelGGL(k_valu<3>, dim3(blocks), dim3(256), 0, 0, o, iters); break;
          case 4: hipLaunchKernelGGL(k_valu<4>, dim3(blocks), dim3(256), 0, 0, o, iters); break;
          case 5: hipLaunchKernelGGL(k_valu<5>, dim3(blocks), dim3(256), 0, 0, o, iters); break;
          case 6: hipLaunchKernelGGL(k_valu<6>, dim3(blocks), dim3(256), 0, 0, o, iters); break;
        }
        CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
        float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
        const double winst_per_simd = (double)wps * iters * 16 * 8;  // per SIMD
        if (rep) printf("%-12s waves/SIMD %d: %.3f ms  %.2f ns per 'op' per SIMD (%.2f cycles @2.4GHz)\n",
                        names[op], wps, ms, ms * 1e6 / winst_per_simd, ms * 1e6 / winst_per_simd * 2.4);
      }
    }
  return 0;
}
