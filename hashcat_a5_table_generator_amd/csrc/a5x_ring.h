// a5x_ring.h -- byte-stream placement into a per-wave LDS ring (device only; used by
// k_expand_fast (a5x_fx6.h) and the -s / -s -r positional engine (a5x_modes.hip)).
//
// An entry is a uint4: 15 content bytes (zero past the length) + the length in byte
// 15.  fx7_put appends one entry at LDS byte address P by OR-ing its byte-shifted
// dwords into a ring that is kept zeroed between flushes (ds_or_b32): the dwords an
// entry touches beyond its own bytes receive zeros, so no ordering between lanes or
// entries is needed.
#pragma once
#include <stdint.h>

// LDS byte addresses as plain uint32_t (ds_* instructions take a VGPR address + an offset)
typedef __attribute__((address_space(3))) uint32_t fx6_lds32;
__device__ __forceinline__ uint32_t fx6_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
__device__ __forceinline__ void fx6_st(uint32_t a, uint32_t v) { *(fx6_lds32*)(uintptr_t)a = v; }

// 16-byte LDS accesses at a byte address (16-B aligned) and an XOR into a ring dword
typedef uint32_t fx6_v4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) fx6_v4 fx6_lds128;
__device__ __forceinline__ uint4 fx6_ld16(uint32_t a) {
  const fx6_v4 v = *(const fx6_lds128*)(uintptr_t)a;
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void fx6_st16(uint32_t a, uint4 v) {
  const fx6_v4 x = {v.x, v.y, v.z, v.w};
  *(fx6_lds128*)(uintptr_t)a = x;
}
__device__ __forceinline__ void fx7_xor(uint32_t a, uint32_t v) {
  __hip_atomic_fetch_xor((fx6_lds32*)(uintptr_t)a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}

// byte shift of a piece: w_k = bytes [4k - n, 4k - n + 4) of the piece (v_perm selector;
// n replicated into every byte by a perm with selector 0)
__device__ __forceinline__ uint32_t fx6_sel(uint32_t n) { return 0x07060504u - __builtin_amdgcn_perm(0u, n, 0u); }

// ---------------------------------------------------------------------------
// OR placement: the ring is kept zeroed between rounds and every piece ORs
// its byte-shifted dwords into it (ds_or_b32).  Entries are zero past their length,
// so the dwords a piece touches beyond its own bytes receive zeros: no ordering, no
// pending-dword register, no shared-dword merge across lanes, no trash redirection.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void fx7_or(uint32_t a, uint32_t v) {
  __hip_atomic_fetch_or((fx6_lds32*)(uintptr_t)a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}

// XOR swizzle of a ring byte address at 16-B-block granularity: block bits 4-6 ^= row bits
// 7-9, so each 128-B bank row (ds_write banks (a/4) mod 32) keeps its bytes and the 16-B
// blocks stay whole (the flush's ds_read_b128 / ds_write_b128 stay conflict-free).  The
// ring must start 1 KiB aligned so that logical block 0 is physical block 0.
__device__ __forceinline__ uint32_t fx7_swz(uint32_t a) { return a ^ ((a >> 3) & 0x70u); }

template <bool SWZ = false>
__device__ __forceinline__ void fx7_put(const uint4 e, uint32_t& P) {
  const uint32_t n = P & 3u, base = P - n;
  const uint32_t l = e.w >> 24, e3 = e.w & 0xFFFFFFu;
  const uint32_t sel = fx6_sel(n);
  const uint32_t t = n + l;
  auto at = [&](uint32_t o) { return SWZ ? fx7_swz(base + o) : base + o; };
  fx7_or(at(0u), __builtin_amdgcn_perm(e.x, 0u, sel));
  fx7_or(at(4u), __builtin_amdgcn_perm(e.y, e.x, sel));
  if (__builtin_amdgcn_ballot_w64(t > 8u)) {  // pieces reaching a third dword (wave-uniform)
    fx7_or(at(8u), __builtin_amdgcn_perm(e.z, e.y, sel));
    if (__builtin_amdgcn_ballot_w64(t > 12u)) {
      fx7_or(at(12u), __builtin_amdgcn_perm(e3, e.z, sel));
      if (__builtin_amdgcn_ballot_w64(t > 16u)) fx7_or(at(16u), __builtin_amdgcn_perm(0u, e3, sel));
    }
  }
  P += l;
}

// fx8_put: fx7_put with v_alignbyte shifts and the dword count decided per piece group
// (the -s / -s -r positional engine, a5x_modes.hip).  P1 = (LDS byte address of the
// piece) - 1, so that base = P1 & ~3 and the alignbyte shift (~P1) & 3 = (4 - n) & 3 need
// no selector build; for n = P & 3 = 0 the five slots cover [P - 4, P + 16) (slot 0 ORs
// zero into the dword before P: the ring needs 4 writable bytes in front of it).  Slot
// k >= 2 is written when ns > k (ns: wave-uniform, from the longest entry of the piece,
// so the compare is scalar); slots past a piece's bytes receive zeros.  The entry's byte
// 15 (its length) never reaches slots 0-3; slot 4 masks it.
__device__ __forceinline__ void fx8_put(const uint4 e, uint32_t& P1, uint32_t ns) {
  const uint32_t base = P1 & ~3u, s = ~P1;
  fx7_or(base, __builtin_amdgcn_alignbyte(e.x, 0u, s));
  fx7_or(base + 4u, __builtin_amdgcn_alignbyte(e.y, e.x, s));
  if (ns > 2u) {
    fx7_or(base + 8u, __builtin_amdgcn_alignbyte(e.z, e.y, s));
    if (ns > 3u) {
      fx7_or(base + 12u, __builtin_amdgcn_alignbyte(e.w, e.z, s));
      if (ns > 4u) fx7_or(base + 16u, __builtin_amdgcn_alignbyte(0u, e.w & 0xFFFFFFu, s));
    }
  }
  P1 += e.w >> 24;
}

// ring dwords a piece whose longest entry has lmax bytes can touch after a byte offset
// n in [1, 4] (n + lmax <= 4 ns: ns = 1 + ceil(lmax / 4), at least 2; the -s / -s -r
// positional engine sizes its placement loops with it)
__device__ __forceinline__ uint32_t fx8_slots(uint32_t lmax) { return lmax <= 4u ? 2u : 1u + ((lmax + 3u) >> 2); }

