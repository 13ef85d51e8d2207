// a5x_digest.hip -- fused digest + lookup over an expanded candidate stream.
//
// No counterpart in the reference: main.go only prints candidates (main.go:66) and
// hashcat hashes them (README.MD:69).  Here the "cand\n" stream that the expansion
// kernels leave in HBM is hashed on the device, so candidates never round-trip to the
// host:
//   MD5   RFC 1321 over the candidate bytes (== Go crypto/md5);
//   NTLM  MD4 (RFC 1320) over UTF-16LE of the candidate decoded as Go does for
//         []rune(string): invalid UTF-8 byte -> U+FFFD, runes > U+FFFF -> surrogate
//         pairs (unicode/utf16.Encode).
// Each digest is probed against a device-resident target set: a 2^k-bit prefilter
// indexed by digest word 0, then an open-addressing table of 16-B digests.
//
// Work unit: one wave per 2 KiB block of the stream.  The wave stages the block (+256 B
// of the next one) in LDS, finds line starts with a SWAR newline test (exact per byte),
// compacts them into an ordered start list, and every lane hashes one candidate at a
// time; the candidate owned by a block is the one STARTING in it.  A hit records
// (block, ordinal in block, digest); a per-block start count + scan turns that into
// the global candidate index afterwards (hits are rare).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "a5x.h"
#include "a5x_format.h"
#include "a5x_launch.h"
#include "a5x_md.h"

namespace {

typedef uint64_t u64;
typedef uint32_t u32;

// stream bytes per wave: 4 KiB for MD5 (lanes stay busy over ~3 rounds of candidates),
// 2 KiB for NTLM (the MD4 of UTF-16LE costs about twice per candidate byte)
template <bool MD5> struct DCfg { static constexpr u32 BLK = MD5 ? 4096u : 2048u; };
constexpr u32 DMARGIN = 256;               // next-block bytes staged for straddling lines
constexpr u32 D_ERR_HITCAP = 1u << 10;     // more hits than the caller's buffer

__device__ __forceinline__ u32 d_lane() { return __lane_id(); }

__device__ __forceinline__ u32 d_incl_scan(u32 x) {
  const u32 lane = d_lane();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const u32 y = (u32)__shfl_up((int)x, d, 64);
    if ((int)lane >= d) x += y;
  }
  return x;
}

__device__ __forceinline__ u32 glob4(const uint8_t* base, u64 off, u64 lim) {
  u32 v = 0;
  for (u32 k = 0; k < 4; k++)
    if (off + k < lim) v |= (u32)base[off + k] << (8 * k);
  return v;
}

// message bytes in HBM (lines that run past the staged bytes): 4 bytes at message
// offset i, zero past the stream end
struct MdGlob {
  const uint8_t* g;
  u64 off, lim;
  __device__ __forceinline__ u32 at4(u32 i) const { return glob4(g, off + i, lim); }
};

// Merkle-Damgard over message bytes [0, len) of src (LDS, or global when lds == false):
// RFC 1321/1320 padding (0x80, zeros, 64-bit little-endian bit length).
template <bool MD5>
__device__ __forceinline__ void md_digest(const uint8_t* lbase, u32 loff, const uint8_t* gbase, u64 goff, u64 glim,
                                          bool lds, u32 len, u32* st) {
  st[0] = 0x67452301u; st[1] = 0xefcdab89u; st[2] = 0x98badcfeu; st[3] = 0x10325476u;
  const u32 nb = (len + 8u) / 64u + 1u;
  for (u32 blk = 0; blk < nb; blk++) {
    u32 M[16];
#pragma unroll
    for (u32 j = 0; j < 16; j++) {
      const u32 b = blk * 64u + 4u * j;
      const int k = (int)len - (int)b;
      u32 raw = 0;
      if (k > 0) raw = lds ? lds4(lbase, loff + b) : glob4(gbase, goff + b, glim);
      const u32 keep = k >= 4 ? 0xffffffffu : (k <= 0 ? 0u : ((1u << (8 * k)) - 1u));
      const u32 pad = (k >= 0 && k < 4) ? (0x80u << (8 * k)) : 0u;
      M[j] = (raw & keep) | pad;
    }
    if (blk == nb - 1) {
      M[14] = len << 3;
      M[15] = len >> 29;
    }
    if (MD5) md5_block(st, M); else md4_block(st, M);
  }
}

__device__ __forceinline__ bool probe(const A5xDigLaunch& a, const u32* d) {
  return md_probe(a.bitmap, a.bm_mask, a.table, a.tmask, a.has_zero_target != 0, d);
}

template <u32 BLK>
struct DWave {
  static constexpr u32 BUF = BLK + DMARGIN + 80;  // + slack for the 8-B over-reads of the loader
  uint8_t data[BUF];
  uint16_t starts[BLK + 2];
};

// op 0: probe targets, record hits; op 1: count line starts per block; op 2: write
// every candidate's digest at dig_out[16 * (blk_pre[blk] + i)]
template <bool MD5>
__global__ void __launch_bounds__(256) k_digest_stream(A5xDigLaunch a, int op) {
  extern __shared__ __attribute__((aligned(16))) uint8_t d_dyn[];
  const u32 wv = threadIdx.x / 64, lane = d_lane();
  const u32 nwv = blockDim.x / 64;
  constexpr u32 DBLK = DCfg<MD5>::BLK;
  typedef DWave<DBLK> WT;
  constexpr u32 DBUF = WT::BUF;
  constexpr u32 NM = DBLK / 2048u;  // 32-bit newline masks per lane (32 B each)
  const u32 per = (u32)sizeof(WT);
  WT& W = *(WT*)(d_dyn + wv * ((per + 15u) & ~15u));
  const u64 nblk = (a.nbytes + DBLK - 1) / DBLK;
  u32 err = 0;
  for (u64 blk = (u64)blockIdx.x * nwv + wv; blk < nblk; blk += (u64)gridDim.x * nwv) {
    const u64 bs = blk * DBLK;
    const u32 bl = (u32)min<u64>(DBLK, a.nbytes - bs);                  // block bytes
    const u32 sl = (u32)min<u64>(DBLK + DMARGIN, a.nbytes - bs);        // staged bytes
    __builtin_amdgcn_wave_barrier();
    // stage [bs, bs + sl) (16-B loads; the stream base is 16-B aligned, see the launcher)
    const uint4* g16 = (const uint4*)(a.out + bs);
    uint4* l16 = (uint4*)W.data;
    for (u32 i = lane; i < sl / 16; i += 64) l16[i] = g16[i];
    for (u32 i = (sl & ~15u) + lane; i < sl; i += 64) W.data[i] = a.out[bs + i];
    for (u32 i = sl + lane; i < DBUF; i += 64) W.data[i] = 0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // newline bits of this lane's slice (NM x 32 bytes)
    const u32 q0 = lane * 32u * NM;
    u32 nl[NM], sm[NM];
#pragma unroll
    for (u32 h = 0; h < NM; h++) nl[h] = 0;
#pragma unroll
    for (u32 j = 0; j < 8 * NM; j++) {
      const u32 x = ((const u32*)W.data)[lane * 8 * NM + j] ^ 0x0a0a0a0au;
      const u32 t = ~(((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x | 0x7f7f7f7fu);  // 0x80 where the byte is '\n'
      const u32 f = ((t >> 7) & 1u) | ((t >> 14) & 2u) | ((t >> 21) & 4u) | ((t >> 28) & 8u);
      nl[j >> 3] |= f << (4 * (j & 7));
    }
    auto keep = [&](u32 base) -> u32 {
      return base >= bl ? 0u : (base + 32u <= bl ? 0xffffffffu : ((1u << (bl - base)) - 1u));
    };
#pragma unroll
    for (u32 h = 0; h < NM; h++) nl[h] &= keep(q0 + 32u * h);
    // line starts: byte 0 of the stream, and every byte after a '\n'
    u32 carry = (u32)__shfl_up((int)(nl[NM - 1] >> 31), 1, 64);
    if (lane == 0) carry = bs == 0 ? 1u : (a.out[bs - 1] == '\n' ? 1u : 0u);
    u32 m = 0;
#pragma unroll
    for (u32 h = 0; h < NM; h++) {
      sm[h] = ((nl[h] << 1) | (h ? (nl[h - 1] >> 31) : carry)) & keep(q0 + 32u * h);
      m += (u32)__builtin_popcount(sm[h]);
    }
    const u32 incl = d_incl_scan(m);
    const u32 nst = (u32)__builtin_amdgcn_readlane((int)incl, 63);
    u32 o = incl - m;
#pragma unroll
    for (u32 h = 0; h < NM; h++)
      for (u32 x = sm[h]; x; x &= x - 1) W.starts[o++] = (uint16_t)(q0 + 32u * h + (u32)__builtin_ctz(x));
    if (lane == 0 && a.blk_cnt) a.blk_cnt[blk] = nst;  // ordinals of hits (k_hits_resolve)
    if (op == 1) continue;
    // end of the last line starting here: first '\n' at or after it
    u64 tail_end = 0;
    if (nst) {
      const u32 s_last = W.starts[nst - 1];
      const u32 lim = min(sl, DBLK + DMARGIN);
      // lanes look at 64 consecutive bytes at a time
      u64 found = ~0ull;
      for (u32 base = s_last; base < lim && found == ~0ull; base += 64) {
        const u32 q = base + lane;
        const bool hit = q < lim && W.data[q] == '\n';
        const u64 bal = __ballot(hit);
        if (bal) found = base + (u32)__builtin_ctzll(bal);
      }
      if (found == ~0ull) {  // the line runs past the staged bytes: scan HBM
        u64 g = bs + lim;
        for (;; g += 64) {
          const u64 q = g + lane;
          const bool hit = q < a.nbytes && a.out[q] == '\n';
          const u64 bal = __ballot(hit);
          if (bal) { found = g - bs + (u32)__builtin_ctzll(bal); break; }
          if (g + 64 >= a.nbytes) { found = a.nbytes - bs; break; }  // unterminated (not produced here)
        }
      }
      tail_end = found;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (u32 i = lane; i < nst; i += 64) {
      const u32 s = W.starts[i];
      const u64 e = i + 1 < nst ? (u64)W.starts[i + 1] - 1 : tail_end;  // '\n' position
      const u32 len = (u32)(e - s);
      // every byte of the line staged (bytes past sl are zero-filled) and the 8-B
      // over-read of the last message word inside the buffer
      const bool in_lds = e <= sl && e + 8 <= DBUF;
      u32 d[4];
      if (MD5) {
        md_digest<true>(W.data, s, a.out, bs + s, a.nbytes, in_lds, len, d);
      } else if (in_lds) {  // any length: the UTF-16LE units are made as MD4 blocks fill
        MdLds src;
        src.base = W.data;
        src.off = s;
        ntlm_stream(src, len, d);
      } else {
        MdGlob src;
        src.g = a.out;
        src.off = bs + s;
        src.lim = a.nbytes;
        ntlm_stream(src, len, d);
      }
      if (op == 2) {
        uint4* o4 = (uint4*)(a.dig_out + 16 * (a.blk_pre[blk] + i));
        *o4 = make_uint4(d[0], d[1], d[2], d[3]);
      } else if (probe(a, d)) {
        const u32 h = atomicAdd(a.nhits, 1u);
        if (h < a.hit_cap) {
          A5xHitRaw r;
          r.blk = blk; r.idx = i; r.d[0] = d[0]; r.d[1] = d[1]; r.d[2] = d[2]; r.d[3] = d[3];
          a.hits[h] = r;
        } else {
          err |= D_ERR_HITCAP;
        }
      }
    }
  }
  if (err) atomicOr(a.err, err);
}

// hits: (block, ordinal) -> global candidate index -> (word, candidate in word)
__global__ void __launch_bounds__(64) k_hits_resolve(A5xHitRaw* hits, u32 n, const u64* blk_pre, u64 cand_base,
                                                      const u64* cand_off, u64 nw) {
  for (u32 h = blockIdx.x * 64 + threadIdx.x; h < n; h += gridDim.x * 64) {
    A5xHitRaw r = hits[h];
    const u64 g = cand_base + blk_pre[r.blk] + r.idx;
    u64 lo = 0, hi = nw;  // largest w with cand_off[w] <= g
    while (hi - lo > 1) {
      const u64 mid = (lo + hi) / 2;
      if (cand_off[mid] <= g) lo = mid; else hi = mid;
    }
    r.blk = lo;
    r.idx = g - cand_off[lo];
    hits[h] = r;
  }
}

// Hybrid fused digest: the candidate-bearing words the fused kernel leaves out (not
// FAST: slow / BIG / pass-G words) are listed, then gathered into a compact sub-batch
// that the two-pass path digests.
__global__ void __launch_bounds__(256) k_nonfast_list(const u32* flags, const u64* cand_off, u64 nw, u64 cb, u64 ce,
                                                       u32* list, u32* n) {
  // (words with candidates inside [cb, ce))
  for (u64 w = (u64)blockIdx.x * 256 + threadIdx.x; w < nw; w += (u64)gridDim.x * 256)
    if (cand_off[w + 1] > cand_off[w] && cand_off[w] < ce && cand_off[w + 1] > cb && !(flags[w] & A5X_WF_FAST))
      list[atomicAdd(n, 1u)] = (u32)w;
}

__global__ void __launch_bounds__(256) k_gather_lens(const u64* woff, const u32* idx, u32 m, u64* lens) {
  for (u32 k = blockIdx.x * 256 + threadIdx.x; k < m; k += gridDim.x * 256) lens[k] = woff[idx[k] + 1] - woff[idx[k]];
}

__global__ void __launch_bounds__(64) k_gather_words(const uint8_t* words, const u64* woff, const u32* idx, u32 m,
                                                      const u64* sub_off, uint8_t* out) {
  for (u32 k = blockIdx.x; k < m; k += gridDim.x) {
    const u64 s = woff[idx[k]], L = woff[idx[k] + 1] - s, d = sub_off[k];
    for (u64 i = threadIdx.x; i < L; i += 64) out[d + i] = words[s + i];
  }
}

}  // namespace

hipError_t a5x_launch_nonfast_list(const uint32_t* flags, const uint64_t* cand_off, uint64_t nw, uint64_t cb,
                                   uint64_t ce, uint32_t* list, uint32_t* n, hipStream_t st) {
  if (!nw) return hipSuccess;
  const u64 b = (nw + 255) / 256;
  hipLaunchKernelGGL(k_nonfast_list, dim3((u32)(b < 16384 ? b : 16384)), dim3(256), 0, st, flags, cand_off, nw, cb, ce,
                     list, n);
  return hipGetLastError();
}

hipError_t a5x_launch_gather_words(const uint8_t* words, const uint64_t* woff, const uint32_t* idx, uint32_t m,
                                   uint64_t* lens, const uint64_t* sub_off, uint8_t* out, hipStream_t st) {
  if (!m) return hipSuccess;
  if (lens) {  // pass 1: the lengths
    hipLaunchKernelGGL(k_gather_lens, dim3((m + 255) / 256 < 4096 ? (m + 255) / 256 : 4096), dim3(256), 0, st, woff, idx,
                       m, lens);
  } else {     // pass 2: the bytes at the scanned offsets
    hipLaunchKernelGGL(k_gather_words, dim3(m < 65536 ? m : 65536), dim3(64), 0, st, words, woff, idx, m, sub_off, out);
  }
  return hipGetLastError();
}

size_t a5x_digest_lds(int algo) {
  const u32 per = algo == A5X_ALGO_MD5 ? (u32)sizeof(DWave<DCfg<true>::BLK>) : (u32)sizeof(DWave<DCfg<false>::BLK>);
  return 4u * ((per + 15u) & ~15u);
}

hipError_t a5x_launch_digest_stream(const A5xDigLaunch& L, int op, uint32_t grid, hipStream_t st) {
  if (L.nbytes == 0) return hipSuccess;
  if (((uintptr_t)L.out & 15u) != 0) return hipErrorInvalidValue;
  const u64 nblk = a5x_digest_blocks(L.nbytes, L.algo);
  const u64 want = (nblk + 3) / 4;
  const u32 g = (u32)(want < grid ? want : grid);
  if (L.algo == A5X_ALGO_MD5)
    hipLaunchKernelGGL(k_digest_stream<true>, dim3(g), dim3(256), a5x_digest_lds(L.algo), st, L, op);
  else
    hipLaunchKernelGGL(k_digest_stream<false>, dim3(g), dim3(256), a5x_digest_lds(L.algo), st, L, op);
  return hipGetLastError();
}

uint64_t a5x_digest_blocks(uint64_t nbytes, int algo) {
  const u64 b = algo == A5X_ALGO_MD5 ? DCfg<true>::BLK : DCfg<false>::BLK;
  return (nbytes + b - 1) / b;
}

hipError_t a5x_launch_hits_resolve(A5xHitRaw* hits, uint32_t n, const uint64_t* blk_pre, uint64_t cand_base,
                                   const uint64_t* cand_off, uint64_t nw, hipStream_t st) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_hits_resolve, dim3((n + 63) / 64 < 4096 ? (n + 63) / 64 : 4096), dim3(64), 0, st, hits, n,
                     blk_pre, cand_base, cand_off, nw);
  return hipGetLastError();
}
