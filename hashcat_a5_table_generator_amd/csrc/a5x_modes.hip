// a5x_modes.hip -- gfx950 kernels for the -r, -s and -s -r engines.
//
//   -r     processWordReverse              /root/reference/main.go:208-261 (+263-305)
//   -s     processWordSubstituteAll        /root/reference/main.go:308-365
//   -s -r  processWordSubstituteAllReverse /root/reference/main.go:369-440
//
// The three engines enumerate subsets of a per-word list with a size window:
//   -r     non-overlapping subsets of the match positions (start, keyLength) of
//          the ORIGINAL word (main.go:215-226, 283-305), sizes [max(min,0),
//          min(max,#positions)], each position replaced by subs[0] and applied in
//          descending index order with the reference's running offset
//          (main.go:249-257, bug-compatible; a negative start is the Go slice
//          panic, reported as A5X_E_BOUNDS);
//   -s     the sorted unique patterns present in the word (main.go:310-327), each
//          either kept or replaced by one of its values, sizes [max(min,0), max];
//          the leaf applies strings.ReplaceAll per chosen pattern (main.go:339-341);
//   -s -r  the same patterns with subs[0] only (main.go:387-392), every subset of
//          size [max(min,0), max] (the recursion of main.go:396-437 visits each once).
// Go iterates the leaf's map in random order (main.go:339, 410); the device applies
// the patterns in sorted order, one of the orders the reference can take (for
// confluent words the only result).
//
// Counting is a DP over the list with the subset size as the column (lanes over
// columns):  -r   D[j][c] = D[j+1][c] + D[next(j)][c-1]   (next = first position
//                                                            starting past j's key)
//            -s   D[i][c] = D[i+1][c] + f_i * D[i+1][c-1]  (f_i = values of pattern i;
//                                                            1 for -s -r)
// and candidate t of a word is unranked by walking the same table.  Output bytes
// are not closed-form under sequential ReplaceAll, so a length pass builds every
// candidate once and the expansion pass builds it again and writes it.
//
// Work items: (word, SEG-candidate segment); one wave per item; every lane builds
// one candidate per round in its own LDS buffer (stride 132 B: the 64 lanes' byte
// columns fall in distinct banks), a wave scan of the lengths places them, and the
// lane stores its bytes.  These engines are not the headline path.
//
// Fused digest (op 2, SURVEY 8(a) a8 for -r / -s / -s -r; README.MD:159,163 pipes
// `-s -r` into hashcat): every candidate is hashed (MD5, or NTLM over Go's UTF-16LE)
// where it is built -- the positional engine's LDS ring, the byte builder's lane
// buffer -- and probed against the target set; nothing but hits leaves the CU, and no
// length pass or output layout is needed.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "a5x.h"
#include "a5x_format.h"
#include "a5x_launch.h"
#include "a5x_md.h"
#include "a5x_ring.h"

namespace {

typedef uint64_t u64;
typedef uint32_t u32;
typedef int64_t i64;

#define M_WAVE_SYNC()                                        \
  do {                                                       \
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");   \
    __builtin_amdgcn_wave_barrier();                         \
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   \
  } while (0)

// device error bits (shared with a5x_kernels.hip's A5X_DERR_*)
constexpr u32 M_ERR_OVF = 1u << 1;
constexpr u32 M_ERR_STATE = 1u << 3;
constexpr u32 M_ERR_GUARD = 1u << 5;
constexpr u32 M_ERR_LIMIT = 1u << 6;  // word beyond the mode-engine limits
constexpr u32 M_ERR_PANIC = 1u << 7;  // -r slice-bounds panic (main.go:255)
constexpr u32 M_ERR_CLEN = 1u << 8;   // a candidate longer than the lane buffer
constexpr u32 M_ERR_GWORD = 1u << 30; // (not an error) word longer than A5X_M_LMAX: mode pass G
constexpr u64 M_WB_FAST = 1ull << 62;   // k_mode_count's wbytes of a single-item word: route MI_FAST
constexpr u64 M_WB_FAST2 = 1ull << 61;  // ... route MI_FAST2 (the piece layout with room for more entries)


// positional -s / -s -r words (m_pos_setup): entries (a5x_ring.h) and the token list
constexpr u32 MP_NE = 256;    // entries per word: per pattern [keep, values...], then literal chunks
constexpr u32 MP_PMAX = 16;   // patterns per word (4-bit selector per pattern)
constexpr u32 MP_VMAX = 14;   // values per pattern (selector 1 + v <= 15)

// Per-wave state of one word: LDS (MLds), or an HBM scratch slot for the words of
// mode pass G (MLdsG: lines up to 64 KiB, candidates up to A5X_MG_CBUF - 1 bytes; the
// positional engine, which places through LDS addresses, is not used there).
// NBUF: bytes of the candidate buffers -- the byte builder's two per-lane buffers
// (2 x 64 x STRIDE), the positional engine's ring only (MP_RING), or none (counting
// and closed-form lengths): the smaller layouts run more waves per CU.
constexpr u32 MP_RING = 16 + 64 * A5X_M_CBUF + 48;
// radix words (MInfo::radix), piece expansion (m_fast_expand): the multi-token pieces'
// entries follow the token entries (ent[MP_NE ..]); pieces of one word
#ifndef MF_NPE
#define MF_NPE 128           // multi-token piece entries per word (the piece layout's LDS; 256: C5 -s 10 % slower, 9 vs 11 waves per CU)
#endif
#ifndef MF_NE
#define MF_NE 64             // token entries of the small piece layout (MLdsF, 14 waves per CU);
                             // MF_NE2 in the large one (MLdsF2); words needing more entries (m_pos_setup's
                             // count, S.nent) run on the token ring.  C5 -s: 128 in MLdsF -> 15 % slower
#endif
#ifndef MF_NE2
#define MF_NE2 128
#endif
#ifndef M_PREFETCH
#define M_PREFETCH 1         // m_items: the next item's metadata and word bytes loaded under the current item
#endif
#ifndef MF_TCAP
#define MF_TCAP 48           // tokens (and so pieces) per word in the piece layout; more: the token ring
#endif
#ifndef MF_RING
#define MF_RING 3072         // the piece engine's ring (runs that do not fit wait a round; 4096: C5 -s 7 % slower)
#endif
#ifndef MF_K
#define MF_K 2               // leaves per lane run (odometer steps between them; C5: 2 < 4 < 8)
#endif
#ifndef MF_OFF
#define MF_OFF 0             // 1: radix words stay on the token ring (A/B builds)
#endif
#ifndef MF_ABL
#define MF_ABL 0             // timing ablations (diagnostic builds): 1 = no expansion, 2 = no pieces, 4 = no tokens
#endif
#ifndef MF_EMAX
#define MF_EMAX 64           // entries of one multi-token piece
#endif
template <u32 LMAX, u32 CBUF, u32 NBUF = 2 * 64 * (CBUF + 4), u32 DPN = A5X_M_DPMAX, u32 NPE = 0, u32 NE = MP_NE,
          u32 TC = A5X_M_LMAX + 2>
struct MLdsT {
  static constexpr u32 TCAP = TC;              // tokens per word
  static constexpr u32 N_E = NE;               // token entries (patterns' choices, literal chunks)
  static constexpr u32 ZE = NE + NPE - 1;      // the piece layout's empty entry
  static constexpr u32 L_MAX = LMAX, STRIDE = CBUF + 4, CMAXLEN = CBUF - 1;
  static constexpr bool G = LMAX > A5X_M_LMAX;
  static constexpr bool BUILDER = NBUF >= 2 * 64 * STRIDE, RING = NBUF >= MP_RING;
  static constexpr bool FAST = NPE > 0;  // piece engine layout: no DP table (radix words only)
  u64 dp[DPN ? DPN : 1];
  uint4 ent[NE + NPE];
  uint4 pdesc[NPE ? TC : 1];  // pieces: entry base (bias folded) | selector shifts | strides | sources
  u32 tok[TC];               // entry base | (pattern index + 1) << 16 (0: literal chunk)
  uint8_t mpi[A5X_M_LMAX];   // pattern index + 1 matched at byte q (0: none)
  uint8_t pb[MP_PMAX], occ[MP_PMAX];
  uint8_t elen[NE + NPE];    // entry lengths
  u32 rmag[MP_PMAX];         // radix mode: magic of R_r = 1 + values of pattern r
  uint8_t rr[MP_PMAX];       // R_r
  u32 ntok, radix, shift, nent;  // (nent: token entries m_pos_setup used)
  u32 bitmap[A5X_MTAB_KEYS_MAX / 32];
  alignas(16) uint8_t word[LMAX + 16];
  uint16_t pat[64];          // key index per sorted pattern (-s) / per position (-r)
  uint16_t pst[64];          // -r: start byte
  uint8_t pnx[64];           // -r: first later compatible position
  alignas(16) uint8_t buf[NBUF];
};
typedef MLdsT<A5X_M_LMAX, A5X_M_CBUF> MLds;                // byte builder (general words)
typedef MLdsT<A5X_M_LMAX, A5X_M_CBUF, MP_RING> MLdsR;      // positional expansion
typedef MLdsT<A5X_M_LMAX, A5X_M_CBUF, 16> MLdsC;           // counts, closed-form lengths
typedef MLdsT<A5X_M_LMAX, A5X_M_CBUF, MF_RING + 48, 0, MF_NPE, MF_NE, MF_TCAP> MLdsF;    // piece expansion (radix words)
typedef MLdsT<A5X_M_LMAX, A5X_M_CBUF, MF_RING + 48, 0, MF_NPE, MF_NE2, MF_TCAP> MLdsF2;  // ... with more token entries
typedef MLdsT<A5X_MG_LMAX, A5X_MG_CBUF> MLdsG;             // mode pass G (HBM)

// wave sync over the word state: LDS, or (pass G) HBM written and read by the wave's own
// lanes -- workgroup-scope release / acquire drains and orders those global accesses
template <class SL>
__device__ __forceinline__ void m_sync() {
  if constexpr (SL::G) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  } else {
    M_WAVE_SYNC();
  }
}

struct MT {
  const A5xMHdr* h;
  const uint16_t* bucket;
  const A5xMKey* keys;
  const A5xMVal* vals;
  const uint8_t* blob;
};

struct MInfo {
  u32 L, n, cmin, cmax, cols;
  u64 count;
  u32 bad;    // M_ERR_* of the word (0: fine)
  u32 radix;  // leaves = every choice vector (no size window cuts): leaf t <-> t + cmin as a
              // mixed radix over the patterns (-s, -s -r: R = 1 + values) or the position bit
              // set (-r, positions pairwise disjoint: binary counting)
};

__device__ __forceinline__ u32 m_lane() { return __lane_id(); }

// 4 bytes at byte offset off of a 4-aligned LDS byte array (two dword reads + funnel shift)
__device__ __forceinline__ u32 m_lds4(const uint8_t* base, u32 off) {
  const u32* p = (const u32*)(base + (off & ~3u));
  return __builtin_amdgcn_alignbyte(p[1], p[0], off & 3u);
}

__device__ __forceinline__ u32 m_incl_scan(u32 x) {
  const u32 lane = m_lane();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const u32 y = (u32)__shfl_up((int)x, d, 64);
    if ((int)lane >= d) x += y;
  }
  return x;
}

__device__ __forceinline__ u32 m_wave_or(u32 x) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) x |= (u32)__shfl_xor((int)x, d, 64);
  return x;
}

__device__ __forceinline__ u64 m_uniform64(u64 x) {
  const u32 lo = (u32)__builtin_amdgcn_readfirstlane((int)(u32)x);
  const u32 hi = (u32)__builtin_amdgcn_readfirstlane((int)(u32)(x >> 32));
  return ((u64)hi << 32) | lo;
}

__device__ __forceinline__ u64 m_readlane64(u64 x, u32 l) {
  const u32 lo = (u32)__builtin_amdgcn_readlane((int)(u32)x, (int)l);
  const u32 hi = (u32)__builtin_amdgcn_readlane((int)(u32)(x >> 32), (int)l);
  return ((u64)hi << 32) | lo;
}

__device__ __forceinline__ MT m_table(uint8_t* lds, const uint8_t* g, u32 bytes) {
  // stage the mode table (16-B granules, the blob is 16-B padded by the host)
  const uint4* src = (const uint4*)g;
  uint4* dst = (uint4*)lds;
  for (u32 i = threadIdx.x; i < bytes / 16; i += blockDim.x) dst[i] = src[i];
  __syncthreads();
  MT T;
  T.h = (const A5xMHdr*)lds;
  T.bucket = (const uint16_t*)(lds + T.h->off_bucket);
  T.keys = (const A5xMKey*)(lds + T.h->off_keys);
  T.vals = (const A5xMVal*)(lds + T.h->off_vals);
  T.blob = lds + T.h->off_blob;
  return T;
}

// does key k match the word at q (length L)?  w4 = m_lds4(wd, q): the key's first 4
// bytes in one masked dword compare (the blob is 16-B aligned with an 8-byte tail)
__device__ __forceinline__ bool m_match4(const MT& T, const uint8_t* wd, u32 L, u32 q, u32 w4, u32 k) {
  const A5xMKey K = T.keys[k];
  if (K.klen == 0 || q + K.klen > L) return false;
  const u32 n4 = K.klen < 4u ? (u32)K.klen : 4u;
  const u32 mask = n4 == 4u ? ~0u : (1u << (8u * n4)) - 1u;
  if ((w4 ^ m_lds4(T.blob, K.key_off)) & mask) return false;
  const uint8_t* p = T.blob + K.key_off;
  for (u32 i = 4; i < K.klen; i++)
    if (wd[q + i] != p[i]) return false;
  return true;
}

// utf8.DecodeRuneInString width (invalid -> 1), as strings.Replace steps runes
// for an empty old (Go 1.23 unicode/utf8)
__device__ __forceinline__ u32 m_rune_len(const uint8_t* s, u32 n) {
  const u32 b0 = s[0];
  if (b0 < 0x80u) return 1;
  u32 size, lo = 0x80u, hi = 0xBFu;
  if (b0 >= 0xC2u && b0 <= 0xDFu) size = 2;
  else if (b0 >= 0xE0u && b0 <= 0xEFu) {
    size = 3;
    if (b0 == 0xE0u) lo = 0xA0u;
    else if (b0 == 0xEDu) hi = 0x9Fu;
  } else if (b0 >= 0xF0u && b0 <= 0xF4u) {
    size = 4;
    if (b0 == 0xF0u) lo = 0x90u;
    else if (b0 == 0xF4u) hi = 0x8Fu;
  } else {
    return 1;
  }
  if (n < size) return 1;
  if (s[1] < lo || s[1] > hi) return 1;
  for (u32 k = 2; k < size; k++)
    if (s[k] < 0x80u || s[k] > 0xBFu) return 1;
  return size;
}

// strings.ReplaceAll(src[:n], p, v) into dst; returns the length (err |= CLEN when
// the result does not fit the lane buffer)
__device__ u32 m_replace_all(const uint8_t* src, u32 n, const uint8_t* p, u32 pl, const uint8_t* v, u32 vl,
                             uint8_t* dst, u32& err, const u32 CMAXLEN) {
  u32 o = 0;
  if (pl == 0) {  // "" matches before every rune and at the end
    if (vl > CMAXLEN) { err |= M_ERR_CLEN; return 0; }
    for (u32 k = 0; k < vl; k++) dst[o++] = v[k];
    u32 i = 0;
    while (i < n) {
      const u32 sz = m_rune_len(src + i, n - i);
      if (o + sz + vl > CMAXLEN) { err |= M_ERR_CLEN; return 0; }
      for (u32 k = 0; k < sz; k++) dst[o++] = src[i + k];
      for (u32 k = 0; k < vl; k++) dst[o++] = v[k];
      i += sz;
    }
    return o;
  }
  const uint8_t p0 = p[0];
  u32 i = 0;
  while (i < n) {
    bool m = src[i] == p0 && i + pl <= n;
    for (u32 k = 1; m && k < pl; k++) m = src[i + k] == p[k];
    if (m) {
      if (o + vl > CMAXLEN) { err |= M_ERR_CLEN; return 0; }
      for (u32 k = 0; k < vl; k++) dst[o++] = v[k];
      i += pl;
    } else {
      if (o + 1 > CMAXLEN) { err |= M_ERR_CLEN; return 0; }
      dst[o++] = src[i++];
    }
  }
  return o;
}

// An item's word metadata and bytes, loaded by m_items while the wave still runs the
// previous item (the per-item chain of dependent global loads off the critical path):
// w0 / w1 = woff[w], woff[w + 1]; c0 / c1 = cand_off[w], cand_off[w + 1]; s0 = seg_off[w];
// b0 / b1 = word bytes lane and lane + 64.
struct MPre {
  u64 w0, w1, c0, c1, s0;
  u32 b0, b1;
};

// Per-word setup (wave-uniform result): word -> LDS, the pattern / position list,
// the DP table and the count.
// dp = false: a radix word's count in closed form, no DP table (callers that never
// unrank a leaf through it: k_mode_count)
template <class SL>
__device__ MInfo m_setup(SL& S, const MT& T, const A5xModeLaunch& a, u64 w, bool dp = true,
                         const MPre* pre = nullptr) {
  const u32 lane = m_lane();
  MInfo I;
  I.L = I.n = I.cmin = I.cmax = I.cols = 0;
  I.count = 0;
  I.bad = 0;
  const u64 w0 = pre ? pre->w0 : a.woff[w], w1 = pre ? pre->w1 : a.woff[w + 1];
  if (w1 - w0 > SL::L_MAX) { I.bad = w1 - w0 <= A5X_MG_LMAX ? M_ERR_GWORD : M_ERR_LIMIT; return I; }
  const u32 L = (u32)(w1 - w0);
  I.L = L;
  m_sync<SL>();  // previous item's readers of S are done
  if (pre) {
    if (lane < L) S.word[lane] = (uint8_t)pre->b0;
    if (lane + 64 < L) S.word[lane + 64] = (uint8_t)pre->b1;
  } else {
    for (u32 i = lane; i < L; i += 64) S.word[i] = a.words[w0 + i];
  }
  m_sync<SL>();
  u32 n = 0;
  if (a.mode == A5X_MODE_REVERSE) {
    // positions in (start, keyLength) order (main.go:215-226): starts q = lane, lane+64
    for (u32 q0 = 0; q0 < L; q0 += 64) {
      const u32 q = q0 + lane;
      u32 k0 = 0, k1 = 0, m = 0, w4 = 0;
      u64 mb = 0;  // matches among the bucket's first 64 keys
      if (q < L) {
        const u32 b = S.word[q];
        k0 = T.bucket[b];
        k1 = T.bucket[b + 1];
        w4 = m_lds4(S.word, q);
        for (u32 k = k0; k < k1; k++)
          if (m_match4(T, S.word, L, q, w4, k)) {
            m++;
            if (k - k0 < 64) mb |= 1ull << (k - k0);
          }
      }
      const u32 incl = m_incl_scan(m);
      const u32 tot = (u32)__builtin_amdgcn_readlane((int)incl, 63);
      u32 o = n + incl - m;
      if (n + tot <= A5X_M_NMAX && m) {
        for (u64 x = mb; x; x &= x - 1) {
          S.pat[o] = (uint16_t)(k0 + (u32)__builtin_ctzll(x));
          S.pst[o] = (uint16_t)q;
          o++;
        }
        for (u32 k = k0 + 64; k < k1; k++)
          if (m_match4(T, S.word, L, q, w4, k)) { S.pat[o] = (uint16_t)k; S.pst[o] = (uint16_t)q; o++; }
      }
      n += tot;
    }
    if (n > A5X_M_NMAX) { I.bad = M_ERR_LIMIT; return I; }
    m_sync<SL>();
    if (lane < n) {
      const u32 end = S.pst[lane] + T.keys[S.pat[lane]].klen;
      u32 nx = n;
      for (u32 k = lane + 1; k < n; k++)
        if (S.pst[k] >= end) { nx = k; break; }
      S.pnx[lane] = (uint8_t)nx;
    }
  } else {
    // unique patterns present (main.go:312-319), sorted = increasing key index
    const u32 nk = T.h->nkeys, nwd = (nk + 31) / 32;
    for (u32 i = lane; i < nwd; i += 64) S.bitmap[i] = 0;
    m_sync<SL>();
    for (u32 q = lane; q < L; q += 64) {
      const u32 b = S.word[q], w4 = m_lds4(S.word, q);
      for (u32 k = T.bucket[b]; k < T.bucket[b + 1]; k++)
        if (m_match4(T, S.word, L, q, w4, k)) atomicOr(&S.bitmap[k >> 5], 1u << (k & 31));
    }
    if (T.h->has_empty && L > 0 && lane == 0) atomicOr(&S.bitmap[0], 1u);
    m_sync<SL>();
    // (pass G: the bitmap was built by L2 atomics; read it from L2, not a stale L1 line)
    auto bm = [&](u32 i) -> u32 {
      if constexpr (SL::G) return __hip_atomic_load(&S.bitmap[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else return S.bitmap[i];
    };
    const u32 d0 = 2 * lane < nwd ? bm(2 * lane) : 0u;
    const u32 d1 = 2 * lane + 1 < nwd ? bm(2 * lane + 1) : 0u;
    const u32 m = (u32)__builtin_popcount(d0) + (u32)__builtin_popcount(d1);
    const u32 incl = m_incl_scan(m);
    n = (u32)__builtin_amdgcn_readlane((int)incl, 63);
    if (n > A5X_M_NMAX) { I.bad = M_ERR_LIMIT; return I; }
    u32 o = incl - m;
    for (u32 x = d0; x; x &= x - 1) S.pat[o++] = (uint16_t)(64 * lane + (u32)__builtin_ctz(x));
    for (u32 x = d1; x; x &= x - 1) S.pat[o++] = (uint16_t)(64 * lane + 32 + (u32)__builtin_ctz(x));
  }
  I.n = n;
  I.radix = 0;
  if (a.mx < 0) return I;
  const u32 cmax = min((u32)a.mx, n);
  const u32 cmin = a.mn > 0 ? (u32)a.mn : 0u;
  if (cmin > cmax) return I;
  const u32 cols = cmax + 1;
  I.cmin = cmin; I.cmax = cmax; I.cols = cols;
  m_sync<SL>();
  // radix words: the size window [cmin, cmax] keeps every choice vector but (cmin = 1) the
  // all-keep one; -r also needs pairwise disjoint positions (every subset is a leaf)
  bool rad = cmin <= 1 && cmax >= n;
  u64 rcount = 0;  // their count in closed form
  if (a.mode == A5X_MODE_REVERSE) {
    rad = rad && n <= 62 && !__ballot(lane < n && S.pnx[lane] != lane + 1);
    rcount = rad ? (1ull << n) - cmin : 0;
  } else if (rad) {
    u32 R = 1;
    if (lane < n) {
      const u32 nv = T.keys[S.pat[lane]].nvals;
      R = 1 + (a.mode == A5X_MODE_SUBALL ? nv : (nv ? 1u : 0u));
    }
    u64 P = 1;
    for (u32 r = 0; r < n && P < (1ull << 27); r++) P *= (u32)__builtin_amdgcn_readlane((int)R, (int)r);
    rad = P < (1ull << 27);
    rcount = rad ? P - cmin : 0;
  }
  // (the limit holds for every layout, so that every kernel agrees on the word)
  if ((n + 1) * cols > A5X_M_DPMAX) { I.bad = M_ERR_LIMIT; return I; }
  if (SL::FAST || (!dp && rad)) {  // (the piece layout has no DP table: radix words only)
    if (!rad) { I.bad = M_ERR_STATE; return I; }
    I.radix = 1;
    I.count = rcount;
    return I;
  }
  u64* D = S.dp;
  const u32 c = lane;
  if (c < cols) D[n * cols + c] = c == 0 ? 1ull : 0ull;
  u32 ovf = 0;
  for (int r = (int)n - 1; r >= 0; r--) {
    m_sync<SL>();
    if (c < cols) {
      u64 x = D[(r + 1) * cols + c];
      if (c > 0) {
        u64 y;
        if (a.mode == A5X_MODE_REVERSE) {
          y = D[S.pnx[r] * cols + c - 1];
        } else {
          u64 f = T.keys[S.pat[r]].nvals;
          if (a.mode == A5X_MODE_SUBALL_REVERSE) f = f ? 1u : 0u;
          if (__builtin_mul_overflow(f, D[(r + 1) * cols + c - 1], &y)) { ovf = 1; y = ~0ull; }
        }
        if (__builtin_add_overflow(x, y, &x)) { ovf = 1; x = ~0ull; }
      }
      D[r * cols + c] = x;
    }
  }
  m_sync<SL>();
  u64 cnt = 0;
  for (u32 k = cmin; k <= cmax; k++)
    if (__builtin_add_overflow(cnt, D[k], &cnt)) ovf = 1;
  if (m_wave_or(ovf)) { I.bad = M_ERR_OVF; return I; }
  I.count = m_uniform64(cnt);
  if (rad && I.count != rcount) { I.bad = M_ERR_STATE; return I; }
  I.radix = rad ? 1u : 0u;
  return I;
}

// -r: leaf t -> the chosen non-overlapping positions (bit j = position j)
template <class SL>
__device__ __forceinline__ u64 m_rsel(const SL& S, const MInfo& I, u64 t, u32& err) {
  if (I.radix) return t + I.cmin;  // binary counting over the disjoint positions
  const u64* D = S.dp;
  const u32 cols = I.cols, n = I.n;
  u32 c = I.cmin;
  while (c < I.cmax && t >= D[c]) { t -= D[c]; c++; }
  u64 sel = 0;
  u32 r = 0;
  while (c > 0) {
    if (r >= n) { err |= M_ERR_STATE; break; }
    const u64 a0 = D[(r + 1) * cols + c];
    if (t < a0) { r++; continue; }
    t -= a0;
    sel |= 1ull << r;
    r = S.pnx[r];
    c--;
  }
  return sel;
}

// -r: the candidate's length does not depend on where (or how wrongly) the replacements
// land: L + sum (|subs[0]| - |key|); panics surface in the expansion pass, which builds it
template <class SL>
__device__ __forceinline__ u32 m_rlen(const SL& S, const MT& T, const MInfo& I, u64 sel) {
  int l = (int)I.L;
  for (u64 m = sel; m; m &= m - 1) {
    const A5xMKey K = T.keys[S.pat[__builtin_ctzll(m)]];
    if (K.nvals) l += (int)T.vals[K.val_base].len - (int)K.klen;
  }
  return (u32)l;
}

// Build candidate t (0 <= t < count) of the word set up in S into this lane's
// buffer; returns its length and the buffer holding it.
template <class SL>
__device__ u32 m_build(SL& S, const MT& T, const MInfo& I, int mode, u64 t, const uint8_t** outp, u32& err,
                       bool len_only = false) {
  const u32 lane = m_lane();
  constexpr u32 CMAXLEN = SL::CMAXLEN;
  static_assert(SL::BUILDER, "m_build needs the builder layout");
  uint8_t* b0 = S.buf + lane * SL::STRIDE;
  uint8_t* b1 = S.buf + (64 + lane) * SL::STRIDE;
  const u64* D = S.dp;
  const u32 cols = I.cols, n = I.n;
  if (mode == A5X_MODE_REVERSE) {
    u64 sel = m_rsel(S, I, t, err);
    u32 len = I.L;
    if (len_only) {
      *outp = nullptr;
      return m_rlen(S, T, I, sel);
    }
    for (u32 i = 0; i < len; i++) b0[i] = S.word[i];
    // combo indices descending, running offset (main.go:249-257)
    int off = 0;
    while (sel) {
      const u32 j = 63u - (u32)__builtin_clzll(sel);
      sel &= ~(1ull << j);
      const A5xMKey K = T.keys[S.pat[j]];
      if (K.nvals == 0) { err |= M_ERR_PANIC; break; }  // pos.subs[0] on an empty list
      const A5xMVal V = T.vals[K.val_base];
      const int st = (int)S.pst[j] + off;
      if (st < 0) { err |= M_ERR_PANIC; break; }       // result[:actualStart], actualStart < 0
      const int dl = (int)V.len - (int)K.klen;
      const int nl = (int)len + dl;
      if (nl > (int)CMAXLEN) { err |= M_ERR_CLEN; break; }
      const u32 tail = (u32)st + K.klen;  // <= len
      if (dl > 0) {
        for (u32 i = len; i-- > tail;) b0[i + dl] = b0[i];
      } else if (dl < 0) {
        for (u32 i = tail; i < len; i++) b0[i + dl] = b0[i];
      }
      const uint8_t* v = T.blob + V.off;
      for (u32 i = 0; i < V.len; i++) b0[st + i] = v[i];
      len = (u32)nl;
      off += dl;
    }
    *outp = b0;
    return len;
  }
  // -s / -s -r: chosen patterns in sorted order, ReplaceAll each (main.go:339-341)
  u32 c = I.cmin;
  while (c < I.cmax && t >= D[c]) { t -= D[c]; c++; }
  const uint8_t* src = S.word;
  uint8_t* dst = b0;
  u32 len = I.L;
  for (u32 r = 0; r < n && c > 0; r++) {
    const u64 a0 = D[(r + 1) * cols + c];
    if (t < a0) continue;
    t -= a0;
    const A5xMKey K = T.keys[S.pat[r]];
    u32 v = 0;
    if (mode == A5X_MODE_SUBALL && K.nvals > 1) {
      const u64 b = D[(r + 1) * cols + c - 1];
      v = (u32)(t / b);
      t -= (u64)v * b;
    }
    const A5xMVal V = T.vals[K.val_base + v];
    len = m_replace_all(src, len, T.blob + K.key_off, K.klen, T.blob + V.off, V.len, dst, err, CMAXLEN);
    src = dst;
    dst = dst == b0 ? b1 : b0;
    c--;
  }
  *outp = src;
  return len;
}

// ---------------------------------------------------------------------------
// Positional -s / -s -r words.  When every pattern present in the word is one valid
// UTF-8 codepoint, every value of those patterns is valid UTF-8 of <= 15 bytes, and no
// value of a pattern contains a LATER (sorted) pattern, the sequential ReplaceAll of a
// leaf (main.go:339-341, applied in sorted order) equals replacing each ORIGINAL
// occurrence of a chosen pattern by its value: occurrences of distinct codepoints never
// overlap, a valid value cannot complete a codepoint across its boundaries, and only a
// later pass could rewrite an inserted value.  Such a word is a token list (literal
// chunks and pattern occurrences); a candidate is the concatenation of its tokens'
// entries (a5x_ring.h) picked by the leaf's per-pattern choice, and its length is
// L + sum_p occ_p (|v_p| - |p|): no pass builds a candidate only to measure it.
// ---------------------------------------------------------------------------
__device__ bool m_valid_utf8(const uint8_t* p, u32 n) {
  for (u32 i = 0; i < n;) {
    const u32 sz = m_rune_len(p + i, n - i);
    if (sz == 1 && p[i] >= 0x80u) return false;
    i += sz;
  }
  return true;
}

__device__ bool m_contains(const uint8_t* h, u32 hn, const uint8_t* nd, u32 nn) {
  for (u32 i = 0; i + nn <= hn; i++) {
    u32 k = 0;
    while (k < nn && h[i + k] == nd[k]) k++;
    if (k == nn) return true;
  }
  return false;
}

__device__ __forceinline__ uint4 m_entry(const uint8_t* p, u32 n) {
  u64 lo = 0, hi = 0;
  for (u32 i = 0; i < n; i++) {
    if (i < 8) lo |= (u64)p[i] << (8 * i);
    else hi |= (u64)p[i] << (8 * (i - 8));
  }
  return make_uint4((u32)lo, (u32)(lo >> 32), (u32)hi, (u32)(hi >> 32) | (n << 24));
}

// -r positional words: every position's key and subs[0] have the same length (so the
// running-offset bug of main.go:249-257 moves nothing), positions do not overlap, and
// each key has a value (no panic).  A leaf is then the word with each chosen position's
// bytes replaced in place: tokens = literal chunks and positions (entries [key, subs[0]],
// selected by bit j of the leaf's position set), every candidate L + 1 bytes long.
template <class SL>
__device__ u32 m_rpos_setup(SL& S, const MT& T, const MInfo& I) {
  const u32 lane = m_lane(), n = I.n, L = I.L;
  if (n == 0 || L > A5X_M_LMAX) return 0;
  u32 ok = 1;
  if (lane < n) {
    const A5xMKey K = T.keys[S.pat[lane]];
    ok = K.nvals >= 1 && K.klen >= 1 && K.klen <= 15 && T.vals[K.val_base].len == K.klen &&
         (lane + 1 >= n || (u32)S.pst[lane] + K.klen <= (u32)S.pst[lane + 1]);
  }
  if (__ballot(!ok)) return 0;
  m_sync<SL>();
  if (lane < n) {  // position entries: [key, subs[0]] at 2 j
    const A5xMKey K = T.keys[S.pat[lane]];
    S.ent[2 * lane] = m_entry(T.blob + K.key_off, K.klen);
    S.ent[2 * lane + 1] = m_entry(T.blob + T.vals[K.val_base].off, K.klen);
  }
  m_sync<SL>();
  // tokens in byte order, lane-parallel: lane j <= n takes the literal gap before
  // position j (j == n: after the last one), cut into <= 15-byte chunks, then position j
  u32 gs = 0, ge = 0;
  if (lane <= n) {
    gs = lane == 0 ? 0u : (u32)S.pst[lane - 1] + T.keys[S.pat[lane - 1]].klen;
    ge = lane < n ? (u32)S.pst[lane] : L;
  }
  const u32 nch = (lane <= n && ge > gs) ? (ge - gs + 14u) / 15u : 0u;
  const u32 ntk = nch + (lane < n ? 1u : 0u);
  const u32 tinc = m_incl_scan(ntk), cinc = m_incl_scan(nch);
  const u32 nt = (u32)__builtin_amdgcn_readlane((int)tinc, 63);
  const u32 nlit = (u32)__builtin_amdgcn_readlane((int)cinc, 63);
  const bool over = 2 * n + nlit > SL::N_E || nt > SL::TCAP;
  if (!over && lane <= n) {
    const u32 t = tinc - ntk, e = 2 * n + cinc - nch;
    for (u32 c = 0; c < nch; c++) {
      const u32 q = gs + 15u * c, len = min(15u, ge - q);
      u64 lo = 0, hi = 0;
      for (u32 k = 0; k < len; k++) {
        const u64 x = S.word[q + k];
        if (k < 8) lo |= x << (8 * k); else hi |= x << (8 * (k - 8));
      }
      S.ent[e + c] = make_uint4((u32)lo, (u32)(lo >> 32), (u32)hi, (u32)(hi >> 32) | (len << 24));
      S.tok[t + c] = e + c;
    }
    if (lane < n) S.tok[t + nch] = (2 * lane) | ((lane + 1) << 16);
  }
  if (lane == 0) {
    S.ntok = over ? 0u : nt;
    S.nent = 2 * n + nlit;
    S.radix = 0;
  }
  m_sync<SL>();
  return (u32)__builtin_amdgcn_readfirstlane((int)S.ntok);
}

// Tokens and entries of the word set up in S (after m_setup): returns the token count,
// or 0 when the word is not positional (byte builder path).
// check = false: the word is known positional (its item was routed MI_FAST by the
// length pass, which ran the checks): the per-value checks are skipped.
template <class SL>
__device__ u32 m_pos_setup(SL& S, const MT& T, const MInfo& I, int mode, bool check = true) {
  if (mode == A5X_MODE_REVERSE) return m_rpos_setup(S, T, I);
  const u32 lane = m_lane(), n = I.n, L = I.L;
  if (n == 0 || n > MP_PMAX || L > A5X_M_LMAX) return 0;
  u32 ok = 1, ne = 0;
  if (lane < n) {
    const A5xMKey K = T.keys[S.pat[lane]];
    const uint8_t* kp = T.blob + K.key_off;
    const u32 nv = mode == A5X_MODE_SUBALL ? K.nvals : (K.nvals ? 1u : 0u);
    if (check)
      ok = K.klen >= 1 && K.klen <= 4 && m_rune_len(kp, K.klen) == K.klen && (K.klen > 1 || kp[0] < 0x80u) &&
           nv <= MP_VMAX;
    for (u32 v = 0; check && ok && v < nv; v++) {
      const A5xMVal V = T.vals[K.val_base + v];
      const uint8_t* vp = T.blob + V.off;
      ok = V.len <= 15 && m_valid_utf8(vp, V.len);
      for (u32 j = lane + 1; ok && j < n; j++) {
        const A5xMKey Kj = T.keys[S.pat[j]];
        ok = !m_contains(vp, V.len, T.blob + Kj.key_off, Kj.klen);
      }
    }
    ne = 1 + nv;
  }
  if (__ballot(!ok)) return 0;
  const u32 incl = m_incl_scan(ne);
  const u32 npe = (u32)__builtin_amdgcn_readlane((int)incl, 63);
  if (npe > SL::N_E) return 0;
  M_WAVE_SYNC();
  if (lane < n) {  // pattern entries: [keep, value 0, value 1, ...]
    const u32 b = incl - ne;
    const A5xMKey K = T.keys[S.pat[lane]];
    S.pb[lane] = (uint8_t)b;
    S.occ[lane] = 0;
    S.ent[b] = m_entry(T.blob + K.key_off, K.klen);
    for (u32 v = 0; v + 1 < ne; v++) {
      const A5xMVal V = T.vals[K.val_base + v];
      S.ent[b + 1 + v] = m_entry(T.blob + V.off, V.len);
    }
  }
  // Occurrences and the token list, lane-parallel over bytes (L <= 128: two passes of
  // 64).  Patterns are single codepoints (<= 4 bytes, compared as one masked dword), so at
  // most one starts at a byte and occurrences never overlap; literal bytes form runs cut
  // into <= 15-byte chunks.  Tokens in byte order: occurrences, literal chunks.
  u32 pkey = 0, pmask = 0, plen = 0;
  if (lane < n) {
    const A5xMKey K = T.keys[S.pat[lane]];
    const uint8_t* kp = T.blob + K.key_off;
    for (u32 i = 0; i < K.klen; i++) pkey |= (u32)kp[i] << (8 * i);
    plen = K.klen;
    pmask = plen >= 4 ? 0xffffffffu : ((1u << (8 * plen)) - 1u);
  }
  for (u32 q0 = 0; q0 < L; q0 += 64) {
    const u32 q = q0 + lane;
    u32 m = 0;
    if (q < L) {
      const u32 w4 = m_lds4(S.word, q);
      for (u32 i = 0; i < n; i++) {
        const u32 ki = (u32)__builtin_amdgcn_readlane((int)pkey, (int)i);
        const u32 mi = (u32)__builtin_amdgcn_readlane((int)pmask, (int)i);
        const u32 li = (u32)__builtin_amdgcn_readlane((int)plen, (int)i);
        if (!m && (w4 & mi) == ki && q + li <= L) m = i + 1;
      }
      S.mpi[q] = (uint8_t)m;
    }
  }
  M_WAVE_SYNC();
  u32 nt = 0, nlit = 0, rs_carry = 0, occ = 0;
  for (u32 q0 = 0; q0 < L; q0 += 64) {  // token starts, in order; positions -> S.elen (free here)
    const u32 q = q0 + lane;
    const bool in = q < L;
    const u32 m = in ? S.mpi[q] : 0u;
    bool cov = false;  // inside an occurrence that starts at q - 1 .. q - 3
    for (u32 d = 1; d <= 3; d++) {
      const u32 md = (in && q >= d) ? S.mpi[q - d] : 0u;
      const u32 ld = (u32)__shfl((int)plen, (int)(md ? md - 1 : 0));
      cov = cov || (md && ld > d);
    }
    const bool lit = in && !m && !cov;
    bool litp = false;  // byte q - 1 literal (lane 0: from the previous pass)
    {
      const u32 mp = (in && q >= 1) ? S.mpi[q - 1] : 1u;
      bool covp = false;
      for (u32 d = 2; d <= 4; d++) {
        const u32 md = (in && q >= d) ? S.mpi[q - d] : 0u;
        const u32 ld = (u32)__shfl((int)plen, (int)(md ? md - 1 : 0));
        covp = covp || (md && ld > d - 1);
      }
      litp = q >= 1 && !mp && !covp;
    }
    // start of this byte's literal run (segmented max scan over lanes)
    u32 rs = lit && !litp ? q + 1 : 0u;  // (q + 1: 0 = none)
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const u32 y = (u32)__shfl_up((int)rs, d, 64);
      if ((int)lane >= d) rs = max(rs, y);
    }
    rs = max(rs, rs_carry);
    const u32 runq = rs ? rs - 1 : 0u;
    const bool lstart = lit && ((q - runq) % 15u == 0u);
    const bool tstart = (in && m) || lstart;
    const u64 tb = __ballot(tstart), lb = __ballot(lstart);
    const u32 ti = nt + (u32)__popcll(tb & ((1ull << lane) - 1ull));
    const u32 li = nlit + (u32)__popcll(lb & ((1ull << lane) - 1ull));
    if (tstart && ti < SL::TCAP) {
      S.elen[ti] = (uint8_t)q;
      S.tok[ti] = m ? (S.pb[m - 1] | (m << 16)) : (npe + li);
    }
    for (u32 i = 0; i < n; i++) {
      const u32 c = (u32)__popcll(__ballot(in && m == i + 1));
      if (lane == i) occ += c;
    }
    nt += (u32)__popcll(tb);
    nlit += (u32)__popcll(lb);
    rs_carry = (u32)__builtin_amdgcn_readlane((int)rs, 63);
  }
  const bool over = npe + nlit > SL::N_E || nt > SL::TCAP;
  if (lane < n) S.occ[lane] = (uint8_t)occ;
  M_WAVE_SYNC();
  if (!over) {  // literal chunk entries: bytes [q, next token start)
    for (u32 k = lane; k < nt; k += 64) {
      const u32 d = S.tok[k];
      if (d >> 16) continue;
      const u32 q = S.elen[k], qe = k + 1 < nt ? (u32)S.elen[k + 1] : L, len = qe - q;
      const u32 x0 = m_lds4(S.word, q), x1 = m_lds4(S.word, q + 4), x2 = m_lds4(S.word, q + 8), x3 = m_lds4(S.word, q + 12);
      u64 lo = (u64)x0 | ((u64)x1 << 32), hi = (u64)x2 | ((u64)x3 << 32);
      lo = len >= 8 ? lo : (lo & ((1ull << (8 * len)) - 1ull));
      hi = len >= 16 ? hi : len > 8 ? (hi & ((1ull << (8 * (len - 8))) - 1ull)) : 0ull;
      S.ent[d] = make_uint4((u32)lo, (u32)(lo >> 32), (u32)hi, ((u32)(hi >> 32) & 0xFFFFFFu) | (len << 24));
    }
  }
  if (lane == 0) {
    S.ntok = over ? 0u : nt;
    S.nent = npe + nlit;
    // radix mode: no effective size window (min <= 1, max >= #patterns) -- the leaves are
    // every per-pattern choice vector (minus the all-keep one when min = 1), enumerated
    // as the mixed radix over patterns (pattern 0 least significant, digit 0 = keep);
    // exact 32-bit magic division needs leaf (R - 1) < 2^32: count < 2^27
    S.radix = I.radix;
    S.shift = I.cmin;  // leaf 0 (all keep) skipped when min = 1
  }
  if (lane < n) {
    const A5xMKey K = T.keys[S.pat[lane]];
    const u32 nv = mode == A5X_MODE_SUBALL ? K.nvals : (K.nvals ? 1u : 0u);
    const u32 R = 1 + nv;
    S.rr[lane] = (uint8_t)R;
    S.rmag[lane] = R > 1 ? (u32)((((u64)1 << 32) + R - 1) / R) : 0u;
  }
  for (u32 e = lane; e < SL::N_E; e += 64) S.elen[e] = (uint8_t)(S.ent[e].w >> 24);
  M_WAVE_SYNC();
  return (u32)__builtin_amdgcn_readfirstlane((int)S.ntok);
}

// Sum over leaves t in [0, x) of (len + 1) in radix mode (closed form; lanes over
// patterns): x (L + 1) + sum_r occ_r sum_{t'} delta_r(digit_r(t')), t' = t + shift.
template <class SL>
__device__ u64 m_pos_prefix(const SL& S, const MInfo& I, u64 x) {
  const u32 lane = m_lane(), n = I.n;
  auto G = [&](u64 y) -> i64 {  // this lane's pattern: sum_{t' < y} delta(digit(t'))
    if (lane >= n) return 0;
    u64 P = 1;  // place value of pattern lane
    for (u32 q = 0; q < lane; q++) P *= S.rr[q];
    const u32 b = S.pb[lane], R = S.rr[lane];
    const int k0 = S.elen[b];
    i64 sumd = 0;
    for (u32 v = 1; v < R; v++) sumd += (int)S.elen[b + v] - k0;
    const u64 cyc = P * R, full = y / cyc, rem = y - full * cyc, dv = rem / P;
    i64 g = (i64)(full * P) * sumd;
    for (u32 v = 1; v < dv; v++) g += (i64)P * ((int)S.elen[b + v] - k0);
    if (dv >= 1 && dv < R) g += (i64)(rem - dv * P) * ((int)S.elen[b + dv] - k0);
    return g * (i64)S.occ[lane];
  };
  i64 tot = G(x + S.shift) - G(S.shift);
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) tot += (i64)__shfl_xor((long long)tot, d, 64);
  return x * (u64)(I.L + 1) + (u64)tot;
}

// Leaf t of a positional word: per-pattern selectors (4 bits each: 0 keep, 1 + v value
// v) by walking the DP table as m_build does; returns the candidate length.
template <class SL>
__device__ u32 m_pos_sel(const SL& S, const MT& T, const MInfo& I, int mode, u64 t, u64& sel) {
  if (mode == A5X_MODE_REVERSE) {  // positional -r: the position set; length L
    u32 err = 0;
    sel = m_rsel(S, I, t, err);
    return I.L;
  }
  if (S.radix) {  // mixed-radix digits by magic division (pattern 0 least significant)
    u32 x = (u32)t + S.shift, len = I.L;
    u64 sv = 0;
    for (u32 r = 0; r < I.n; r++) {
      const u32 mg = S.rmag[r];
      const u32 q = __umulhi(x, mg) + (mg ? 0u : x);
      const u32 dgt = x - q * S.rr[r];
      sv |= (u64)dgt << (4 * r);
      len += (u32)((int)S.occ[r] * ((int)S.elen[S.pb[r] + dgt] - (int)S.elen[S.pb[r]]));
      x = q;
    }
    sel = sv;
    return len;
  }
  const u64* D = S.dp;
  const u32 cols = I.cols, n = I.n;
  u32 c = I.cmin;
  while (c < I.cmax && t >= D[c]) { t -= D[c]; c++; }
  int len = (int)I.L;
  u64 sv = 0;
  for (u32 r = 0; r < n && c > 0; r++) {
    const u64 a0 = D[(r + 1) * cols + c];
    if (t < a0) continue;
    t -= a0;
    const A5xMKey K = T.keys[S.pat[r]];
    u32 v = 0;
    if (mode == A5X_MODE_SUBALL && K.nvals > 1) {
      const u64 b = D[(r + 1) * cols + c - 1];
      v = ((t | b) >> 32) ? (u32)(t / b) : (u32)t / (u32)b;
      t -= (u64)v * b;
    }
    len += (int)S.occ[r] * ((int)T.vals[K.val_base + v].len - (int)K.klen);
    sv |= (u64)(1 + v) << (4 * r);
    c--;
  }
  sel = sv;
  return (u32)len;
}

// bytes [lo, hi) of the 16-B block at out offset X
__device__ __forceinline__ void m_store_part(uint8_t* out, u64 X, const uint4 x, u64 lo, u64 hi) {
  const u32 w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
  for (u32 b = 0; b < 16; b++)
    if (X + b >= lo && X + b < hi) out[X + b] = (uint8_t)(w[b >> 2] >> (8 * (b & 3)));
}

__device__ __forceinline__ void m_store16_nt(uint8_t* p, const uint4 x) {
  typedef u32 v4u __attribute__((ext_vector_type(4)));
  v4u y = {x.x, x.y, x.z, x.w};
  __builtin_nontemporal_store(y, (v4u*)p);
}

// Expand leaves [tb, te) of the positional word set up in S; the first one's bytes
// start at a.out + pos0.  64 leaves per round: lengths (formula) -> wave scan ->
// every token's entry OR-placed into the zeroed ring (S.buf) -> complete 16-B blocks
// streamed with dwordx4 stores (the item's first and last blocks byte-exact).
template <class SL>
__device__ void m_pos_expand(SL& S, const MT& T, const MInfo& I, const A5xModeLaunch& a, u64 tb, u64 te, u64 pos0,
                             u32 ntok, u32& err) {
  const u32 lane = m_lane();
  uint4* r4 = (uint4*)&S.buf[0];
  constexpr u32 RB = sizeof(S.buf) / 16;
  static_assert(SL::RING && sizeof(S.buf) >= 16 + 64 * A5X_M_CBUF + 32, "ring: one round of 64 candidates");
  const u32 ringa = fx6_addr(r4);
  for (u32 i = lane; i < RB; i += 64) r4[i] = make_uint4(0, 0, 0, 0);
  M_WAVE_SYNC();
  u64 B = pos0 & ~15ull, pos = pos0;
  const u64 lo = pos0;
  const uint4 nl = make_uint4(0x0Au, 0u, 0u, 1u << 24);
  const bool rev = a.mode == A5X_MODE_REVERSE;  // token selector: bit j of the position set
  for (u64 t0 = tb; t0 < te; t0 += 64) {
    const u64 t = t0 + lane;
    u64 sel = 0;
    u32 len = 0;
    if (t < te) {
      len = m_pos_sel(S, T, I, a.mode, t, sel) + 1;
      if (len > A5X_M_CBUF) { err |= M_ERR_CLEN; len = 0; }
    }
    const u32 incl = m_incl_scan(len);
    const u32 tot = (u32)__builtin_amdgcn_readlane((int)incl, 63);
    u32 P = ringa + (u32)(pos - B) + incl - len;
    if (len) {
      for (u32 k = 0; k < ntok; k++) {
        const u32 d = S.tok[k], pi = d >> 16;
        const u32 ix = (d & 0xFFFFu) + (pi ? (rev ? (u32)(sel >> (pi - 1)) & 1u : (u32)(sel >> (4 * (pi - 1))) & 15u) : 0u);
        fx7_put(S.ent[ix], P);
      }
      fx7_put(nl, P);
    }
    pos += tot;
    M_WAVE_SYNC();
    const u32 nb = (u32)((pos - B) >> 4);
    if (B + 16ull * nb > a.out_cap) { err |= M_ERR_GUARD; return; }
    for (u32 b = lane; b < nb; b += 64) {
      const uint4 x = r4[b];
      const u64 X = B + 16ull * b;
      if (X >= lo) m_store16_nt(a.out + X, x);
      else m_store_part(a.out, X, x, lo, X + 16);
      r4[b] = make_uint4(0, 0, 0, 0);
    }
    if (lane == 0 && nb) {
      const uint4 x = r4[nb];
      r4[nb] = make_uint4(0, 0, 0, 0);
      r4[0] = x;
    }
    B += 16ull * nb;
    M_WAVE_SYNC();
  }
  if (lane == 0 && pos > B) {
    if (pos > a.out_cap) err |= M_ERR_GUARD;
    else m_store_part(a.out, B, r4[0], lo > B ? lo : B, pos);
  }
  M_WAVE_SYNC();
}

// ---------------------------------------------------------------------------
// Piece engine (radix positional words: MInfo::radix and a token list).  The tokens
// are grouped left to right into pieces of <= 15 bytes with <= 3 selector sources (a
// -r position bit, a -s pattern digit) and <= MF_EMAX entries, each entry the bytes of
// its tokens for one combination of its sources -- the big pieces of the default engine
// (a5x_plan.h) for these engines: a candidate is a few entry reads and ORs instead of
// one per token.  A lane takes a run of MF_K consecutive leaves and advances the leaf's
// selector as an odometer: -r binary counting over the positions; -s packed 4-bit
// digits stored as digit + 16 - R, so that + 1 carries into the next pattern by itself
// (the fields that wrapped to 0 get their bias back).  A piece's entry is
// base + sum_s field_s * stride_s (the biases folded into base).
// ---------------------------------------------------------------------------

// concatenation of entry x at byte off of (lo, hi) (off + its length <= 15)
__device__ __forceinline__ void m_cat(u64& lo, u64& hi, u32& off, const uint4 x) {
  const u64 clo = (u64)x.x | ((u64)x.y << 32), chi = (u64)x.z | ((u64)(x.w & 0xFFFFFFu) << 32);
  const u32 sh = 8u * off;
  if (off == 0) {
    lo |= clo;
    hi |= chi;
  } else if (off < 8) {
    lo |= clo << sh;
    hi |= (clo >> (64u - sh)) | (chi << sh);
  } else {
    hi |= clo << (sh - 64u);
  }
  off += x.w >> 24;
}

// Pieces of the positional word set up in S (after m_pos_setup): descriptors in
// S.pdesc, multi-token pieces' entries at S.ent[MP_NE ..].  Returns the piece count;
// biasm = the -s field biases.  (The grouping loop is wave-uniform: every lane runs it.)
template <class SL>
__device__ u32 m_piece_setup_serial(SL& S, const MInfo& I, int mode, u32 ntok, u64& biasm) {
  const u32 lane = m_lane();
  const bool rev = mode == A5X_MODE_REVERSE;
  biasm = 0;
  if (!rev)
    for (u32 r = 0; r < I.n; r++) biasm |= (u64)(16u - S.rr[r]) << (4 * r);
  u32 np = 0, pe = 0, k = 0;
  while (k < ntok) {
    u32 k1 = k, ns = 0, E = 1, ml = 0;
    u32 s0 = 0, s1 = 0, s2 = 0, R0 = 1, R1 = 1, R2 = 1;
    while (k1 < ntok) {
      const u32 d = S.tok[k1], pi = d >> 16, eb = d & 0xFFFFu;
      const u32 R = pi ? (rev ? 2u : (u32)S.rr[pi - 1]) : 1u;
      u32 mlk = 0;
      for (u32 v = 0; v < R; v++) mlk = max(mlk, S.ent[eb + v].w >> 24);
      const bool known = pi && ((ns > 0 && s0 == pi) || (ns > 1 && s1 == pi) || (ns > 2 && s2 == pi));
      const bool add = pi && !known;
      const u32 E2 = add ? E * R : E, ns2 = ns + (add ? 1u : 0u);
      if (k1 > k && (ml + mlk > 15u || ns2 > 3u || E2 > MF_EMAX || pe + E2 > MF_NPE - 1u)) break;
      if (add) {
        if (ns == 0) { s0 = pi; R0 = R; }
        else if (ns == 1) { s1 = pi; R1 = R; }
        else { s2 = pi; R2 = R; }
      }
      ns = ns2;
      E = E2;
      ml += mlk;
      k1++;
    }
    u32 base;
    if (k1 == k + 1) {
      base = S.tok[k] & 0xFFFFu;  // one token: its own entries, indexed by its digit
    } else {
      base = SL::N_E + pe;
      for (u32 e = lane; e < E; e += 64) {
        const u32 d0 = e % R0, d1 = (e / R0) % R1, d2 = e / (R0 * R1);
        u64 lo = 0, hi = 0;
        u32 off = 0;
        for (u32 kk = k; kk < k1; kk++) {
          const u32 d = S.tok[kk], pi = d >> 16;
          const u32 dg = !pi ? 0u : pi == s0 ? d0 : pi == s1 ? d1 : d2;
          m_cat(lo, hi, off, S.ent[(d & 0xFFFFu) + dg]);
        }
        S.ent[base + e] = make_uint4((u32)lo, (u32)(lo >> 32), (u32)hi, ((u32)(hi >> 32) & 0xFFFFFFu) | (off << 24));
        S.elen[base + e] = (uint8_t)off;
      }
      pe += E;
    }
    if (lane == 0) {
      const u32 mk = rev ? 1u : 15u;
      auto sh = [&](u32 src) -> u32 { return src ? (rev ? src - 1u : 4u * (src - 1u)) : 0u; };
      const u32 st0 = ns > 0 ? 1u : 0u, st1 = ns > 1 ? R0 : 0u, st2 = ns > 2 ? R0 * R1 : 0u;
      int b = (int)base;
      if (!rev) b -= (int)((16u - R0) * st0 + (16u - R1) * st1 + (16u - R2) * st2);
      S.pdesc[np] = make_uint4((u32)b, sh(s0) | (sh(s1) << 8) | (sh(s2) << 16) | (mk << 24),
                               st0 | (st1 << 8) | (st2 << 16), ns | (fx8_slots(ml) << 8));
    }
    np++;
    k = k1;
  }
  if (lane == 0) {  // the empty entry (leaves past a run's end)
    S.ent[SL::ZE] = make_uint4(0, 0, 0, 0);
    S.elen[SL::ZE] = 0;
  }
  m_sync<SL>();
  return np;
}

// m_piece_setup_serial's pieces (the same grouping), built lane-parallel for words of
// <= 64 tokens: every token's choices and longest entry at once (lane = token), the
// greedy grouping as a scalar loop over those registers (readlane: no LDS round trip
// per step), descriptors lane = piece, entries lane = entry of any multi-token piece.
template <class SL>
__device__ u32 m_piece_setup(SL& S, const MInfo& I, int mode, u32 ntok, u64& biasm) {
  if (ntok > 64) return m_piece_setup_serial(S, I, mode, ntok, biasm);
  const u32 lane = m_lane();
  const bool rev = mode == A5X_MODE_REVERSE;
  {
    u64 bl = (!rev && lane < I.n) ? (u64)(16u - S.rr[lane]) << (4 * lane) : 0ull;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) bl |= (u64)__shfl_xor((long long)bl, d, 64);
    biasm = bl;
  }
  u32 tpi = 0, tR = 1, tml = 0, teb = 0;
  if (lane < ntok) {
    const u32 d = S.tok[lane];
    tpi = d >> 16;
    teb = d & 0xFFFFu;
    tR = tpi ? (rev ? 2u : (u32)S.rr[tpi - 1]) : 1u;
    for (u32 v = 0; v < tR; v++) tml = max(tml, S.ent[teb + v].w >> 24);
  }
  u32 np = 0, pe = 0, k = 0;
  u32 pk0 = 0, pk1 = 0, psrc = 0, pR = 0, pE = 0, pbase = 0, pns = 0, pml = 0;  // lane p: piece p
  while (k < ntok) {
    u32 k1 = k, ns = 0, E = 1, ml = 0;
    u32 s0 = 0, s1 = 0, s2 = 0, R0 = 1, R1 = 1, R2 = 1;
    while (k1 < ntok) {
      const u32 pi = (u32)__builtin_amdgcn_readlane((int)tpi, (int)k1);
      const u32 R = (u32)__builtin_amdgcn_readlane((int)tR, (int)k1);
      const u32 mlk = (u32)__builtin_amdgcn_readlane((int)tml, (int)k1);
      const bool known = pi && ((ns > 0 && s0 == pi) || (ns > 1 && s1 == pi) || (ns > 2 && s2 == pi));
      const bool add = pi && !known;
      const u32 E2 = add ? E * R : E, ns2 = ns + (add ? 1u : 0u);
      if (k1 > k && (ml + mlk > 15u || ns2 > 3u || E2 > MF_EMAX || pe + E2 > MF_NPE - 1u)) break;
      if (add) {
        if (ns == 0) { s0 = pi; R0 = R; }
        else if (ns == 1) { s1 = pi; R1 = R; }
        else { s2 = pi; R2 = R; }
      }
      ns = ns2;
      E = E2;
      ml += mlk;
      k1++;
    }
    const bool multi = k1 > k + 1;
    const u32 base = multi ? SL::N_E + pe : (u32)__builtin_amdgcn_readlane((int)teb, (int)k);
    if (lane == np) {
      pk0 = k; pk1 = k1; psrc = s0 | (s1 << 8) | (s2 << 16); pR = R0 | (R1 << 8) | (R2 << 16);
      pE = multi ? E : 0u; pbase = base; pns = ns; pml = ml;
    }
    if (multi) pe += E;
    np++;
    k = k1;
  }
  if (lane < np) {
    const u32 mk = rev ? 1u : 15u;
    const u32 s0 = psrc & 255u, s1 = (psrc >> 8) & 255u, s2 = psrc >> 16;
    const u32 R0 = pR & 255u, R1 = (pR >> 8) & 255u, R2 = pR >> 16;
    auto sh = [&](u32 src) -> u32 { return src ? (rev ? src - 1u : 4u * (src - 1u)) : 0u; };
    const u32 st0 = pns > 0 ? 1u : 0u, st1 = pns > 1 ? R0 : 0u, st2 = pns > 2 ? R0 * R1 : 0u;
    int b = (int)pbase;
    if (!rev) b -= (int)((16u - R0) * st0 + (16u - R1) * st1 + (16u - R2) * st2);
    S.pdesc[lane] = make_uint4((u32)b, sh(s0) | (sh(s1) << 8) | (sh(s2) << 16) | (mk << 24),
                               st0 | (st1 << 8) | (st2 << 16), pns | (fx8_slots(pml) << 8));
  }
  // the multi-token pieces' entries: lane = entry g of [0, pe)
  for (u32 g0 = 0; g0 < pe; g0 += 64) {
    const u32 g = g0 + lane;
    u32 p = 0;
    for (u32 q = 0; q < np; q++) {
      const u32 bq = (u32)__builtin_amdgcn_readlane((int)pbase, (int)q) - SL::N_E;
      const u32 eq = (u32)__builtin_amdgcn_readlane((int)pE, (int)q);
      p = (eq && g >= bq && g < bq + eq) ? q : p;
    }
    const u32 k0 = (u32)__shfl((int)pk0, (int)p), k1 = (u32)__shfl((int)pk1, (int)p);
    const u32 src = (u32)__shfl((int)psrc, (int)p), Rp = (u32)__shfl((int)pR, (int)p);
    const u32 e = g - ((u32)__shfl((int)pbase, (int)p) - SL::N_E);
    if (g < pe) {
      const u32 R0 = Rp & 255u, R1 = (Rp >> 8) & 255u;
      const u32 s0 = src & 255u, s1 = (src >> 8) & 255u;
      const u32 d0 = e % R0, d1 = (e / R0) % R1, d2 = e / (R0 * R1);
      u64 lo = 0, hi = 0;
      u32 off = 0;
      for (u32 kk = k0; kk < k1; kk++) {
        const u32 d = S.tok[kk], pi = d >> 16;
        const u32 dg = !pi ? 0u : pi == s0 ? d0 : pi == s1 ? d1 : d2;
        m_cat(lo, hi, off, S.ent[(d & 0xFFFFu) + dg]);
      }
      S.ent[SL::N_E + g] = make_uint4((u32)lo, (u32)(lo >> 32), (u32)hi, ((u32)(hi >> 32) & 0xFFFFFFu) | (off << 24));
      S.elen[SL::N_E + g] = (uint8_t)off;
    }
  }
  if (lane == 0) {  // the empty entry (leaves past a run's end)
    S.ent[SL::ZE] = make_uint4(0, 0, 0, 0);
    S.elen[SL::ZE] = 0;
  }
  m_sync<SL>();
  return np;
}

__device__ __forceinline__ u32 m_piece_ix(const uint4 pd, u64 sel) {
  const u32 mk = pd.y >> 24;  // (pd.w: sources | fx8 slots << 8)
  const u32 f0 = (u32)(sel >> (pd.y & 63u)) & mk, f1 = (u32)(sel >> ((pd.y >> 8) & 63u)) & mk,
            f2 = (u32)(sel >> ((pd.y >> 16) & 63u)) & mk;
  return pd.x + f0 * (pd.z & 255u) + f1 * ((pd.z >> 8) & 255u) + f2 * ((pd.z >> 16) & 255u);
}

// selector of leaf t (radix word): -r the position set t + cmin; -s the biased digits
template <class SL>
__device__ __forceinline__ u64 m_fast_sel(const SL& S, const MInfo& I, bool rev, u64 t) {
  if (rev) return t + I.cmin;
  u32 x = (u32)t + I.cmin;  // < 2^27 (MInfo::radix)
  u64 sel = 0;
  for (u32 r = 0; r < I.n; r++) {
    const u32 mg = S.rmag[r], R = S.rr[r];
    const u32 q = __umulhi(x, mg) + (mg ? 0u : x);
    sel |= (u64)(x - q * R + 16u - R) << (4 * r);
    x = q;
  }
  return sel;
}

__device__ __forceinline__ u64 m_fast_step(u64 sel, bool rev, u64 biasm) {
  const u64 y = sel + 1;
  if (rev) return y;
  const u32 nf = (u32)__builtin_ctzll(y) >> 2;  // fields below the first that did not wrap
  return y | (biasm & (nf >= 16 ? ~0ull : (1ull << (4 * nf)) - 1ull));
}

__device__ __forceinline__ void m_digest_probe(const A5xModeLaunch& a, const uint8_t* base, u32 off, u32 len, bool on,
                                               u64 w, u64 t);

// Fused MD5, one leaf per 64-lane slot of SLOT bytes (SLOT - 1 >= the leaf, <= 55): the leaf
// is OR-placed at ring + SLOT lane with a 0x80 pad byte after it (the slot is zero beyond),
// so its MD5 message block is the slot itself plus the bit length -- no prefix scan, no
// per-word masks (k_expand_fast's fxd_round does the same for FAST words).  Reads the
// lane's slot back, zeroes it for the next round and probes the target set.
template <u32 SLOT>
__device__ __forceinline__ void m_slot_md5_probe(const A5xModeLaunch& a, u32 slot, u32 len, bool on, u64 w, u64 t) {
  static_assert(SLOT % 16 == 0 && SLOT <= 64, "one MD5 block per slot");
  if (on) fx7_or((slot + len) & ~3u, 0x80u << (8u * ((slot + len) & 3u)));
  M_WAVE_SYNC();
  u32 M[16];
#pragma unroll
  for (u32 q = 0; q < 4; q++) {
    uint4 v = make_uint4(0, 0, 0, 0);
    if (16u * q < SLOT) {
      v = fx6_ld16(slot + 16u * q);
      fx6_st16(slot + 16u * q, make_uint4(0, 0, 0, 0));
    }
    M[4 * q] = v.x; M[4 * q + 1] = v.y; M[4 * q + 2] = v.z; M[4 * q + 3] = v.w;
  }
  M[14] = on ? len << 3 : 0u;
  M[15] = 0u;
  u32 d[4];
  if (md_block_probe<true>(M, on, a.dg_bitmap, a.dg_bm_mask, a.dg_table, a.dg_tmask, a.dg_has_zero != 0, d)) {
    const u32 h = atomicAdd(a.dg_nhits, 1u);
    if (h < a.dg_hit_cap) {
      A5xHitRaw r;
      r.blk = w;
      r.idx = t;
      r.d[0] = d[0]; r.d[1] = d[1]; r.d[2] = d[2]; r.d[3] = d[3];
      a.dg_hits[h] = r;
    }
  }
  M_WAVE_SYNC();
}

// The piece engine's fused MD5 on the slot layout: rounds of 64 leaves of [tb, te), one
// per lane at ring + 48 lane, while every leaf of the round fits a 48-byte slot.  Returns
// the first leaf it did not hash (a round with a longer leaf: m_fast_expand's run layout
// takes the rest).  The ring is zero before and after.
template <class SL>
__device__ u64 m_fast_digest_slots(SL& S, const MInfo& I, const A5xModeLaunch& a, u64 tb, u64 te, u32 np, u64 w) {
  constexpr u32 SLOT = 48;
  static_assert(sizeof(S.buf) >= 64 * SLOT + 32, "ring: 64 slots");
  const u32 lane = m_lane();
  uint4* r4 = (uint4*)&S.buf[0];
  constexpr u32 RB = sizeof(S.buf) / 16;
  const u32 ringa = fx6_addr(r4);
  for (u32 i = lane; i < RB; i += 64) r4[i] = make_uint4(0, 0, 0, 0);
  M_WAVE_SYNC();
  const bool rev = a.mode == A5X_MODE_REVERSE;
  const u32 Lc = I.L + 1;
  for (u64 t0 = tb; t0 < te; t0 += 64) {
    const u64 t = t0 + lane;
    const bool on = t < te;
    const u64 sel = on ? m_fast_sel(S, I, rev, t) : 0ull;
    u32 len = on && rev ? Lc - 1u : 0u;
    if (!rev) {
      for (u32 p = 0; p < np; p++) len += S.elen[on ? m_piece_ix(S.pdesc[p], sel) : SL::ZE];
    }
    if (__builtin_amdgcn_ballot_w64(on && len > SLOT - 1u)) return t0;  // (uniform)
    u32 P1 = ringa + SLOT * lane - 1u;
    for (u32 p = 0; p < np; p++) {
      const uint4 pd = S.pdesc[p];
      const u32 nsl = (u32)__builtin_amdgcn_readfirstlane((int)(pd.w >> 8));
      fx8_put(S.ent[on ? m_piece_ix(pd, sel) : SL::ZE], P1, nsl);
    }
    m_slot_md5_probe<SLOT>(a, ringa + SLOT * lane, len, on, w, t);
  }
  return te;
}

// Expand leaves [tb, te) of the radix word set up in S (pieces from m_piece_setup);
// the first one's bytes start at a.out + pos0.  A round: 64 runs of MF_K leaves,
// lengths -> wave scan -> the runs that fit the ring OR-place their pieces (piece-major:
// one descriptor read per piece per run) -> complete 16-B blocks streamed out.
// DIG (fused digest, op 2): the leaves are placed without their newline, every lane
// hashes its run's leaves where they lie in the ring and probes the target set (hits
// as (word w, leaf)), and the round's bytes are zeroed instead of streamed.
template <class SL, bool DIG = false>
__device__ void m_fast_expand(SL& S, const MInfo& I, const A5xModeLaunch& a, u64 tb, u64 te, u64 pos0, u32 np,
                              u64 biasm, u32& err, u64 w = 0) {
  if constexpr (DIG) {
    if (a.dg_algo == A5X_ALGO_MD5) {
      tb = m_fast_digest_slots(S, I, a, tb, te, np, w);
      if (tb >= te) return;
    }
  }
  const u32 lane = m_lane();
  uint4* r4 = (uint4*)&S.buf[0];
  constexpr u32 RB = sizeof(S.buf) / 16;
  constexpr u32 CAP = (RB - 3) * 16;  // (the ORs' zero overhang past the round's bytes)
  static_assert(CAP >= MF_K * A5X_M_CBUF + 16, "ring: one run of the longest candidates");
  const u32 ringa = fx6_addr(r4);
  for (u32 i = lane; i < RB; i += 64) r4[i] = make_uint4(0, 0, 0, 0);
  M_WAVE_SYNC();
  const bool rev = a.mode == A5X_MODE_REVERSE;
  const u32 Lc = I.L + 1;
  u64 B = pos0 & ~15ull, pos = pos0;
  const u64 lo = pos0;
  const uint4 nl = make_uint4(0x0Au, 0u, 0u, 1u << 24);
  const u64 nruns = (te - tb + MF_K - 1) / MF_K;
  for (u64 rr = 0; rr < nruns;) {
    const u64 run = rr + lane;
    const u64 t = tb + run * MF_K;
    const u32 nc = run < nruns ? (u32)min((u64)MF_K, te - t) : 0u;
    u64 sel[MF_K];
    sel[0] = nc ? m_fast_sel(S, I, rev, t) : 0ull;
#pragma unroll
    for (int c = 1; c < MF_K; c++) sel[c] = m_fast_step(sel[c - 1], rev, biasm);
    u32 clen[MF_K], len = 0;
#pragma unroll
    for (int c = 0; c < MF_K; c++) clen[c] = (u32)c < nc ? (rev ? Lc : 1u) - (DIG ? 1u : 0u) : 0u;
    if (!rev) {  // (leaves past the run read the empty entry: no per-leaf branches)
      for (u32 p = 0; p < np; p++) {
        const uint4 pd = S.pdesc[p];
#pragma unroll
        for (int c = 0; c < MF_K; c++) clen[c] += S.elen[(u32)c < nc ? m_piece_ix(pd, sel[c]) : SL::ZE];
      }
    }
#pragma unroll
    for (int c = 0; c < MF_K; c++) len += clen[c];
    const u32 incl = m_incl_scan(len);
    const u32 used = (u32)(pos - B);
    const bool fit = nc > 0 && used + incl <= CAP;
    const u32 nact = (u32)__popcll(__ballot(fit));
    const u32 tot = nact ? (u32)__builtin_amdgcn_readlane((int)incl, (int)nact - 1) : 0u;
    if (fit) {
      // fx8_put: the piece's dword count from its longest entry (uniform, scalar branches)
      u32 P1[MF_K];
      P1[0] = ringa + used + incl - len - 1u;
#pragma unroll
      for (int c = 1; c < MF_K; c++) P1[c] = P1[c - 1] + clen[c - 1];
      for (u32 p = 0; p < np; p++) {
        const uint4 pd = S.pdesc[p];
        const u32 nsl = (u32)__builtin_amdgcn_readfirstlane((int)(pd.w >> 8));
#pragma unroll
        for (int c = 0; c < MF_K; c++) fx8_put(S.ent[(u32)c < nc ? m_piece_ix(pd, sel[c]) : SL::ZE], P1[c], nsl);
      }
      if (!DIG) {
#pragma unroll
        for (int c = 0; c < MF_K; c++) fx8_put((u32)c < nc ? nl : make_uint4(0, 0, 0, 0), P1[c], 2u);
      }
    }
    pos += tot;
    rr += nact;
    M_WAVE_SYNC();
    if constexpr (DIG) {  // hash the round's leaves in the ring, then zero its bytes
      u32 off = used + incl - len;
#pragma unroll
      for (int c = 0; c < MF_K; c++) {
        m_digest_probe(a, (const uint8_t*)r4, off, clen[c], fit && (u32)c < nc, w, t + c);
        off += clen[c];
      }
      M_WAVE_SYNC();
      for (u32 b = lane; b < (tot + 31u) / 16u && b < RB; b += 64) r4[b] = make_uint4(0, 0, 0, 0);
      pos = B = 0;
      M_WAVE_SYNC();
      continue;
    }
    const u32 nb = (u32)((pos - B) >> 4);
    if (B + 16ull * nb > a.out_cap) { err |= M_ERR_GUARD; return; }
    for (u32 b = lane; b < nb; b += 64) {
      const uint4 x = r4[b];
      const u64 X = B + 16ull * b;
      if (X >= lo) m_store16_nt(a.out + X, x);
      else m_store_part(a.out, X, x, lo, X + 16);
      r4[b] = make_uint4(0, 0, 0, 0);
    }
    if (lane == 0 && nb) {
      const uint4 x = r4[nb];
      r4[nb] = make_uint4(0, 0, 0, 0);
      r4[0] = x;
    }
    B += 16ull * nb;
    M_WAVE_SYNC();
  }
  if (lane == 0 && pos > B) {
    if (pos > a.out_cap) err |= M_ERR_GUARD;
    else m_store_part(a.out, B, r4[0], lo > B ? lo : B, pos);
  }
  M_WAVE_SYNC();
}

// Hash candidate t of word w (len bytes at base + off: LDS, or a pass-G slot in HBM,
// readable 8 bytes past the end) and record a hit.  Wave-collective (NTLM's block loop):
// every lane calls it, on = whether the lane holds a candidate.
__device__ __forceinline__ void m_digest_probe(const A5xModeLaunch& a, const uint8_t* base, u32 off, u32 len, bool on,
                                               u64 w, u64 t) {
  u32 d[4];
  if (a.dg_algo == A5X_ALGO_MD5) md_lds<true>(base, off, on ? len : 0u, d);
  else ntlm_lds(base, off, on ? len : 0u, d);
  if (on && md_probe(a.dg_bitmap, a.dg_bm_mask, a.dg_table, a.dg_tmask, a.dg_has_zero != 0, d)) {
    const u32 h = atomicAdd(a.dg_nhits, 1u);
    if (h < a.dg_hit_cap) {
      A5xHitRaw r;
      r.blk = w;
      r.idx = t;
      r.d[0] = d[0]; r.d[1] = d[1]; r.d[2] = d[2]; r.d[3] = d[3];
      a.dg_hits[h] = r;
    }
  }
}

// Fused digest of leaves [tb, te) of the positional word w set up in S: 64 leaves per
// round placed into the zeroed ring exactly as m_pos_expand places them (without the
// newline), hashed there by their lanes, then the round's bytes are zeroed again.
template <class SL>
__device__ void m_pos_digest(SL& S, const MT& T, const MInfo& I, const A5xModeLaunch& a, u64 w, u64 tb, u64 te,
                             u32 ntok, u32& err) {
  const u32 lane = m_lane();
  uint4* r4 = (uint4*)&S.buf[0];
  constexpr u32 RB = sizeof(S.buf) / 16;
  static_assert(SL::RING && sizeof(S.buf) >= 16 + 64 * A5X_M_CBUF + 32, "ring: one round of 64 candidates");
  const u32 ringa = fx6_addr(r4);
  for (u32 i = lane; i < RB; i += 64) r4[i] = make_uint4(0, 0, 0, 0);
  M_WAVE_SYNC();
  const bool rev = a.mode == A5X_MODE_REVERSE;
  for (u64 t0 = tb; t0 < te; t0 += 64) {
    const u64 t = t0 + lane;
    u64 sel = 0;
    u32 len = 0;
    if (t < te) {
      len = m_pos_sel(S, T, I, a.mode, t, sel);
      if (len + 1 > A5X_M_CBUF) { err |= M_ERR_CLEN; len = 0; }
    }
    if (a.dg_algo == A5X_ALGO_MD5 && !__builtin_amdgcn_ballot_w64(t < te && len > 55u)) {
      // every leaf fits one MD5 block: one 64-byte slot per lane (m_slot_md5_probe)
      u32 P = ringa + 64u * lane;
      if (t < te && len) {
        for (u32 k = 0; k < ntok; k++) {
          const u32 d = S.tok[k], pi = d >> 16;
          const u32 ix = (d & 0xFFFFu) + (pi ? (rev ? (u32)(sel >> (pi - 1)) & 1u : (u32)(sel >> (4 * (pi - 1))) & 15u) : 0u);
          fx7_put(S.ent[ix], P);
        }
      }
      m_slot_md5_probe<64>(a, ringa + 64u * lane, len, t < te, w, t);
      continue;
    }
    const u32 incl = m_incl_scan(len);
    const u32 tot = (u32)__builtin_amdgcn_readlane((int)incl, 63);
    const u32 o = incl - len;
    u32 P = ringa + o;
    if (t < te && len) {
      for (u32 k = 0; k < ntok; k++) {
        const u32 d = S.tok[k], pi = d >> 16;
        const u32 ix = (d & 0xFFFFu) + (pi ? (rev ? (u32)(sel >> (pi - 1)) & 1u : (u32)(sel >> (4 * (pi - 1))) & 15u) : 0u);
        fx7_put(S.ent[ix], P);
      }
    }
    M_WAVE_SYNC();
    m_digest_probe(a, (const uint8_t*)r4, o, len, t < te, w, t);
    M_WAVE_SYNC();
    for (u32 b = lane; b < (tot + 31u) / 16u && b < RB; b += 64) r4[b] = make_uint4(0, 0, 0, 0);
    M_WAVE_SYNC();
  }
}

__device__ __forceinline__ void m_err(u32* e, u32 bits) {
  if (bits && m_lane() == 0) atomicOr(e, bits);
}

extern __shared__ __attribute__((aligned(16))) uint8_t m_dyn[];

// per-word count, segments and flags of a set-up word
template <class SL>
__device__ __forceinline__ void m_count_word(SL& S, const MT& T, const A5xModeLaunch& a, u64 w) {
  if (!SL::G && a.rfast && (a.flags[w] & A5X_WF_FAST)) {  // counted by the -r FAST probe
    if (m_lane() == 0) a.nseg[w] = (a.count[w] + a.SEG - 1) / a.SEG;
    return;
  }
  const MInfo I = m_setup(S, T, a, w, false);
  const bool gw = I.bad == M_ERR_GWORD;  // (LDS pass only) routed to mode pass G
  if (m_lane() == 0) {
    const u64 cnt = I.bad ? 0 : I.count;
    a.count[w] = cnt;
    a.nseg[w] = (cnt + a.SEG - 1) / a.SEG;
    a.flags[w] = gw ? A5X_WF_GLOB : I.bad == M_ERR_OVF ? A5X_WF_ERR_OVF : (I.bad ? A5X_WF_ERR_BIG : 0u);
    if (SL::G) a.flags[w] |= A5X_WF_GLOB;
    if (gw) {
      const u32 k = atomicAdd(a.glob_n, 1u);
      a.glob_list[k] = (u32)w;
    }
  }
  if constexpr (!SL::G) {
    // single-item positional words: their output bytes in closed form here, so the length
    // pass takes them without another setup (wbytes = ~0: the length pass computes them)
    u64 wb = ~0ull;
    if (!I.bad && I.count > 0 && I.count <= a.SEG && a.mode != A5X_MODE_DEFAULT) {
      const u32 ntok = m_pos_setup(S, T, I, a.mode);
      if (ntok && a.mode == A5X_MODE_REVERSE) wb = I.count * (u64)(I.L + 1);
      else if (ntok && S.radix) wb = m_pos_prefix(S, I, I.count) - m_pos_prefix(S, I, 0);
      if (wb != ~0ull && I.radix && !MF_OFF && ntok <= MF_TCAP)
        wb |= S.nent <= MF_NE ? M_WB_FAST : S.nent <= MF_NE2 ? M_WB_FAST2 : 0ull;
    }
    if (m_lane() == 0) a.wbytes[w] = wb;
  }
  m_err(a.err, gw ? 0u : I.bad);
}

// one wave per word (or per word of cl_list): count, segments, per-word error flags
__global__ void __launch_bounds__(64) k_mode_count(A5xModeLaunch a) {
  const u64 n = a.cl_list ? (u64)*a.cl_n : a.nw;
  if (blockIdx.x >= n) return;  // (before staging the table)
  MLdsC& S = *(MLdsC*)m_dyn;
  const MT T = m_table(m_dyn + sizeof(MLdsC), a.mtab, a.mtab_bytes);
  for (u64 i = blockIdx.x; i < n; i += gridDim.x) m_count_word(S, T, a, a.cl_list ? (u64)a.cl_list[i] : i);
}

// Lane-per-word keyspace of -s / -s -r (processWordSubstituteAll(Reverse), main.go:
// 308-365, 369-440) for the words the wave kernel would find radix and positional:
// every pattern present passes the static per-key checks of compile_mtable (A5xMKey.pad:
// one codepoint, values of <= 15 valid UTF-8 bytes containing no key), <= MCT_PMAX
// patterns, no size-window cut (min <= 1, max >= #patterns).  Then, with R_p = 1 +
// (values of p) and P = prod R_p (< 2^27):  count = P - max(min, 0) and, each value of p
// chosen in P / R_p leaves, bytes = count (L + 1) + sum_p occ_p (P / R_p) sum_v (|v| - |p|)
// -- k_mode_count's results (m_setup + m_pos_setup + m_pos_prefix) for these words
// without the wave's per-word setup.  Every other word goes to cl_list.
#define MCT_SLOT 64  // per-lane word slot in LDS: words of <= MCT_SLOT - 8 bytes
#define MCT_PMAX 16  // patterns per word (the positional engine's MP_PMAX)
__global__ void __launch_bounds__(256) k_mode_count_thread(A5xModeLaunch a) {
  const MT T = m_table(m_dyn, a.mtab, a.mtab_bytes);
  const u32 tb = (a.mtab_bytes + 15u) & ~15u;
  uint8_t* ws = m_dyn + tb + threadIdx.x * MCT_SLOT;
  u32* pl = (u32*)(m_dyn + tb + blockDim.x * MCT_SLOT) + threadIdx.x;  // pattern j at pl[j * 256]
  const bool sub = a.mode == A5X_MODE_SUBALL;
  const u32 okbit = sub ? 1u : 2u, dsh = sub ? 8u : 20u;
  const u32 cmin = a.mn > 0 ? (u32)a.mn : 0u;
  const u64 stride = (u64)gridDim.x * blockDim.x;
  const u64 nin = a.in_list ? (u64)*a.in_n : a.nw;  // (in_list: the words the FAST probe left)
  const u64 nw_r = (nin + blockDim.x - 1) / blockDim.x * blockDim.x;  // every lane runs every pass
  for (u64 x = (u64)blockIdx.x * blockDim.x + threadIdx.x; x < nw_r; x += stride) {
    const bool valid = x < nin;
    const u64 w = !valid ? 0 : a.in_list ? (u64)a.in_list[x] : x;
    u64 w0 = 0, L64 = 0;
    if (valid) { w0 = a.woff[w]; L64 = a.woff[w + 1] - w0; }
    bool dfr = !valid || L64 == 0 || L64 + 8 > MCT_SLOT || a.mx < 0 || cmin > 1;
    const u32 L = dfr ? 0u : (u32)L64;
    for (u32 q = 0; q < MCT_SLOT / 4; q++) {
      u32 v = 0;
      for (u32 b = 0; b < 4; b++)
        if (4 * q + b < L) v |= (u32)a.words[w0 + 4 * q + b] << (8 * b);
      ((u32*)ws)[q] = v;
    }
    u32 n = 0, nlit = 0, lend = 0, nocc = 0;
    for (u32 q = 0; q < L && !dfr; q++) {
      const u32 b = ws[q], w4 = m_lds4(ws, q);
      for (u32 k = T.bucket[b]; k < T.bucket[b + 1] && !dfr; k++) {
        const A5xMKey K = T.keys[k];
        if (q + K.klen > L) continue;
        bool m;
        if (K.klen <= 4) {
          const u32 mask = K.klen == 4 ? ~0u : (1u << (8u * K.klen)) - 1u;
          m = ((w4 ^ m_lds4(T.blob, K.key_off)) & mask) == 0;
        } else {
          m = true;
          for (u32 i = 0; m && i < K.klen; i++) m = ws[q + i] == T.blob[K.key_off + i];
        }
        if (!m) continue;
        if (!(K.pad & okbit)) { dfr = true; break; }  // (not one codepoint: never positional)
        u32 j = 0;
        while (j < n && (pl[j * 256] & 0xFFFFu) != k) j++;
        if (j == n) {
          if (n == MCT_PMAX) { dfr = true; break; }
          pl[n * 256] = k | (1u << 16);
          n++;
        } else {
          pl[j * 256] += 1u << 16;
        }
        nocc++;
        nlit += (q - lend + 14u) / 15u;  // the literal run before this occurrence, in <= 15-byte chunks
        lend = q + K.klen;               // (codepoint keys in a word never overlap)
      }
    }
    nlit += (L - lend + 14u) / 15u;
    if (n == 0 || (u32)a.mx < n) dfr = true;  // (no pattern, or a size-window cut: the DP)
    u64 P = 1;
    u32 npe = 0;
    for (u32 j = 0; j < n && !dfr; j++) {
      const A5xMKey K = T.keys[pl[j * 256] & 0xFFFFu];
      const u32 R = 1u + (sub ? (u32)K.nvals : (K.nvals ? 1u : 0u));
      P *= R;
      npe += R;
      if (P >= (1ull << 27)) dfr = true;
    }
    u64 count = 0, wb = ~0ull;
    if (!dfr) {
      count = P - cmin;
      i64 extra = 0;
      for (u32 j = 0; j < n; j++) {
        const u32 e = pl[j * 256];
        const A5xMKey K = T.keys[e & 0xFFFFu];
        const u32 R = 1u + (sub ? (u32)K.nvals : (K.nvals ? 1u : 0u));
        const int d = (int)((K.pad >> dsh) & 0xFFFu) - 2048;
        extra += (i64)(e >> 16) * (i64)(P / R) * d;
      }
      const u64 bytes = (u64)((i64)(count * (u64)(L + 1)) + extra);
      // m_pos_setup's table limits (entries of the patterns, then the literal chunks)
      const bool pos = L <= A5X_M_LMAX && npe <= MP_NE && npe + nlit <= MP_NE;
      if (pos && count > 0 && count <= a.SEG)
        wb = bytes | (MF_OFF || nocc + nlit > MF_TCAP ? 0ull
                      : npe + nlit <= MF_NE ? M_WB_FAST : npe + nlit <= MF_NE2 ? M_WB_FAST2 : 0ull);
      a.count[w] = count;
      a.nseg[w] = (count + a.SEG - 1) / a.SEG;
      a.flags[w] = 0;
      a.wbytes[w] = wb;
    }
    const u64 dm = __ballot(dfr && valid);
    if (dm) {
      const u32 lane = m_lane(), leader = (u32)__builtin_ctzll(dm);
      u32 base = 0;
      if (lane == leader) base = atomicAdd(a.cl_n, (u32)__popcll(dm));
      base = (u32)__shfl((int)base, (int)leader);
      if (dfr && valid) a.cl_list[base + (u32)__popcll(dm & ((1ull << lane) - 1ull))] = (u32)w;
    }
  }
}

// mode pass G: one wave per HBM scratch slot over the listed words
__device__ __forceinline__ MLdsG& m_gslot(const A5xModeLaunch& a) {
  return *(MLdsG*)(a.gscr + (u64)blockIdx.x * ((sizeof(MLdsG) + 255) & ~(size_t)255));
}
__global__ void __launch_bounds__(64) k_mode_count_g(A5xModeLaunch a) {
  MLdsG& S = m_gslot(a);
  const MT T = m_table(m_dyn, a.mtab, a.mtab_bytes);
  const u32 ng = *a.glob_n;
  for (u32 i = blockIdx.x; i < ng; i += gridDim.x) m_count_word(S, T, a, a.glob_list[i]);
}

// Run the candidates [t0, t0 + nc) of the set-up word: op 0 = sum of (len+1),
// op 1 = write them at out[base + prefix - out_base] when their global index
// (g0 + t) is inside [cand_begin, cand_end).
template <class SL>
__device__ u64 m_run(SL& S, const MT& T, const MInfo& I, const A5xModeLaunch& a, u64 t0, u32 nc, int op,
                     u64 g0, u64 base, u32& err, u32 ntok = 0, u64 cw0 = 0) {
  const u32 lane = m_lane();
  u64 run = 0;
  for (u32 k0 = 0; k0 < nc; k0 += 64) {
    const u32 k = k0 + lane;
    const bool v = k < nc;
    const uint8_t* p = nullptr;
    u32 len = 0;
    if constexpr (!SL::G) {
      if (v && ntok && op == 0) {  // positional word: the length formula
        u64 sel;
        len = m_pos_sel(S, T, I, a.mode, t0 + k, sel) + 1;
        if (len > A5X_M_CBUF) { err |= M_ERR_CLEN; len = 0; }
      }
    }
    if (v && !(ntok && op == 0)) {
      if (op == 0 && a.mode == A5X_MODE_REVERSE) {
        len = m_rlen(S, T, I, m_rsel(S, I, t0 + k, err)) + 1;
      } else {
        if constexpr (SL::BUILDER) len = m_build(S, T, I, a.mode, t0 + k, &p, err) + 1;
        else err |= M_ERR_STATE;  // (item routed to the wrong layout)
      }
    }
    if (op == 2) {  // fused digest: the candidate where the builder left it (len - 1 bytes)
      const uint8_t* base = p ? p : S.word;
      const u64 g = cw0 + t0 + k;  // (op 2: g0 is the word; hashed only inside [cand_begin, cand_end))
      m_digest_probe(a, base, 0, len ? len - 1 : 0u, v && len > 0 && g >= a.cand_begin && g < a.cand_end, g0, t0 + k);
      continue;
    }
    const u32 incl = m_incl_scan(len);
    const u32 tot = (u32)__builtin_amdgcn_readlane((int)incl, 63);
    if (op == 1 && v) {
      const u64 g = g0 + t0 + k;
      if (g >= a.cand_begin && g < a.cand_end) {
        const u64 pos = base + run + (incl - len) - a.out_base;
        if (pos + len > a.out_cap) {
          err |= M_ERR_GUARD;
        } else {
          uint8_t* o = a.out + pos;
          for (u32 i = 0; i + 1 < len; i++) o[i] = p[i];
          o[len - 1] = '\n';
        }
      }
    }
    run += tot;
  }
  return run;
}

// item i (word, SEG-candidate segment): op 0 = seg_bytes, op 1 = expand.  The LDS
// items run in two layouts, routed by item_fl (written by the op-0 closed-form pass):
//   MLdsC / MLdsR (small: more waves per CU): op 0 of every item -- closed-form or
//     formula lengths of positional words, -r lengths; op 1 of positional items (ring);
//   MLds (byte builder): op 0 of non-positional -s / -s -r items, op 1 of every
//     non-positional item.
constexpr uint8_t MI_POS = 1;       // positional: lengths done, ring expansion
constexpr uint8_t MI_BUILD = 2;     // byte builder for the expansion, lengths done
constexpr uint8_t MI_BUILD_LEN = 3; // byte builder for the lengths too
constexpr uint8_t MI_FAST = 4;      // positional radix word: lengths done, piece engine
constexpr uint8_t MI_FAST2 = 6;     // ... in the piece layout with more token entries (MLdsF2)
constexpr uint8_t MI_SKIP = 5;      // -r FAST word (A5xModeLaunch::rfast): k_expand_fast writes it
template <class SL>
__device__ void m_item(SL& S, const MT& T, const A5xModeLaunch& a, u64 i, int op, const MPre* pre = nullptr) {
  const u64 w = a.item_w[i];
  const u64 cw0 = pre ? pre->c0 : a.cand_off[w], cnt = (pre ? pre->c1 : a.cand_off[w + 1]) - cw0;
  const u64 t0 = (i - (pre ? pre->s0 : a.seg_off[w])) * a.SEG;
  if (t0 >= cnt) { m_err(a.err, M_ERR_STATE); return; }
  const u32 nc = (u32)min(a.SEG, cnt - t0);
  const MInfo I = m_setup(S, T, a, w, true, pre);
  if (I.bad || I.count != cnt) { m_err(a.err, I.bad ? I.bad : M_ERR_STATE); return; }
  u32 err = 0, ntok = 0;
  if constexpr (SL::FAST) {  // op 1 / op 2 (fused digest) of MI_FAST / MI_FAST2 items
    ntok = op != 0 ? ((MF_ABL & 4) ? 1u : m_pos_setup(S, T, I, a.mode, false)) : 0u;
    if (!ntok) {
      err |= M_ERR_STATE;
    } else {
      u64 biasm = 0;
      const u32 np = (MF_ABL & 2) ? 0u : m_piece_setup(S, I, a.mode, ntok, biasm);
      if (op == 2) {  // (the item's candidates inside [cand_begin, cand_end))
        const u64 rb = a.cand_begin > cw0 ? a.cand_begin - cw0 : 0;
        const u64 re = a.cand_end - cw0 < t0 + nc ? a.cand_end - cw0 : t0 + nc;
        const u64 tb = rb > t0 ? rb : t0;
        if (a.cand_end > cw0 && tb < re) m_fast_expand<SL, true>(S, I, a, tb, re, 0, np, biasm, err, w);
        m_err(a.err, m_wave_or(err));
        return;
      }
      const u64 rb = a.cand_begin > cw0 ? a.cand_begin - cw0 : 0;
      const u64 re = a.cand_end - cw0 < t0 + nc ? a.cand_end - cw0 : t0 + nc;  // (cand_end > cw0 here)
      const u64 tb = rb > t0 ? rb : t0;
      if (a.cand_end > cw0 && tb < re && !(MF_ABL & 1))
        m_fast_expand(S, I, a, tb, re, tb == t0 ? a.seg_boff[i] - a.out_base : 0, np, biasm, err);
    }
    m_err(a.err, m_wave_or(err));
    return;
  }
  if constexpr (!SL::G && !SL::BUILDER) {
    ntok = a.mode != A5X_MODE_DEFAULT ? m_pos_setup(S, T, I, a.mode) : 0u;
    if (op == 2) {  // fused digest: positional items here, the others to the byte builder
      if constexpr (SL::RING) {
        const u64 rb = a.cand_begin > cw0 ? a.cand_begin - cw0 : 0;  // (inside [cand_begin, cand_end))
        const u64 re = a.cand_end - cw0 < t0 + nc ? a.cand_end - cw0 : t0 + nc;
        const u64 tb = rb > t0 ? rb : t0;
        if (ntok && a.cand_end > cw0 && tb < re) m_pos_digest(S, T, I, a, w, tb, re, ntok, err);
        if (m_lane() == 0) a.item_fl[i] = ntok ? MI_POS : MI_BUILD;
      }
      m_err(a.err, m_wave_or(err));
      return;
    }
    if (op == 1) {
      if constexpr (SL::RING) {
        // the leaves of this item inside [cand_begin, cand_end); the first one's bytes start
        // at seg_boff[i] (or at out_base itself when the range starts inside the item)
        const u64 rb = a.cand_begin > cw0 ? a.cand_begin - cw0 : 0;
        const u64 re = a.cand_end - cw0 < t0 + nc ? a.cand_end - cw0 : t0 + nc;  // (cand_end > cw0 here)
        const u64 tb = rb > t0 ? rb : t0;
        if (!ntok) err |= M_ERR_STATE;
        else if (a.cand_end > cw0 && tb < re)
          m_pos_expand(S, T, I, a, tb, re, tb == t0 ? a.seg_boff[i] - a.out_base : 0, ntok, err);
      }
      m_err(a.err, m_wave_or(err));
      return;
    }
    if (m_lane() == 0)
      a.item_fl[i] = ntok ? (I.radix && !MF_OFF && ntok <= MF_TCAP && S.nent <= MF_NE2
                                 ? (S.nent <= MF_NE ? MI_FAST : MI_FAST2) : MI_POS)
                          : a.mode == A5X_MODE_REVERSE ? MI_BUILD : MI_BUILD_LEN;
    if (!ntok && a.mode != A5X_MODE_REVERSE) return;  // lengths need the byte builder
    if (ntok && S.radix) {  // op 0, radix mode: closed form, no candidate is visited
      const u64 run = m_pos_prefix(S, I, t0 + nc) - m_pos_prefix(S, I, t0);
      if (m_lane() == 0) a.seg_bytes[i] = run;
      return;
    }
  }
  if constexpr (!SL::G && SL::BUILDER)
    if (op == 0 && m_lane() == 0) a.item_fl[i] = MI_BUILD;
  const u64 base = op == 1 ? a.seg_boff[i] : 0;
  // (op 2: m_run's g0 carries the word index for the hit records)
  const u64 run = m_run(S, T, I, a, t0, nc, op, op == 2 ? w : cw0, base, err, ntok, cw0);
  if (op == 0 && m_lane() == 0) a.seg_bytes[i] = run;
  m_err(a.err, m_wave_or(err));
}

// one wave per item of layout SL (route: which item_fl values it takes; 0 = all); the
// items of pass-G words are left to k_mode_items_g
template <class SL>
__device__ __forceinline__ void m_items(const A5xModeLaunch& a, int op, uint8_t route) {
  SL& S = *(SL*)m_dyn;
  const MT T = m_table(m_dyn + sizeof(SL), a.mtab, a.mtab_bytes);
  // 64 items per step, filtered lane-parallel (pass-G words, -r FAST words, other routes,
  // closed-form sizes); the wave then runs the items that need it one after the other
  const u32 lane = m_lane();
  for (u64 b0 = a.item_begin + (u64)blockIdx.x * 64; b0 < a.item_end; b0 += (u64)gridDim.x * 64) {
    const u64 i = b0 + lane;
    bool take = false;
    if (i < a.item_end) {
      const u64 w = a.item_w[i];
      const u32 fl = a.flags[w];
      if (fl & A5X_WF_GLOB) {
      } else if (a.rfast && (fl & A5X_WF_FAST)) {  // k_expand_fast writes it (mode_unit)
        if (op == 0 && !route) {
          // -r: every candidate L + 1 bytes; -s / -s -r: one item, sized by the probe
          const u64 cnt = a.cand_off[w + 1] - a.cand_off[w], t0 = (i - a.seg_off[w]) * a.SEG;
          const u64 nc = cnt - t0 < a.SEG ? cnt - t0 : a.SEG;
          a.seg_bytes[i] = a.mode == A5X_MODE_REVERSE ? nc * (a.woff[w + 1] - a.woff[w] + 1) : a.wbytes[w];
          a.item_fl[i] = MI_SKIP;
        }
      } else if (op == 2) {
        // fused digest: single-item words routed to a piece layout by k_mode_count (wbytes
        // flags) go to that layout's kernel, every other item to k_mode_digest_pos (route
        // 0), which marks the byte builder's (MI_BUILD) for k_mode_digest_b
        const u64 wb = a.wbytes[w];
        const uint8_t wr = wb == ~0ull ? 0 : (wb & M_WB_FAST) ? MI_FAST : (wb & M_WB_FAST2) ? MI_FAST2 : 0;
        take = route == MI_BUILD ? wr == 0 && a.item_fl[i] == MI_BUILD : route ? wr == route : wr == 0;
      } else if (route) {
        take = a.item_fl[i] == route;
      } else if (op == 0 && a.wbytes[w] != ~0ull) {  // sized by k_mode_count (one item)
        const u64 wb = a.wbytes[w];
        a.seg_bytes[i] = wb & ~(M_WB_FAST | M_WB_FAST2);
        a.item_fl[i] = (wb & M_WB_FAST) ? MI_FAST : (wb & M_WB_FAST2) ? MI_FAST2 : MI_POS;
      } else {
        take = true;
      }
    }
    // the taken items' metadata, all loads together; each item's word bytes are loaded
    // while the wave runs the item before it
    u64 lw0 = 0, lw1 = 0, lc0 = 0, lc1 = 0, ls0 = 0;
    if (take) {
      const u64 w = a.item_w[i];
      lw0 = a.woff[w]; lw1 = a.woff[w + 1];
      lc0 = a.cand_off[w]; lc1 = a.cand_off[w + 1]; ls0 = a.seg_off[w];
    }
    u64 m = __ballot(take);
    auto meta = [&](u32 l, MPre& P) {
      P.w0 = m_readlane64(lw0, l); P.w1 = m_readlane64(lw1, l);
      P.c0 = m_readlane64(lc0, l); P.c1 = m_readlane64(lc1, l); P.s0 = m_readlane64(ls0, l);
      const u64 L = P.w1 - P.w0;
      P.b0 = (L <= A5X_M_LMAX && lane < L) ? a.words[P.w0 + lane] : 0u;
      P.b1 = (L <= A5X_M_LMAX && lane + 64 < L) ? a.words[P.w0 + lane + 64] : 0u;
    };
    if (!M_PREFETCH) {
      for (; m; m &= m - 1) m_item(S, T, a, b0 + (u64)__builtin_ctzll(m), op);
      continue;
    }
    MPre cur;
    if (m) meta((u32)__builtin_ctzll(m), cur);
    while (m) {
      const u32 l = (u32)__builtin_ctzll(m);
      m &= m - 1;
      MPre nxt;
      if (m) meta((u32)__builtin_ctzll(m), nxt);  // (consumed after this item: latency hidden)
      m_item(S, T, a, b0 + l, op, &cur);
      cur = nxt;
    }
  }
}
__global__ void __launch_bounds__(64) k_mode_items_len(A5xModeLaunch a) { m_items<MLdsC>(a, 0, 0); }
__global__ void __launch_bounds__(64) k_mode_items_len_b(A5xModeLaunch a) { m_items<MLds>(a, 0, MI_BUILD_LEN); }
__global__ void __launch_bounds__(64) k_mode_items_pos(A5xModeLaunch a) { m_items<MLdsR>(a, 1, MI_POS); }
__global__ void __launch_bounds__(64) k_mode_items_b(A5xModeLaunch a) { m_items<MLds>(a, 1, MI_BUILD); }
__global__ void __launch_bounds__(64) k_mode_items_fast(A5xModeLaunch a) { m_items<MLdsF>(a, 1, MI_FAST); }
__global__ void __launch_bounds__(64) k_mode_items_fast2(A5xModeLaunch a) { m_items<MLdsF2>(a, 1, MI_FAST2); }
__global__ void __launch_bounds__(64) k_mode_digest_pos(A5xModeLaunch a) { m_items<MLdsR>(a, 2, 0); }
__global__ void __launch_bounds__(64) k_mode_digest_fast(A5xModeLaunch a) { m_items<MLdsF>(a, 2, MI_FAST); }
__global__ void __launch_bounds__(64) k_mode_digest_fast2(A5xModeLaunch a) { m_items<MLdsF2>(a, 2, MI_FAST2); }
__global__ void __launch_bounds__(64) k_mode_digest_b(A5xModeLaunch a) { m_items<MLds>(a, 2, MI_BUILD); }

// the items of the listed pass-G words inside [item_begin, item_end), dealt to the slots
__global__ void __launch_bounds__(64) k_mode_items_g(A5xModeLaunch a, int op) {
  MLdsG& S = m_gslot(a);
  const MT T = m_table(m_dyn, a.mtab, a.mtab_bytes);
  const u32 ng = *a.glob_n;
  for (u32 k = 0; k < ng; k++) {
    const u64 w = a.glob_list[k];
    const u64 i0 = max(a.seg_off[w], a.item_begin), i1 = min(a.seg_off[w + 1], a.item_end);
    for (u64 i = i0; i < i1; i++)
      if ((i + k) % gridDim.x == blockIdx.x) m_item(S, T, a, i, op);
  }
}

// query q: {item containing g, index inside the item, byte offset of g}; G: only the
// queries inside pass-G words (the LDS pass skips those)
template <class SL>
__device__ void m_locate(SL& S, const MT& T, const A5xModeLaunch& a, const u64* cands, u32 q, u64* out) {
  const u64 g = cands[q];
  const u64 total = a.cand_off[a.nw];
  if (g >= total) {
    if (!SL::G && m_lane() == 0) { out[3 * q] = a.nitems; out[3 * q + 1] = 0; out[3 * q + 2] = a.seg_boff[a.nitems]; }
    return;
  }
  u64 lo = 0, hi = a.nw;  // largest w with cand_off[w] <= g
  while (hi - lo > 1) {
    const u64 mid = (lo + hi) / 2;
    if (a.cand_off[mid] <= g) lo = mid; else hi = mid;
  }
  const u64 w = lo, local = g - a.cand_off[w];
  if (((a.flags[w] & A5X_WF_GLOB) != 0) != SL::G) return;
  const u64 item = a.seg_off[w] + local / a.SEG;
  const u64 t0 = (local / a.SEG) * a.SEG;
  const u32 r = (u32)(local - t0);
  u64 pre = 0;
  if (!SL::G && r && a.rfast && (a.flags[w] & A5X_WF_FAST)) {
    // a FAST word (k_expand_fast numbering): -r candidates are all L + 1 bytes; -s / -s -r
    // (one item): candidates [0, r) summed from the word's plan record, lanes over them
    if (a.mode == A5X_MODE_REVERSE) {
      pre = (u64)r * (a.woff[w + 1] - a.woff[w] + 1);
    } else {
      const u64* rec = a.rec + a.roff[w];
      u32 rr = r;
      u64 sum = 0;
      if (a.flags[w] & A5X_WF_VIRT) {
        // a virtual word: the sub-word holding g, its bytes before g from its record
        u64 v = w + a.vpre[w];
        while (a.vcand_off[v + 1] <= g) v++;
        rec = a.vrec + a.vroff[v];
        rr = (u32)(g - a.vcand_off[v]);
        if (m_lane() == 0) sum = a.vbyte_off[v] - a.vbyte_off[w + a.vpre[w]];
      }
      const u32 np = (u32)rec[0] & 15u;
      for (u32 cnd = m_lane(); cnd < rr; cnd += 64) {
        u32 n = cnd + 1, len = 0;
        for (u32 p = 0; p < np; p++) {
          const u64 G = rec[1 + p];
          const u32 R = ((u32)(G >> 40) & 31u) + 1u, eb = (u32)(G >> 32) & 255u;
          const u32 d = n % R;
          n /= R;
          len += (u32)(rec[1 + np + eb + d] >> 56) & 7u;
        }
        sum += len;
      }
#pragma unroll
      for (int dd = 1; dd < 64; dd <<= 1) sum += (u64)__shfl_xor((long long)sum, dd, 64);
      pre = sum;
    }
    if (m_lane() == 0) { out[3 * q] = item; out[3 * q + 1] = r; out[3 * q + 2] = a.seg_boff[item] + pre; }
    return;
  }
  if (r) {
    const MInfo I = m_setup(S, T, a, w);
    if (I.bad || I.count != a.cand_off[w + 1] - a.cand_off[w]) { m_err(a.err, I.bad ? I.bad : M_ERR_STATE); return; }
    u32 err = 0, ntok = 0;
    if constexpr (!SL::G) {
      ntok = a.mode != A5X_MODE_DEFAULT ? m_pos_setup(S, T, I, a.mode) : 0u;
      if (ntok && S.radix) pre = m_pos_prefix(S, I, t0 + r) - m_pos_prefix(S, I, t0);
    }
    if (!(ntok && S.radix)) pre = m_run(S, T, I, a, t0, r, 0, 0, 0, err, ntok);
    m_err(a.err, m_wave_or(err));
  }
  if (m_lane() == 0) { out[3 * q] = item; out[3 * q + 1] = r; out[3 * q + 2] = a.seg_boff[item] + pre; }
}

// one wave per query g
__global__ void __launch_bounds__(64) k_mode_locate(A5xModeLaunch a, const u64* cands, u32 nq, u64* out) {
  MLds& S = *(MLds*)m_dyn;
  const MT T = m_table(m_dyn + sizeof(MLds), a.mtab, a.mtab_bytes);
  for (u32 q = blockIdx.x; q < nq; q += gridDim.x) m_locate(S, T, a, cands, q, out);
}

__global__ void __launch_bounds__(64) k_mode_locate_g(A5xModeLaunch a, const u64* cands, u32 nq, u64* out) {
  MLdsG& S = m_gslot(a);
  const MT T = m_table(m_dyn, a.mtab, a.mtab_bytes);
  for (u32 q = blockIdx.x; q < nq; q += gridDim.x) m_locate(S, T, a, cands, q, out);
}

// per-word byte offsets / bytes from the per-item byte offsets
__global__ void __launch_bounds__(256) k_mode_wordbytes(const u64* seg_off, const u64* seg_boff, u64 nw,
                                                        u64* byte_off, u64* bytes) {
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 w = (u64)blockIdx.x * blockDim.x + threadIdx.x; w <= nw; w += stride) {
    const u64 b = seg_boff[seg_off[w]];
    byte_off[w] = b;
    if (w < nw && bytes) bytes[w] = seg_boff[seg_off[w + 1]] - b;
  }
}

inline u32 m_grid(u64 n, u32 cap) { return (u32)(n < 1 ? 1 : (n < cap ? n : cap)); }
// word / item kernels: every workgroup stages the mode table into LDS once, so the grid is
// a few workgroups per CU looping over the work (262144 groups re-read the table 262144 times)
#ifndef M_GRID_MAX
#define M_GRID_MAX (1u << 18)
#endif

}  // namespace

size_t a5x_mode_lds(uint32_t mtab_bytes) { return sizeof(MLds) + ((mtab_bytes + 15u) & ~15u); }
template <class SL>
static size_t m_lds(uint32_t mtab_bytes) { return sizeof(SL) + ((mtab_bytes + 15u) & ~15u); }

uint64_t a5x_mode_gslot_bytes() { return (sizeof(MLdsG) + 255) & ~(size_t)255; }

hipError_t a5x_launch_mode_count(const A5xModeLaunch& L, hipStream_t st) {
  hipLaunchKernelGGL(k_mode_count, dim3(m_grid(L.nw, M_GRID_MAX)), dim3(64), m_lds<MLdsC>(L.mtab_bytes), st, L);
  return hipGetLastError();
}

hipError_t a5x_launch_mode_count_thread(const A5xModeLaunch& L, hipStream_t st) {
  const size_t lds = ((L.mtab_bytes + 15u) & ~15u) + 256 * (MCT_SLOT + 4 * MCT_PMAX);
  hipLaunchKernelGGL(k_mode_count_thread, dim3(m_grid((L.nw + 255) / 256, 2048)), dim3(256), lds, st, L);
  return hipGetLastError();
}

hipError_t a5x_launch_mode_count_g(const A5xModeLaunch& L, hipStream_t st) {
  hipLaunchKernelGGL(k_mode_count_g, dim3(L.gslots), dim3(64), (L.mtab_bytes + 15u) & ~15u, st, L);
  return hipGetLastError();
}

hipError_t a5x_launch_mode_items(const A5xModeLaunch& L, int op, hipStream_t st) {
  if (L.item_end <= L.item_begin) return hipSuccess;
  const dim3 g(m_grid((L.item_end - L.item_begin + 63) / 64, L.grid_cap ? L.grid_cap : M_GRID_MAX));  // (64 items a step)
  if (op == 0) {
    hipLaunchKernelGGL(k_mode_items_len, g, dim3(64), m_lds<MLdsC>(L.mtab_bytes), st, L);
    if (L.mode != A5X_MODE_REVERSE)
      hipLaunchKernelGGL(k_mode_items_len_b, g, dim3(64), m_lds<MLds>(L.mtab_bytes), st, L);
  } else if (op == 1) {
    hipLaunchKernelGGL(k_mode_items_fast, g, dim3(64), m_lds<MLdsF>(L.mtab_bytes), st, L);
    hipLaunchKernelGGL(k_mode_items_fast2, g, dim3(64), m_lds<MLdsF2>(L.mtab_bytes), st, L);
    hipLaunchKernelGGL(k_mode_items_pos, g, dim3(64), m_lds<MLdsR>(L.mtab_bytes), st, L);
    hipLaunchKernelGGL(k_mode_items_b, g, dim3(64), m_lds<MLds>(L.mtab_bytes), st, L);
  } else {
    hipLaunchKernelGGL(k_mode_digest_fast, g, dim3(64), m_lds<MLdsF>(L.mtab_bytes), st, L);
    hipLaunchKernelGGL(k_mode_digest_fast2, g, dim3(64), m_lds<MLdsF2>(L.mtab_bytes), st, L);
    hipLaunchKernelGGL(k_mode_digest_pos, g, dim3(64), m_lds<MLdsR>(L.mtab_bytes), st, L);
    hipLaunchKernelGGL(k_mode_digest_b, g, dim3(64), m_lds<MLds>(L.mtab_bytes), st, L);
  }
  if (L.gscr && L.gslots)
    hipLaunchKernelGGL(k_mode_items_g, dim3(L.gslots), dim3(64), (L.mtab_bytes + 15u) & ~15u, st, L, op);
  return hipGetLastError();
}

hipError_t a5x_launch_mode_locate(const A5xModeLaunch& L, const uint64_t* cands, uint32_t n, uint64_t* out,
                                  hipStream_t st) {
  hipLaunchKernelGGL(k_mode_locate, dim3(m_grid(n, 64)), dim3(64), a5x_mode_lds(L.mtab_bytes), st, L, cands, n, out);
  if (L.gscr && L.gslots)
    hipLaunchKernelGGL(k_mode_locate_g, dim3(L.gslots < n ? L.gslots : (n ? n : 1)), dim3(64),
                       (L.mtab_bytes + 15u) & ~15u, st, L, cands, n, out);
  return hipGetLastError();
}

hipError_t a5x_launch_mode_wordbytes(const uint64_t* seg_off, const uint64_t* seg_boff, uint64_t nw,
                                     uint64_t* byte_off, uint64_t* bytes, hipStream_t st) {
  hipLaunchKernelGGL(k_mode_wordbytes, dim3(m_grid((nw + 256) / 256, 65536)), dim3(256), 0, st, seg_off, seg_boff,
                     nw, byte_off, bytes);
  return hipGetLastError();
}
