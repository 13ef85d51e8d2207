// a5x_kernels.hip -- CDNA4 (gfx950) kernels for hashcat -a 5 table expansion.
//
// Hot path = processWord (/root/reference/main.go:168-205): for every word, every
// set of non-overlapping key matches (byte positions of the ORIGINAL word) with
// max(1,min) <= |set| <= max, times every choice of one value per match, spliced
// in and written as "cand\n" (main.go:66).  The candidate multiset per word is the
// contract (the reference's output order is nondeterministic, main.go:77).
//
// Pipeline (one HIP stream, see a5x_host.cpp):
//   k_keyspace_thread  one lane per word: matching + closed-form mixed-radix
//                      count/bytes for words whose matches are disjoint single
//                      keys (SURVEY 8(a) fast path); everything else deferred.
//   k_keyspace_wave    one wave per deferred word: interval DP G[p][c] (counts)
//                      and H[p][c] (bytes) in LDS, lanes over the count column c.
//   k_scan_*           exclusive scan of (count, bytes) -> global candidate and
//                      byte offsets per word.
//   k_plan             chunk -> first word map (chunks of CH candidates).
//   k_expand<A|B>      one wave per chunk: per-word setup in LDS, each lane unranks
//                      one candidate (mixed radix or DP walk), wave scan of
//                      lengths, bytes OR-ed into a per-wave LDS ring at their
//                      final offsets, complete 16-B blocks streamed to HBM with
//                      global_store_dwordx4 (1 KiB per wave instruction).
//   k_digest           per-word order-independent multiset digest of the output
//                      (verification only).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string.h>

#include <type_traits>

#include "a5x_format.h"
#include "a5x_plan.h"
#include "a5x_launch.h"

#define WAVE_SYNC()                                          \
  do {                                                       \
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");   \
    __builtin_amdgcn_wave_barrier();                         \
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   \
  } while (0)

// Wave sync of the per-word path: its WaveLds / ring live in LDS, except in pass G
// (LMAX == A5X_LMAX_G) where they are HBM scratch written and read by the wave's own
// lanes (one CU): workgroup-scope release/acquire drains the stores and atomics (the
// CU's L1 never holds a stale copy of its own stores; the ring is only touched by
// L2 atomics).
template <int LMAX>
__device__ __forceinline__ void ws_sync() {
  if constexpr (LMAX > A5X_LMAX_B) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  } else {
    WAVE_SYNC();
  }
}

// Diagnostic build only (-DA5X_STAMPS): per-phase s_memtime cycle sums of the
// fast kernel, read back with a5x_debug_stamps().  Never in the shipped build.
#ifdef A5X_STAMPS
__device__ unsigned long long g_a5x_stamps[16];
#define STAMP_DECL unsigned long long st_t = __builtin_amdgcn_s_memtime(), st_acc[10] = {0,0,0,0,0,0,0,0,0,0};
#define STAMP(i) do { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); st_acc[i] += t_ - st_t; st_t = t_; } while (0)
#define STAMP_FLUSH() do { if (lane_id() == 0) for (int i_ = 0; i_ < 10; i_++) atomicAdd(&g_a5x_stamps[i_], st_acc[i_]); } while (0)
#else
#define STAMP_DECL
#define STAMP(i) do {} while (0)
#define STAMP_FLUSH() do {} while (0)
#endif

enum : u32 {
  A5X_DERR_TABLE = 1u << 0,   // table blob does not fit LDS / bad magic
  A5X_DERR_OVF = 1u << 1,     // u64 overflow in a keyspace
  A5X_DERR_BIG = 1u << 2,     // a word beyond pass-B limits has candidates
  A5X_DERR_STATE = 1u << 3,   // internal consistency (keyspace vs expand)
  A5X_DERR_SCANOVF = 1u << 4, // prefix sum overflow
  A5X_DERR_GUARD = 1u << 5,   // a device bounds guard tripped (see the debug record)
};

// ---------------------------------------------------------------------------
// small helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ u32 lane_id() { return __lane_id(); }

__device__ __forceinline__ u64 shfl_u64(u64 v, int src) {
  u32 lo = __shfl((int)(u32)v, src), hi = __shfl((int)(u32)(v >> 32), src);
  return ((u64)hi << 32) | lo;
}
__device__ __forceinline__ u64 shfl_up_u64(u64 v, int d) {
  u32 lo = __shfl_up((int)(u32)v, d), hi = __shfl_up((int)(u32)(v >> 32), d);
  return ((u64)hi << 32) | lo;
}
__device__ __forceinline__ u64 shfl_xor_u64(u64 v, int m) {
  u32 lo = __shfl_xor((int)(u32)v, m), hi = __shfl_xor((int)(u32)(v >> 32), m);
  return ((u64)hi << 32) | lo;
}
// Wave64 inclusive prefix sum on DPP (VALU only, no LDS): row_shr 1/2/4/8 inside
// each 16-lane row, then row_bcast:15 (rows 1, 3) and row_bcast:31 (rows 2, 3).
// The sequence LLVM's AMDGPU atomic optimizer uses on gfx9.
__device__ __forceinline__ u32 wave_incl_scan_u32(u32 x) {
  x += (u32)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);
  x += (u32)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);
  x += (u32)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);
  x += (u32)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);
  x += (u32)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);
  x += (u32)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);
  return x;
}
__device__ __forceinline__ u32 lane63(u32 x) { return (u32)__builtin_amdgcn_readlane((int)x, 63); }
__device__ __forceinline__ u32 readlane_u32(u32 x, u32 l) { return (u32)__builtin_amdgcn_readlane((int)x, (int)l); }
__device__ __forceinline__ u64 readlane_u64(u64 x, u32 l) {
  return ((u64)readlane_u32((u32)(x >> 32), l) << 32) | (u64)readlane_u32((u32)x, l);
}
// Whole-wave reductions on DPP (row_shr 1/2/4/8, row_bcast 15/31, as the scan above):
// no cross-lane address registers (ds_bpermute index VGPRs that the compiler would
// keep live through the whole kernel).  The result is uniform (lane 63).
#define A5X_DPP_REDUCE(x, OP)                                                                 \
  do {                                                                                         \
    x = OP(x, (u32)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false));            \
    x = OP(x, (u32)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false));            \
    x = OP(x, (u32)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false));            \
    x = OP(x, (u32)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false));            \
    x = OP(x, (u32)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false));            \
    x = OP(x, (u32)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false));            \
  } while (0)
__device__ __forceinline__ u32 a5x_max(u32 a, u32 b) { return a > b ? a : b; }
__device__ __forceinline__ u32 a5x_or(u32 a, u32 b) { return a | b; }
__device__ __forceinline__ u32 wave_max_u32(u32 x) {
  A5X_DPP_REDUCE(x, a5x_max);
  return lane63(x);
}
__device__ __forceinline__ u32 wave_or_u32(u32 x) {
  A5X_DPP_REDUCE(x, a5x_or);
  return lane63(x);
}
// 64-bit sum (mod 2^64, so also for two's-complement i64) in three 24/24/16-bit parts:
// each part's 64-lane sum fits 32 bits
__device__ __forceinline__ u64 wave_sum_u64(u64 x) {
  u32 a = wave_incl_scan_u32((u32)x & 0xFFFFFFu);
  u32 b = wave_incl_scan_u32((u32)(x >> 24) & 0xFFFFFFu);
  u32 c = wave_incl_scan_u32((u32)(x >> 48));
  return (u64)lane63(a) + ((u64)lane63(b) << 24) + ((u64)lane63(c) << 48);
}
__device__ __forceinline__ i64 wave_sum_i64(i64 x) { return (i64)wave_sum_u64((u64)x); }
// readfirstlane returns int: convert through u32 so nothing sign-extends
__device__ __forceinline__ u32 uniform(u32 x) { return (u32)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __forceinline__ u64 uniform64(u64 x) {
  return ((u64)uniform((u32)(x >> 32)) << 32) | (u64)uniform((u32)x);
}

__device__ __forceinline__ u32 keep_bytes(u32 v, u32 n) { return n >= 4 ? v : (v & ((1u << (8 * n)) - 1u)); }

// unaligned 4-byte read from LDS (base must have 8 readable bytes past off)
__device__ __forceinline__ u32 lds_ld4(const uint8_t* base, u32 off) {
  const u32* p = (const u32*)(base + (off & ~3u));
  u32 lo = p[0], hi = p[1];
  return __builtin_amdgcn_alignbyte(hi, lo, off & 3u);
}

// whole workgroup copies the table blob (multiple of 16 B) into LDS
__device__ __forceinline__ void load_table(uint8_t* dst, const uint8_t* src, u32 bytes) {
  const uint4* s = (const uint4*)src;
  uint4* d = (uint4*)dst;
  for (u32 i = threadIdx.x; i < bytes / 16; i += blockDim.x) d[i] = s[i];
}

// does key k match the word (global bytes) at p?  caller checked p+klen <= L
__device__ __forceinline__ bool key_match_global(const uint8_t* wp, u32 p, const A5xKey& key, const Tab& T) {
  const A5xChoice c0 = T.ch[key.choice_base];
  u32 kl = key.klen;
  for (u32 i = 1; i < kl; i++) {  // byte 0 matched by the bucket
    u32 kb = i < 4 ? ((c0.first4 >> (8 * i)) & 255u) : T.blob[c0.blob_off + i];
    if (wp[p + i] != kb) return false;
  }
  return true;
}


// ---------------------------------------------------------------------------
// Keyspace, one lane per word (radix fast path; SURVEY 8(a) closed form)
// ---------------------------------------------------------------------------
struct KsArgs {
  const uint8_t* table;
  u32 table_bytes;
  const uint8_t* words;
  const u64* woff;
  u64 nw;
  int mn, mx;
  u64* count;
  u64* bytes;
  u32* flags;
  u32* defer_list;
  u32* defer_n;
  u32* nbig;
  u32* nslow;
  u32* big_list;   // words for k_expand_b (index = *nbig at append)
  u32* slow_list;  // words for k_expand_slow (index = *nslow at append)
  u32* err;
  u64* rec;     // FAST plan records: tile t owns rec[t * FW_TILE_REC, (t + 1) * FW_TILE_REC)
  u32* roff;    // per word: record offset (u64 units) into rec
  u32* cplx_list;  // words for k_keyspace_cplx
  u32* cplx_n;
  u32 cplx_cap;    // record slots (FW_RMAX u64 each) at rec + cplx_base
  u64 cplx_base;
  u32* glob_list;  // pass G words (k_keyspace_wave -> k_keyspace_g)
  u32* glob_n;
  uint8_t* gscr;   // pass G scratch slots
  int rmode;       // 1 / 2 / 3: -r / -s / -s -r FAST probe (k_keyspace_thread only;
                   // mode_unit below): the other words are appended to defer_list
  u32 rcmin;       // -r: max(min, 0) (0 or 1 for a FAST word)
  u64* rnseg;      // -r: mode-engine items per FAST word (ceil(count / rseg))
  u64 rseg;
  // -s / -s -r virtual words (k_keyspace_vsub over the probe's leftover list defer_list)
  u32* vout_list;  // the words left to the mode engine
  u32* vout_n;
  u64* vn;         // per word: sub-words - 1 (virtual words; 0 elsewhere)
  u64* vrsz;       // per word: record u64 of its FAST entries (virtual words; k_vwords_sizes the rest)
  u64* vrec;       // per virtual word: its sub-word records, then one meta u64 per sub-word
  unsigned long long* vrec_n;  // bump counter of vrec (u64 units)
  u64 vrec_cap;
  uint16_t* vocc;  // per word 16 u16: the occurrence row of k_keyspace_thread's -s / -s -r words
                   // with a repeated pattern (null: none logged)
  u32* vlong_list;  // k_keyspace_vsub small instantiation: the words for the large one
  u32* vlong_n;
  const u32* hiflag;  // k_keyspace_thread: the batch has bytes >= 0x80 (null: the byte walk only)
};

// Whether the batch's words hold bytes >= 0x80, judged on its first 256 KiB (the choice
// only picks the faster of two exact walks: k_keyspace_thread<true> steps over UTF-8
// continuation bytes, <false> walks every byte); one atomic per wave that saw one.
__global__ void __launch_bounds__(256) k_hibytes(const uint8_t* words, const u64* woff, u64 nw, u32* flag) {
  const uintptr_t b0 = (uintptr_t)(words + woff[0]) & ~(uintptr_t)3, b1 = (uintptr_t)(words + woff[nw]);
  const u64 nd = min((u64)((b1 - b0 + 3) / 4), (u64)65536);  // (16 readable bytes past the batch)
  const u32* d = (const u32*)b0;
  u32 acc = 0;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < nd; i += (u64)gridDim.x * blockDim.x) acc |= d[i];
  if (__builtin_amdgcn_ballot_w64((acc & 0x80808080u) != 0u) && lane_id() == 0) atomicOr(flag, 1u);
}

// -r / -s / -s -r on the FAST path (the mode-engine probe of k_keyspace_thread, rmode =
// 1 / 2 / 3).  The lone units of the position-synchronous walk are the word's match
// positions when those are pairwise disjoint.
//   -r (processWordReverse, main.go:208-261): every key's subs[0] keeps the key's length
//      (the running offset of main.go:251-256 then moves nothing); candidate = any subset
//      of the positions replaced by subs[0]: a unit of 2 choices (choice 0 = the key,
//      choice 1 = subs[0], a5x_format.h) per position.
//   -s / -s -r (main.go:308-365, 369-440): every pattern occurs once in the word and
//      passes the static positional checks (A5xKey.pad0, key_pos_facts: one codepoint,
//      values containing no key), so sequential ReplaceAll = replacing each occurrence:
//      a unit of 1 + values (-s) or 2 (-s -r: subs[0]) choices per pattern.  seen: the
//      patterns met so far (key index mod 64; a collision is taken for a repeat).
// The size window cuts nothing when min <= 1 and max >= #units; count = P - min (min 0:
// the all-keep word is index P of the FAST numbering, whose digits wrap to zero).
// Returns false when the unit does not qualify (the mode engine takes the word).
__device__ __forceinline__ bool mode_unit(const Tab& T, Unit& U, int rmode, u64& seen, bool check) {
  const A5xKey key = T.keys[U.key];
  if (rmode == 1) {
    if (key.nvals < 1 || T.ch[key.choice_base + 1].len != key.klen) return false;
    U.R = 2; U.ml = key.klen; U.mnl = key.klen; U.spos = 0; U.sneg = 0; U.maxd = 0;
    return true;
  }
  if (check) {
    if (!(key.pad0 & (rmode == 2 ? 1u : 2u)) || key.nvals < 1) return false;
    const u64 bit = 1ull << (U.key & 63u);
    if (seen & bit) return false;
    seen |= bit;
  }
  if (rmode == 3) {  // subs[0] only
    const u32 vl = T.ch[key.choice_base + 1].len, kl = key.klen;
    U.R = 2; U.ml = max(kl, vl); U.mnl = min(kl, vl);
    U.spos = vl > kl ? vl - kl : 0u; U.sneg = kl > vl ? kl - vl : 0u; U.maxd = (int)vl - (int)kl;
  }
  return true;
}

// Append the lanes with pred to list[*ctr ...] (one atomic per wave); returns the
// lane's slot (valid where pred).  Every lane of the wave must call it.
__device__ __forceinline__ u32 wave_append(bool pred, u32* ctr) {
  const u64 m = __ballot(pred);
  if (!m) return 0;
  const u32 lane = lane_id(), leader = (u32)__builtin_ctzll(m);
  u32 base = 0;
  if (lane == leader) base = atomicAdd(ctr, (u32)__popcll(m));
  base = (u32)__shfl((int)base, (int)leader);
  return base + (u32)__popcll(m & ((1ull << lane) - 1ull));
}

#ifndef KS_ABL
#define KS_ABL 0  // keyspace timing ablations (variant builds only, wrong output): 1 no build pass,
                  // 2 no planner in the count pass, 4 no record stores
#endif

// k_keyspace_thread's open group holds KS_GCAP entries (a unit with more choices
// makes the word complex: k_keyspace_cplx plans it with FW_UMAXR)
#define KS_GCAP 8

// The open group of plan_word lives in LDS (<= FW_UMAXR u64 per lane, lane-strided);
// entries and group descriptors go straight to the word's record in HBM.
struct DevRecSink {
  u64* g;       // LDS: g[a * 256]
  u64* c;       // LDS: cluster choices c[a * 256] (k_keyspace_cplx only)
  u64* rec;     // global record base
  u32 np;
  __device__ u64* cbuf() const { return c; }
  __device__ u32 cstride() const { return 256u; }
  __device__ u64 gld(u32, u32 a) const { return g[a * 256u]; }
  __device__ void gst(u32, u32 a, u64 v) { g[a * 256u] = v; }
  __device__ void ent(u32 i, u64 v) { if (!(KS_ABL & 4)) rec[1 + np + i] = v; }
  __device__ void desc(u32 i, u64 v) { if (!(KS_ABL & 4)) rec[1 + i] = v; }
};

// A word's bytes staged in LDS (the keyspace tile); 8 readable bytes past any word.
struct LWord {
  const uint8_t* base;
  u32 off;
  __device__ __forceinline__ u32 at(u32 i) const { return base[off + i]; }
  __device__ __forceinline__ u64 ld(u32 i, u32 n) const {
    const u64 v = (u64)lds_ld4(base, off + i) | ((u64)lds_ld4(base, off + i + 4) << 32);
    return keep_bytes64(v, n);
  }
};

#ifndef KS_WB
#define KS_WB 8192  // tile word bytes staged in LDS (larger tiles read global memory)
#endif

template <class W>
__device__ __forceinline__ u32 ks_classify(const W& wd, u64 L64, const Tab& T, const KsArgs& a, WordClass& C) {
  if (L64 > A5X_LMAX_A && a.mx >= 1) return A5X_WF_DEFER;  // long words: the wave kernel
  C = classify_word(wd, (u32)L64, T, a.mn, a.mx, A5X_RING_A - 16);
  u32 f = C.flags;
  if (C.ovf) atomicOr(a.err, A5X_DERR_OVF);
  if ((f & A5X_WF_DEFER) || !(f & (A5X_WF_FAST | A5X_WF_RADIX | A5X_WF_ERR_OVF)))
    f = A5X_WF_DEFER;  // capped windows, unit limits, non-FAST clusters: the DP kernel
  return f;
}

template <class W>
__device__ __forceinline__ void ks_build(const W& wd, u32 L, const Tab& T, const KsArgs& a, u32 f, u64 count, u64* rec,
                                         u64* g) {
  DevRecSink sk;
  sk.g = g; sk.c = g + 256 * FW_UMAXR; sk.rec = rec; sk.np = ff_np(f);
  const Plan P = plan_word<true>(wd, L, T, sk, fb_balanced_cap(count + 1));
  rec[0] = fr_hdr(P.np, P.ng, P.ne, P.maxl, P.nbig, P.bstarts, P.bRp);
  if (!P.ok || P.ng != ff_ng(f) || P.ne != ff_ne(f) || P.np != ff_np(f)) atomicOr(a.err, A5X_DERR_STATE);
}

// Position-synchronous word walk of k_keyspace_thread: every lane steps through byte
// positions q = 0, 1, ... of its own word together (one fixed-size body per
// position), so a wave of words costs max(L) steps instead of the union of 64
// data-dependent loops.  At q: the keys of the first-byte bucket are compared (4
// bytes at once; keys of <= 4 bytes); a lone match starts a unit handed to the
// Planner (and the closed-form count).  Two matches at one position or a match
// inside a unit's span (overlapping keys: clusters), or a key longer than 4 bytes
// at q, make the word "complex": k_keyspace_cplx walks it with next_unit.
// ulog (count pass only): the lane's lone units as (q << 10 | key) at ulog[i * 256];
// nlog = their number, KS_ULOG + 1 when they do not fit (the build pass re-walks).
#ifndef KS_ULOG
#define KS_ULOG 16
#endif
__device__ bool psk_norep;  // (psk_walk's rep when the caller does not track repeats: never written)
#ifndef PSK_KB
#define PSK_KB 2  // bucket keys read together per position (more: a loop)
#endif
template <bool COUNT, bool UTF, class PL>
__device__ __forceinline__ void psk_walk(const LWord& lw, u32 L, bool act0, u32 Lmax, u32 bmax, const Tab& T,
                                         PL& pl, CountAcc& A, bool& cplx, int rmode, uint16_t* ulog = nullptr,
                                         u32* nlog = nullptr, bool logrep = false, bool& rep = psk_norep) {
  u32 cur_end = 0;
  u64 seen = 0;
  // one position q of the lane's word; returns the bytes to the next position that can
  // start a key (UTF: the continuation bytes after q are passed over)
  auto pos = [&](u32 q) -> u32 {
    // three dependent LDS trips per position: the word's 4 bytes, the byte's bucket, the
    // bucket's keys (compact first-4-bytes | length records, read together)
    const u32 w4 = lds_ld4(lw.base, lw.off + q);
    const u32 c1 = UTF && ((w4 >> 8) & 0xC0u) == 0x80u ? 1u : 0u;
    const u32 c2 = c1 && ((w4 >> 16) & 0xC0u) == 0x80u ? 1u : 0u;
    const u32 c3 = c2 && (w4 >> 30) == 2u ? 1u : 0u;
    const u32 bk = T.bucket2[w4 & 255u];
    const u32 ks = bk & 0xFFFFu, ke = bk >> 16;
    const u32 nk1 = T.hdr->nkeys ? T.hdr->nkeys - 1u : 0u;
    u32 nm = 0, kk = 0;
    u64 kmv[PSK_KB];
#pragma unroll
    for (u32 i = 0; i < PSK_KB; i++) kmv[i] = T.kmatch[min(ks + i, nk1)];
    auto test = [&](u32 k2, u64 km) {
      const u32 kl = (u32)(km >> 32) & 0xFFFFu;
      if (k2 < ke && q + kl <= L) {
        if (kl > 4) {
          cplx = true;
        } else {
          const u32 m = kl >= 4 ? 0xFFFFFFFFu : ((1u << (8 * kl)) - 1u);
          if ((w4 & m) == (u32)km) { nm++; kk = k2; }
        }
      }
    };
#pragma unroll
    for (u32 i = 0; i < PSK_KB; i++) test(ks + i, kmv[i]);
    for (u32 i = PSK_KB; i < bmax; i++) test(ks + i, T.kmatch[min(ks + i, nk1)]);
    if (nm > 1 || (nm == 1 && q < cur_end)) {
      cplx = true;
    } else if (nm == 1 && !cplx) {
      Unit U;
      lone_unit(T, q, kk, U);
      // -s / -s -r with rep: a positional pattern met again is a tied occurrence -- no
      // unit (the word is not FAST); the walk goes on logging the occurrences for
      // k_keyspace_vsub (seen holds key index mod 64: a collision is taken for a repeat)
      const bool again = logrep && rmode >= 2 && ((seen >> (kk & 63u)) & 1u) &&
                         (T.keys[kk].pad0 & (rmode == 2 ? 1u : 2u)) && T.keys[kk].nvals >= 1;
      bool logit = again;
      if (again) {
        rep = true;
        cur_end = U.e;
      } else if (rmode && !mode_unit(T, U, rmode, seen, true)) {
        cplx = true;
      } else if (U.R > KS_GCAP) {
        cplx = true;
      } else {
        if (COUNT) count_unit(A, U);
        if (!(KS_ABL & 2)) pl.unit(U);
        cur_end = U.e;
        logit = true;
      }
      if (COUNT && ulog && logit) {
        const bool fits = *nlog < KS_ULOG && kk < 1024u && q < 64u;
        if (fits) ulog[*nlog * 256u] = (uint16_t)((q << 10) | kk);
        *nlog = fits ? *nlog + 1u : (u32)KS_ULOG + 1u;
      }
    }
    return 1u + c1 + c2 + c3;
  };
  if constexpr (!UTF) {
    // every lane at byte q together (q wave-uniform)
    for (u32 q = 0; q < Lmax; q++)
      if (act0 && q < L && !cplx) (void)pos(q);
  } else {
    // a batch with UTF-8 and a table whose keys start on lead bytes only (lead_only): every
    // lane at its own position, continuation bytes passed over (2-byte letters: half the
    // steps; the instantiation k_keyspace_thread<true>)
    u32 q = 0;
    for (u32 it = 0; it < Lmax; it++) {
      const bool act = act0 && q < L && !cplx;
      if (!__builtin_amdgcn_ballot_w64(act)) break;
      if (act) q += pos(q);
    }
  }
}


// One lane per word, one 256-word tile per workgroup iteration: classification,
// closed-form (count, bytes), and for FAST words the plan record, packed densely
// in word order inside the tile's record region (workgroup scan of the sizes).
// The tile's word bytes are staged in LDS with 16-B loads.
template <bool UTF>
__global__ void __launch_bounds__(256) k_keyspace_thread(KsArgs a) {
  // (hiflag: the batch has bytes >= 0x80 -- k_hibytes; the other instantiation does nothing)
  if (a.hiflag && (*a.hiflag != 0u) != UTF) return;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const u32 tb = (a.table_bytes + 15u) & ~15u;
  u64* gbuf = (u64*)(smem + tb);                       // 256 x KS_GCAP open-group entries
  u32* wsum = (u32*)(smem + tb + 256 * KS_GCAP * 8);   // per-wave sums of the scan
  uint8_t* wb = smem + tb + 256 * KS_GCAP * 8 + 64;    // KS_WB + 32 tile bytes
  uint16_t* ulog = (uint16_t*)(wb + KS_WB + 32) + threadIdx.x;  // KS_ULOG x 256 unit log
  load_table(smem, a.table, a.table_bytes);
  __syncthreads();
  const Tab T = tab_view(smem);
  const u32 bmax = T.hdr->max_bucket;
  const u32 tid = threadIdx.x, lane = lane_id(), wv = tid / 64;
  const u64 ntiles = (a.nw + FW_TILE - 1) / FW_TILE;
  for (u64 tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const u64 w = tile * FW_TILE + tid;
    const bool valid = w < a.nw;
    const u64 t0 = tile * FW_TILE, t1 = min(a.nw, t0 + FW_TILE);
    const u64 A0 = a.woff[t0] & ~15ull, A1 = a.woff[t1];
    const bool staged = A1 - A0 <= KS_WB;
    if (staged) {
      const uint4* src = (const uint4*)(a.words + A0);
      const u32 nq = (u32)((A1 - A0 + 15) / 16);
      for (u32 i = tid; i < nq + 2; i += 256) {
        uint4 v = make_uint4(0, 0, 0, 0);
        if (A0 + 16ull * (i + 1) <= A1) {
          v = src[i];
        } else if (i < nq) {  // the tile's last partial quad: never read past the batch
          u32 x[4] = {0, 0, 0, 0};
          for (u32 b = 0; A0 + 16ull * i + b < A1; b++) x[b >> 2] |= (u32)a.words[A0 + 16ull * i + b] << (8 * (b & 3));
          v = make_uint4(x[0], x[1], x[2], x[3]);
        }
        ((uint4*)wb)[i] = v;
      }
    }
    __syncthreads();
    u64 s = 0, L64 = 0;
    if (valid) {
      s = a.woff[w];
      L64 = a.woff[w + 1] - s;
    }
    const bool longw = valid && L64 > A5X_LMAX_A && a.mx >= 1;   // the wave DP kernel
    const bool trivial = valid && (a.mx < 1 || L64 == 0);       // processWord emits nothing
    bool cplx = valid && !longw && !trivial && !staged;
    const bool psk = valid && !longw && !trivial && staged;
    const u32 L = psk ? (u32)L64 : 0u;
    LWord lw;
    lw.base = wb; lw.off = psk ? (u32)(s - A0) : 0u;
    // ---- pass 1: units -> counts + piece plan (count mode) ----
    CountAcc A;
    count_init(A, L);
    NullSink ns;
    Planner<false, LWord, NullSink, KS_GCAP> pl(lw, T, ns);
    u32 nlog = 0;
    const bool rm = a.rmode != 0;
    bool rep = false;  // (-s / -s -r with vocc: a repeated pattern; the occurrences logged)
    psk_walk<true, UTF>(lw, L, psk, wave_max_u32(L), bmax, T, pl, A, cplx, a.rmode, ulog, &nlog, a.vocc != nullptr, rep);
    WordClass C;
    C.flags = 0; C.count = 0; C.bytes = 0; C.ovf = false; C.clusters = false;
    u32 f = 0;
    if (psk && !cplx) {
      pl.finish(L);
      C = classify_finish(A, pl.P, L, a.mn, a.mx, A5X_RING_A - 16);
      f = C.flags;
      if (C.ovf) atomicOr(a.err, A5X_DERR_OVF);
      if ((f & A5X_WF_DEFER) || !(f & (A5X_WF_FAST | A5X_WF_RADIX | A5X_WF_ERR_OVF))) f = A5X_WF_DEFER;
    }
    if (trivial) f = A5X_WF_RADIX | A5X_WF_FAST;
    if (longw) f = A5X_WF_DEFER;
    if (rm) {
      // mode FAST words (mode_unit): count = P - rcmin, the all-keep word's L + 1 bytes
      // added when min = 0; -s / -s -r words only as one mode-engine item (the length pass
      // takes their bytes whole); every other word (flags 0) is left to the mode engine
      const u64 cnt = A.P - a.rcmin;
      const bool rf = psk && !cplx && !rep && (f & A5X_WF_FAST) && !(f & A5X_WF_DEFER) && A.nunits > 0 &&
                      C.count > 0 && (a.rmode == 1 || cnt <= a.rseg);
      f = rf ? f : 0u;
      C.bytes = rf ? C.bytes + (a.rcmin ? 0ull : (u64)(L + 1)) : 0ull;
      C.count = rf ? cnt : 0ull;
    }
    // ---- record sizes -> exclusive workgroup scan ----
    const bool fast = psk && !cplx && (f & A5X_WF_FAST) && C.count > 0;
    const u32 rs = fast ? ff_rsize(f) : 0u;
    const u32 inc = wave_incl_scan_u32(rs);
    if (lane == 63) wsum[wv] = inc;
    __syncthreads();
    u32 base = 0;
    for (u32 k = 0; k < wv; k++) base += wsum[k];
    const u32 ro = base + inc - rs;
    const bool build = fast && ro + rs <= FW_TILE_REC;
    // ---- pass 2: the records of the FAST words (same walk, build mode) ----
    {
      u64* rec = a.rec + tile * FW_TILE_REC + ro;
      DevRecSink sk;
      sk.g = gbuf + tid; sk.c = sk.g; sk.rec = rec; sk.np = ff_np(f);  // no clusters here
      Planner<true, LWord, DevRecSink, KS_GCAP> pb(lw, T, sk, build ? fb_balanced_cap(C.count + 1) : 0u);
      CountAcc A2;
      bool c2 = false;
      // replay the logged units (no second byte walk); words with more units re-walk
      const bool replay = nlog <= KS_ULOG;
      const u32 nrep = build && replay ? nlog : 0u;
      for (u32 i = 0; i < wave_max_u32((KS_ABL & 1) ? 0u : nrep); i++) {
        if (i < nrep) {
          const u32 e = ulog[i * 256u];
          Unit U;
          lone_unit(T, e >> 10, e & 1023u, U);
          u64 seen = 0;
          if (rm) (void)mode_unit(T, U, a.rmode, seen, false);  // (qualified in the count pass)
          pb.unit(U);
        }
      }
      const bool walk = build && !replay;
      if (!(KS_ABL & 1)) psk_walk<false, UTF>(lw, L, walk, wave_max_u32(walk ? L : 0u), bmax, T, pb, A2, c2, a.rmode);
      if (build && !(KS_ABL & 1)) {
        pb.finish(L);
        pb.pick_balanced();
        const Plan& P = pb.P;
        rec[0] = fr_hdr(P.np, P.ng, P.ne, P.maxl, P.nbig, P.bstarts, P.bRp);
        if (c2 || !P.ok || P.ng != ff_ng(f) || P.ne != ff_ne(f) || P.np != ff_np(f)) atomicOr(a.err, A5X_DERR_STATE);
        a.roff[w] = (u32)(tile * FW_TILE_REC + ro);
      }
    }
    if (fast && !build) {
      // the tile's record budget is spent: the slow path takes the word (-r: the mode engine)
      f = rm ? 0u : C.clusters ? A5X_WF_DEFER : (f & (A5X_WF_RADIX | A5X_WF_BIN));
    }
    if (rm) {
      // Whether a word is FAST must not depend on its tile (hit numbering, FAST order vs the
      // mode engine's, is per word: a5x_format_hits re-runs a sub-batch, shards re-tile): a
      // word of an unstaged tile, or one past the tile's record budget, is listed for
      // k_keyspace_rprobe, which probes it alone and plans it into a fixed overflow slot.
      const bool rov = (valid && !longw && !trivial && !staged) || (fast && !build);
      const bool kept = valid && !rov && (f & A5X_WF_FAST) != 0;
      if (valid) {
        a.count[w] = kept ? C.count : 0ull;
        a.bytes[w] = kept ? C.bytes : 0ull;
        a.flags[w] = kept ? f : 0u;
        a.rnseg[w] = kept ? (C.count + a.rseg - 1) / a.rseg : 0ull;
      }
      const u32 ri = wave_append(rov, a.cplx_n);
      if (rov) a.cplx_list[ri] = (u32)w;
      const u32 mi = wave_append(valid && !kept && !rov, a.defer_n);  // the mode engine's words
      if (valid && !kept && !rov) a.defer_list[mi] = (u32)w;
      if (a.vocc && valid && !kept) {
        // the occurrence row of a word with a repeated pattern (k_keyspace_vsub): <= 15
        // entries q << 10 | key, row[15] = their number; 0xFFFF: not logged (vsub walks)
        const bool logged = rep && !cplx && psk && nlog <= 15u;
        u32 r[8];
#pragma unroll
        for (u32 k = 0; k < 8; k++) {
          const u32 e0 = 2 * k < nlog ? ulog[(2 * k) * 256u] : 0u, e1 = 2 * k + 1 < nlog ? ulog[(2 * k + 1) * 256u] : 0u;
          r[k] = e0 | (e1 << 16);
        }
        r[7] = (r[7] & 0xFFFFu) | ((logged ? nlog : 0xFFFFu) << 16);
        uint4* row = (uint4*)(a.vocc + w * 16);
        row[0] = make_uint4(r[0], r[1], r[2], r[3]);
        row[1] = make_uint4(r[4], r[5], r[6], r[7]);
      }
      __syncthreads();
      continue;
    }
    // ---- lists (one atomic per wave each) and per-word results ----
    const u32 ci = wave_append(cplx, a.cplx_list ? a.cplx_n : a.defer_n);
    if (cplx) a.cplx_list[ci] = (u32)w;
    const bool dfr = valid && !cplx && (f & A5X_WF_DEFER);
    const u32 di = wave_append(dfr, a.defer_n);
    if (dfr) a.defer_list[di] = (u32)w;
    const bool slow = valid && !cplx && !(f & (A5X_WF_DEFER | A5X_WF_FAST | A5X_WF_ERR_OVF));
    const u32 si = wave_append(slow, a.nslow);
    if (slow) a.slow_list[si] = (u32)w;
    if (valid && !cplx) {
      a.count[w] = (f & A5X_WF_DEFER) ? 0 : C.count;
      a.bytes[w] = (f & A5X_WF_DEFER) ? 0 : C.bytes;
      a.flags[w] = f;
    }
    __syncthreads();  // wb / wsum are rewritten by the next tile
  }
}

#define RP_SLOT 80  // k_keyspace_rprobe: per-lane LDS word slot (words <= A5X_LMAX_A bytes + over-read)

// The -r / -s / -s -r FAST probe of the words k_keyspace_thread could not decide inside
// its tile (an unstaged tile, or the tile's record budget spent), one lane per listed
// word with the word copied to the lane's own LDS slot: the same count walk, mode_unit
// qualification, closed form and plan as there, so a word is FAST (and numbered in FAST
// order) whatever batch it is in.  Records go to slot i of cplx_base; a list longer
// than cplx_cap leaves its tail undecided (count 0) and the host reruns the keyspace
// with room for all (a5x_host.cpp run_keyspace_mode).
__global__ void __launch_bounds__(256) k_keyspace_rprobe(KsArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const u32 tb = (a.table_bytes + 15u) & ~15u;
  u64* gbuf = (u64*)(smem + tb);                           // 256 x KS_GCAP open-group entries
  uint8_t* slots = smem + tb + 256 * KS_GCAP * 8;          // 256 x RP_SLOT word bytes
  load_table(smem, a.table, a.table_bytes);
  __syncthreads();
  const Tab T = tab_view(smem);
  const u32 bmax = T.hdr->max_bucket;
  const u32 tid = threadIdx.x;
  const u32 n = *a.cplx_n;
  for (u32 b0 = blockIdx.x * 256u; b0 < n; b0 += gridDim.x * 256u) {
    const u32 i = b0 + tid;
    const bool valid = i < n && i < a.cplx_cap;
    const u64 w = valid ? a.cplx_list[i] : 0ull;
    const u64 s = valid ? a.woff[w] : 0ull;
    const u32 L = valid ? (u32)(a.woff[w + 1] - s) : 0u;  // <= A5X_LMAX_A (longer words never listed)
    u32* sl = (u32*)(slots + tid * RP_SLOT);
    for (u32 q = 0; q < RP_SLOT / 4; q++) {
      u32 v = 0;
      for (u32 bb = 0; bb < 4; bb++)
        if (4 * q + bb < L) v |= (u32)a.words[s + 4 * q + bb] << (8 * bb);
      sl[q] = v;
    }
    LWord lw;
    lw.base = slots; lw.off = tid * RP_SLOT;
    CountAcc A;
    count_init(A, L);
    NullSink ns;
    Planner<false, LWord, NullSink, KS_GCAP> pl(lw, T, ns);
    bool cplx = false;
    psk_walk<true, false>(lw, L, valid, wave_max_u32(L), bmax, T, pl, A, cplx, a.rmode);
    WordClass C;
    C.flags = 0; C.count = 0; C.bytes = 0; C.ovf = false; C.clusters = false;
    u32 f = 0;
    if (valid && !cplx) {
      pl.finish(L);
      C = classify_finish(A, pl.P, L, a.mn, a.mx, A5X_RING_A - 16);
      f = C.flags;
      if (C.ovf) atomicOr(a.err, A5X_DERR_OVF);
      if ((f & A5X_WF_DEFER) || !(f & (A5X_WF_FAST | A5X_WF_RADIX | A5X_WF_ERR_OVF))) f = A5X_WF_DEFER;
    }
    const u64 cnt = A.P - a.rcmin;
    const bool rf = valid && !cplx && (f & A5X_WF_FAST) && !(f & A5X_WF_DEFER) && A.nunits > 0 && C.count > 0 &&
                    (a.rmode == 1 || cnt <= a.rseg);
    u64* rec = a.rec + a.cplx_base + (u64)i * FW_RMAX;
    {
      DevRecSink sk;
      sk.g = gbuf + tid; sk.c = sk.g; sk.rec = rec; sk.np = ff_np(f);
      Planner<true, LWord, DevRecSink, KS_GCAP> pb(lw, T, sk, rf ? fb_balanced_cap(C.count + 1) : 0u);
      CountAcc A2;
      bool c2 = false;
      psk_walk<false, false>(lw, L, rf, wave_max_u32(rf ? L : 0u), bmax, T, pb, A2, c2, a.rmode);
      if (rf) {
        pb.finish(L);
        pb.pick_balanced();
        const Plan& P = pb.P;
        rec[0] = fr_hdr(P.np, P.ng, P.ne, P.maxl, P.nbig, P.bstarts, P.bRp);
        if (c2 || !P.ok || P.ng != ff_ng(f) || P.ne != ff_ne(f) || P.np != ff_np(f)) atomicOr(a.err, A5X_DERR_STATE);
        a.roff[w] = (u32)(a.cplx_base + (u64)i * FW_RMAX);
      }
    }
    if (valid) {
      a.count[w] = rf ? cnt : 0ull;
      a.bytes[w] = rf ? C.bytes + (a.rcmin ? 0ull : (u64)(L + 1)) : 0ull;
      a.flags[w] = rf ? f : 0u;
      a.rnseg[w] = rf ? (cnt + a.rseg - 1) / a.rseg : 0ull;
    }
    const u32 mi = wave_append(valid && !rf, a.defer_n);  // the mode engine's words
    if (valid && !rf) a.defer_list[mi] = (u32)w;
  }
}

// ---------------------------------------------------------------------------
// -s / -s -r virtual words (processWordSubstituteAll / ...Reverse, main.go:308-440)
// ---------------------------------------------------------------------------
// The probe (mode_unit) refuses a positional word whose patterns repeat: ReplaceAll gives
// every occurrence of a pattern the same value, so those occurrences are one tied digit,
// which the FAST plan (one digit per unit) cannot express.  Fixing the choices of the
// tied patterns splits the word into S = prod R_tied sub-words: sub-word s writes tied
// pattern t's choice d_t (digits of s, first tied pattern least significant; choice 0 =
// the pattern kept, then its values, -s -r: subs[0] only) into the word and keeps the
// once-occurring patterns as units, so it is a plain FAST word.  The word's candidates
// are its sub-words' in order: sub-word 0 (every tied pattern kept) has P - min(min, 1)
// candidates (min 0: FAST index P wraps to the all-keep word), every other sub-word P
// (its all-keep combination of the units still substitutes a tied pattern).  The window
// cuts nothing: min <= 1 (the probe's condition) and #patterns <= max.
// vrec per virtual word: its sub-words' records back to back, then one meta u64 per
// sub-word (count | record u64 << 24 | bytes << 32); roff[w] = their base.
// Two instantiations by lane slot size (odd dword counts: lane slots on distinct LDS banks).
// The small one takes words of <= VS_WSLOT_S - 4 bytes whose sub-words fit VS_SLOT_S - 8
// and hands the rest to the large one (vlong_list); its smaller per-lane LDS admits more
// waves per CU.  Both make the same decision for a word that fits both.
#define VS_SLOT 92   // sub-word bytes per lane (sub-words <= VS_SLOT - 8 bytes; 23 dwords)
#define VS_WSLOT 76  // word bytes per lane (words <= A5X_LMAX_A + over-read; 19 dwords)
#ifndef VS_SLOT_S
#define VS_SLOT_S 52   // small instantiation: sub-words <= 44 bytes (13 dwords)
#endif
#ifndef VS_WSLOT_S
#define VS_WSLOT_S 36  // small instantiation: words <= 32 bytes (9 dwords)
#endif
#define VS_OCC 16    // pattern occurrences per word
#define VS_SMAX 16   // sub-words per word
#define VS_TMAX 4    // tied patterns per word
#ifndef VS_ABL
#define VS_ABL 0     // k_keyspace_vsub timing ablations (variant builds only, wrong output): 1 no build
                     // pass, 2 no count pass, 4 no tasks (walk + pattern analysis only)
#endif
#ifndef VS_GCAP
#define VS_GCAP 4    // entries per open group of the sub-word planner (C5 -s A/B, 4 vs 8 = KS_GCAP:
                     // keyspace 27.1 vs 29.2 ms, the same words split, expansion unchanged; 2: most
                     // words past 8 pieces)
#endif
#ifndef VS_PATCH
#define VS_PATCH 1   // the sub-words of a fixed-width uniform word written without the planner
                     // (0: every sub-word planned, the A/B baseline)
#endif
#define VS_DESC 10   // u64 descriptor of a fixed-width virtual word (k_keyspace_vsub -> k_vwords_fill, FvWord)
#ifndef FV_SLOT
#define FV_SLOT 100  // k_vwords_fill: per-lane sub-word bytes (25 dwords: an odd stride keeps lanes on distinct
                     // banks; 64 / 68 / 100: 5.08 / 4.04 / 3.87 ms on C5 -s); fixed-width words up to FV_SLOT - 8 bytes
#endif
#ifndef VS_BLOCK
#define VS_BLOCK 128 // k_keyspace_vsub workgroup: two waves share the table copy (C5 -s A/B, profiles/r05r_ab_vsub_block_c5.txt:
                     // 16.98 ms vs 17.85 ms at 64, 17.19 at 256)
#endif

struct VsWord {
  u32 L, nocc, nt, S;
  u64 tk;  // tied pattern t's key: bits [10 t, 10 t + 10)
  u32 tr;  // its radix: bits [5 t, 5 t + 5)
};

// Appends bytes to a lane's LDS sub-word slot a dword at a time (pending bytes in acc).
struct SubW {
  u32* d;
  u32 n, na;  // dwords stored, pending bytes
  u64 acc;
  __device__ __forceinline__ u32 len() const { return 4 * n + na; }
  __device__ __forceinline__ void put(u32 v, u32 k) {  // k <= 4 bytes of v
    acc |= (u64)keep_bytes(v, k) << (8 * na);
    na += k;
    if (na >= 4) {
      d[n++] = (u32)acc;
      acc >>= 32;
      na -= 4;
    }
  }
  __device__ __forceinline__ void run(const uint8_t* src, u32 i0, u32 i1) {  // src[i0, i1)
    for (u32 i = i0; i < i1; i += 4) put(lds_ld4(src, i), min(4u, i1 - i));
  }
  __device__ __forceinline__ void sync() { d[n] = (u32)acc; }  // the partial dword readable
};

// Sub-word s of the word at orig (LDS) written to the lane's slot sub; every untied
// occurrence goes to pl (and A) as a unit at its sub-word position.  occ: the word's
// occurrences (q << 10 | key, strided by 256).  Returns the length, 0 when it does not
// fit the slot.
template <u32 SLOT, class PL>
__device__ u32 vs_build(const Tab& T, const VsWord& V, const uint8_t* orig, uint8_t* sub, const uint16_t* occ, u32 s,
                        int rmode, PL& pl, CountAcc& A) {
  u32 ch[VS_TMAX];
  u32 x = s;
#pragma unroll
  for (u32 t = 0; t < VS_TMAX; t++) {
    const u32 R = (V.tr >> (5 * t)) & 31u;
    const u32 key = (u32)(V.tk >> (10 * t)) & 1023u;
    const bool on = t < V.nt;
    const u32 d = on ? x % R : 0u;
    x = on ? x / R : x;
    ch[t] = on ? T.keys[key].choice_base + d : 0u;
  }
  SubW W;
  W.d = (u32*)sub; W.n = 0; W.na = 0; W.acc = 0;
  u32 prev = 0;
  for (u32 j = 0; j < V.nocc; j++) {
    const u32 e = occ[j * VS_BLOCK];
    const u32 q = e >> 10, key = e & 1023u;
    if (W.len() + (q - prev) + 16u > SLOT - 8u) return 0;  // (values <= 15 bytes)
    W.run(orig, prev, q);
    u32 ci = ~0u;
#pragma unroll
    for (u32 t = 0; t < VS_TMAX; t++)
      if (t < V.nt && ((u32)(V.tk >> (10 * t)) & 1023u) == key) ci = ch[t];
    u32 kl;
    if (ci == ~0u) {  // a once-occurring pattern: a unit of the sub-word
      Unit U;
      lone_unit(T, W.len(), key, U);
      kl = U.e - U.s;
      u64 seen = 0;
      (void)mode_unit(T, U, rmode, seen, false);
      count_unit(A, U);
      W.sync();
      pl.unit(U);
      W.put(lds_ld4(orig, q), kl);  // (keys <= 4 bytes)
    } else {
      kl = T.keys[key].klen;
      const u64 cv = T.cval[ci];
      const u32 cl = (u32)(cv >> 56);
      if (cl <= 7) {
        W.put((u32)cv, min(4u, cl));
        if (cl > 4) W.put((u32)(cv >> 32), cl - 4);
      } else {
        const A5xChoice c = T.ch[ci];
        W.put(c.first4, 4);
        for (u32 i = 4; i < c.len; i++) W.put(T.blob[c.blob_off + i], 1);
      }
    }
    prev = q + kl;
  }
  if (W.len() + (V.L - prev) > SLOT - 8u) return 0;
  W.run(orig, prev, V.L);
  W.sync();
  return W.len();
}

// classify_finish's FAST conditions for a sub-word; its count (cmin: the all-keep word
// cut, sub-word 0 with min >= 1), bytes and record size (0 without candidates)
__device__ __forceinline__ bool vs_fast(const CountAcc& A, const Plan& PL, u32 Ls, u32 cmin, u32& rs, u64& cnt,
                                        u64& byt) {
  if (!A.ok || A.ovf || !PL.ok) return false;
  if (!(PL.np <= FW_PMAX && PL.ne <= 255 && 1 + PL.np + PL.ne <= FW_RMAX && PL.maxl <= FW_MAXL && PL.minl >= 3 &&
        A.P < FW_PMAX_CNT && PL.nbig <= FB_NMAX && PL.bent <= FB_EMAX))
    return false;  // (A.P < 2^24: the sub-word's meta entry packs its count into 24 bits)
  cnt = A.P - cmin;
  byt = A.P * (u64)(Ls + 1) + A.Dp - A.Dn - (cmin ? (u64)(Ls + 1) : 0ull);
  rs = cnt ? 1u + PL.np + PL.ne : 0u;
  return true;
}

// The word (lane l of the wave) that owns task t of the wave: the largest l with
// tbase[l] <= t (tbase: exclusive scan of the sub-word counts, 64 entries)
__device__ __forceinline__ u32 vs_owner(const uint16_t* tbase, u32 t) {
  u32 l = 0;
#pragma unroll
  for (u32 st = 32; st; st >>= 1)
    if (tbase[l + st] <= t) l += st;
  return l;
}

// Lane per word of the probe's list (defer_list): the word's occurrences and tied
// patterns; then its sub-words as tasks spread over the wave's lanes (a word's S
// sub-words do not serialise its lane): count pass (per-word sums by LDS atomics), one
// bump allocation per wave, build pass writing the records and metas.  The words it
// cannot split go to vout_list (the mode engine).  A vrec too small leaves the words past
// it undecided (the host reruns the keyspace with room for all).
struct VsWave {  // per-wave LDS state
  uint16_t tbase[65];                 // first task of each lane's word (+ total)
  uint16_t tcbase[65];                // the same for the count pass (uniform words: sub-word 0 only)
  u32 u0[64];                         // uniform word: sub-word 0's pieces | record u64 << 8 | length << 16
  u32 uP[64];                         // ... and its combinations P
  uint16_t tinfo[64 * VS_SMAX];       // per task: pieces | record u64 << 4 (0: none)
  u32 ctot[64], btot[64], rtot[64], bad[64];
  uint4 info[64];                     // word: L | nocc << 8 | nt << 16 | S << 24, tr, tk
  unsigned long long base[64];
  uint16_t tbb[65];                   // first build task (the planner) of each lane's word (+ total)
  u64 upst[64];                       // uniform word: sub-word 0's piece starts (Planner::pst)
  u64 uhdr[64];                       // ... its record header
  u32 ub0[64];                        // ... and the bytes of each other sub-word
};

// Record sink of the build pass: the open group in LDS (lane-strided by VS_BLOCK),
// descriptors and entries straight to the record in HBM (DevRecSink's layout).
struct VsRecSink {
  u64* g;
  u64* rec;
  u32 np;
  __device__ u64* cbuf() const { return nullptr; }  // (no clusters: lone units only)
  __device__ u32 cstride() const { return 1; }
  __device__ u64 gld(u32, u32 a) const { return g[a * VS_BLOCK]; }
  __device__ void gst(u32, u32 a, u64 v) { g[a * VS_BLOCK] = v; }
  __device__ void ent(u32 i, u64 v) { rec[1 + np + i] = v; }
  __device__ void desc(u32 i, u64 v) { rec[1 + i] = v; }
};

#ifndef VS_WPE
#define VS_WPE 3  // waves per SIMD the register budget is cut for (LDS admits ~7 one-wave workgroups per CU)
#endif
template <u32 WSLOT, u32 SLOT, bool SMALL>
__global__ void __launch_bounds__(VS_BLOCK) __attribute__((amdgpu_waves_per_eu(VS_WPE))) k_keyspace_vsub(KsArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const u32 tb = (a.table_bytes + 15u) & ~15u;
  u64* gbuf = (u64*)(smem + tb);                                 // VS_BLOCK x VS_GCAP open-group entries
  uint8_t* wsl = smem + tb + VS_BLOCK * VS_GCAP * 8;             // VS_BLOCK x WSLOT word bytes
  uint8_t* ssl = wsl + VS_BLOCK * WSLOT;                         // VS_BLOCK x SLOT sub-word bytes
  uint16_t* occ0 = (uint16_t*)(ssl + VS_BLOCK * SLOT);           // VS_OCC x VS_BLOCK occurrences
  VsWave* wvs = (VsWave*)(occ0 + VS_BLOCK * VS_OCC);             // one per wave
  load_table(smem, a.table, a.table_bytes);
  __syncthreads();
  const Tab T = tab_view(smem);
  const u32 tid = threadIdx.x, lane = lane_id(), wv = tid / 64;
  VsWave& Q = wvs[wv];
  const u32 n = *a.defer_n;
  const u32 pbit = a.rmode == 2 ? 1u : 2u;
  uint8_t* orig = wsl + tid * WSLOT;
  uint16_t* occ = occ0 + tid;
  uint8_t* sub = ssl + tid * SLOT;
  LWord lw;
  lw.base = ssl; lw.off = tid * SLOT;
  for (u32 b0 = blockIdx.x * VS_BLOCK; b0 < n; b0 += gridDim.x * VS_BLOCK) {
    // ---- word lane: occurrences, tied patterns ----
    const u32 i = b0 + tid;
    const bool valid = i < n;
    const u64 w = valid ? a.defer_list[i] : 0ull;
    const u64 s0 = valid ? a.woff[w] : 0ull;
    const u64 L64 = valid ? a.woff[w + 1] - s0 : 0ull;
    bool ok = valid && L64 >= 1 && L64 <= A5X_LMAX_A;
    const bool lngw = SMALL && ok && L64 > WSLOT - 4u;  // too long for this instantiation's slots
    ok = ok && !lngw;
    VsWord V;
    V.L = ok ? (u32)L64 : 0u; V.nocc = 0; V.nt = 0; V.S = 1; V.tk = 0; V.tr = 0;
    {
      // aligned dwords of the word (the batch's words buffer has 16 readable bytes past
      // the last word), shifted into place; zero past the word
      u32* sl = (u32*)orig;
      const u32* src = (const u32*)(a.words + (s0 & ~3ull));
      const u32 sh = (u32)(s0 & 3u), nd = (V.L + 3u) / 4u;
      u32 lo = V.L ? src[0] : 0u;
      for (u32 q = 0; q < WSLOT / 4; q++) {
        const u32 hi = q < nd ? src[q + 1] : 0u;
        const u32 v = __builtin_amdgcn_alignbyte(hi, lo, sh);
        sl[q] = 4 * q + 4 <= V.L ? v : (4 * q < V.L ? keep_bytes(v, V.L - 4 * q) : 0u);
        lo = hi;
      }
    }
    // occurrences: the probe's row (k_keyspace_thread logged the word's lone matches),
    // else the walk -- lone matches of positional patterns (as psk_walk: two keys at one
    // position, a match inside another, a key longer than 4 bytes -> not split)
    u32 rcnt = 0xFFFFu;
    uint4 r0 = make_uint4(0, 0, 0, 0), r1 = r0;
    if (ok && a.vocc) {
      const uint4* row = (const uint4*)(a.vocc + w * 16);
      r0 = row[0];
      r1 = row[1];
      rcnt = r1.w >> 16;
    }
    if (ok && rcnt != 0xFFFFu) {
      const u32 rw[8] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
#pragma unroll
      for (u32 j = 0; j < 15; j++)
        if (j < rcnt) occ[j * VS_BLOCK] = (uint16_t)(rw[j / 2] >> (16 * (j & 1)));
      V.nocc = rcnt;
    }
    u32 cur_end = 0;
    bool walk = ok && rcnt == 0xFFFFu;
    for (u32 q = 0; walk && q < V.L; q++) {
      const u32 w4 = lds_ld4(orig, q);
      const u32 bk = T.bucket2[w4 & 255u];
      const u32 ks = bk & 0xFFFFu, ke = bk >> 16;
      u32 nm = 0, kk = 0;
      for (u32 k2 = ks; k2 < ke; k2++) {
        const u64 km = T.kmatch[k2];
        const u32 kl = (u32)(km >> 32) & 0xFFFFu;
        if (q + kl > V.L) continue;
        if (kl > 4) { ok = false; break; }
        const u32 m = kl >= 4 ? 0xFFFFFFFFu : ((1u << (8 * kl)) - 1u);
        if ((w4 & m) == (u32)km) { nm++; kk = k2; }
      }
      if (!ok) break;
      if (nm > 1 || (nm == 1 && q < cur_end)) { ok = false; break; }
      if (nm == 1) {
        const A5xKey key = T.keys[kk];
        if (!(key.pad0 & pbit) || key.nvals < 1 || V.nocc >= VS_OCC || kk >= 1024u || q >= 64u) { ok = false; break; }
        occ[V.nocc * VS_BLOCK] = (uint16_t)((q << 10) | kk);
        V.nocc++;
        cur_end = q + key.klen;
      }
    }
    // patterns (distinct keys); the tied ones (>= 2 occurrences) in first-occurrence order
    u32 npat = 0;
    for (u32 j = 0; ok && j < V.nocc; j++) {
      const u32 kj = occ[j * VS_BLOCK] & 1023u;
      bool first = true;
      u32 mult = 0;
      for (u32 j2 = 0; j2 < V.nocc; j2++) {
        const u32 k2 = occ[j2 * VS_BLOCK] & 1023u;
        if (k2 == kj) { mult++; first = first && j2 >= j; }
      }
      if (!first) continue;
      npat++;
      if (mult >= 2) {
        const u32 R = a.rmode == 2 ? (u32)T.keys[kj].nvals + 1u : 2u;
        if (V.nt >= VS_TMAX || V.S * R > VS_SMAX) { ok = false; break; }
        V.tk |= (u64)kj << (10 * V.nt);
        V.tr |= R << (5 * V.nt);
        V.nt++;
        V.S *= R;
      }
    }
    ok = ok && npat >= 1 && (i64)npat <= (i64)a.mx && !(VS_ABL & 4);
    // uniform: every choice of every tied pattern as long as the pattern, so all sub-words
    // share one layout -- the count pass plans sub-word 0 only
    bool uni = true;
#pragma unroll
    for (u32 t = 0; t < VS_TMAX; t++) {
      if (t < V.nt) {
        const A5xKey key = T.keys[(u32)(V.tk >> (10 * t)) & 1023u];
        uni = uni && (a.rmode == 2 ? key.minclen == key.maxclen : T.ch[key.choice_base + 1].len == key.klen);
      }
    }
    // fixed width: every pattern of the word (units and tied) has all its choices as long as
    // itself, so an entry's byte j is word byte (piece start + j) in every sub-word, and every
    // sub-word's record follows from sub-word 0's pieces (the fixed pass)
    bool fixed = VS_PATCH && ok && uni && V.L + 8u <= FV_SLOT;
    for (u32 j = 0; fixed && j < V.nocc; j++) {
      const A5xKey key = T.keys[occ[j * VS_BLOCK] & 1023u];
      fixed = key.nvals >= 1 &&
              (a.rmode == 2 ? key.minclen == key.maxclen : T.ch[key.choice_base + 1].len == key.klen);
    }
    // ---- the wave's task lists: word lane l owns tasks [tbase[l], tbase[l] + S) ----
    const u32 Sl = ok ? V.S : 0u, Sc = ok ? (uni ? 1u : V.S) : 0u;
    const u32 tinc = wave_incl_scan_u32(Sl), tcinc = wave_incl_scan_u32(Sc);
    const u32 ntask = readlane_u32(tinc, 63), nctask = readlane_u32(tcinc, 63);
    Q.tbase[lane] = (uint16_t)(tinc - Sl);
    Q.tcbase[lane] = (uint16_t)(tcinc - Sc);
    if (lane == 63) { Q.tbase[64] = (uint16_t)ntask; Q.tcbase[64] = (uint16_t)nctask; }
    Q.ctot[lane] = 0; Q.btot[lane] = 0; Q.rtot[lane] = 0; Q.bad[lane] = 0;
    Q.info[lane] = make_uint4(V.L | (V.nocc << 8) | (V.nt << 16) | (V.S << 24), V.tr, (u32)V.tk, (u32)(V.tk >> 32));
    WAVE_SYNC();
    auto task_word = [&](const uint16_t* base, u32 t, VsWord& W, u32& l, u32& s) {
      l = vs_owner(base, t);
      s = t - base[l];
      const uint4 in = Q.info[l];
      W.L = in.x & 255u; W.nocc = (in.x >> 8) & 255u; W.nt = (in.x >> 16) & 255u; W.S = in.x >> 24;
      W.tr = in.y; W.tk = (u64)in.z | ((u64)in.w << 32);
    };
    const u32 cmin = a.rcmin;
    // ---- count pass: every sub-word FAST; sizes summed per word ----
    for (u32 t0 = 0; t0 < nctask; t0 += 64) {
      const u32 t = t0 + lane;
      if (t < nctask && (VS_ABL & 2)) {
        u32 l, s;
        VsWord W;
        task_word(Q.tcbase, t, W, l, s);
        Q.tinfo[Q.tbase[l] + s] = 0;
        atomicAdd(&Q.ctot[l], 1u);
      } else if (t < nctask) {
        VsWord W;
        u32 l, s;
        task_word(Q.tcbase, t, W, l, s);
        const u32 wl = wv * 64 + l;
        CountAcc A;
        count_init(A, 0);
        NullSink ns;
        Planner<false, LWord, NullSink, VS_GCAP> pl(lw, T, ns);
        const u32 Ls = vs_build<SLOT>(T, W, wsl + wl * WSLOT, sub, occ0 + wl, s, a.rmode, pl, A);
        u32 rs = 0;
        u64 cnt = 0, byt = 0;
        bool f = Ls != 0;
        if (f) {
          pl.finish(Ls);
          f = vs_fast(A, pl.P, Ls, s == 0 ? cmin : 0u, rs, cnt, byt);
        }
        Q.tinfo[Q.tbase[l] + s] = (uint16_t)(f && rs ? pl.P.np | (rs << 4) : 0u);
        if (s == 0) {
          const u32 rfull = 1u + pl.P.np + pl.P.ne;  // (the record of a sub-word with candidates)
          Q.u0[l] = pl.P.np | (min(rfull, 255u) << 8) | (Ls << 16);
          Q.uP[l] = (u32)min(A.P, (u64)0xFFFFFFFFu);
          Q.upst[l] = pl.pst;
          Q.uhdr[l] = fr_hdr(pl.P.np, pl.P.ng, pl.P.ne, pl.P.maxl, pl.P.nbig, pl.P.bstarts, pl.P.bRp);
        }
        if (!f) atomicOr(&Q.bad[l], Ls ? 1u : 2u);  // (2: a sub-word past the lane slot)
        else {
          atomicAdd(&Q.ctot[l], (u32)min(cnt, (u64)0xFFFFFFFFu));
          atomicAdd(&Q.btot[l], (u32)min(byt, (u64)0xFFFFFFFFu));
          atomicAdd(&Q.rtot[l], rs);
        }
      }
    }
    WAVE_SYNC();
    // ---- word lane: the decision, one bump allocation per wave ----
    u32 ctot = Q.ctot[lane], btot = Q.btot[lane], rtot = Q.rtot[lane];
    bool patch = false;
    if (ok && uni && V.S > 1 && !Q.bad[lane]) {
      // sub-words 1 .. S-1 of a uniform word: sub-word 0's layout with every combination
      const u32 u0 = Q.u0[lane], P = Q.uP[lane], np = u0 & 255u, rfull = (u0 >> 8) & 255u, Ls = u0 >> 16;
      const u32 b0 = btot + (cmin ? Ls + 1u : 0u);  // sub-word 0's bytes + its cut all-keep word
      ctot += (V.S - 1u) * P;
      btot += (V.S - 1u) * b0;
      rtot += (V.S - 1u) * rfull;
      for (u32 s = 1; s < V.S; s++) Q.tinfo[Q.tbase[lane] + s] = (uint16_t)(np | (rfull << 4));
      Q.ub0[lane] = b0;
      patch = fixed && (Q.tinfo[Q.tbase[lane]] >> 4) == rfull;  // (sub-word 0 has candidates)
    }

    const bool lngs = SMALL && ok && (Q.bad[lane] & 2u);  // a sub-word past the small slot: the large one decides
    ok = ok && !Q.bad[lane] && ctot >= 1 && ctot <= a.rseg;  // (one mode-engine item, as the probe's -s words)
    patch = patch && ok;
    const u32 mtot = ok ? (patch ? VS_DESC : rtot + V.S) : 0u;  // (a fixed-width word: its descriptor)
    const u32 minc = wave_incl_scan_u32(mtot);
    unsigned long long wbase = 0;
    if (lane == 63 && minc) wbase = atomicAdd(a.vrec_n, (unsigned long long)minc);
    const unsigned long long base = readlane_u64((u64)wbase, 63) + (minc - mtot);
    const bool room = ok && base + mtot <= a.vrec_cap;
    Q.base[lane] = room ? base : ~0ull;
    Q.rtot[lane] = rtot;
    // the build tasks (the planner); a fixed-width word's sub-words are written by k_vwords_fill
    // from its descriptor, straight into the virtual word list's record area
    patch = patch && room;
    const u32 Sb = room && !patch ? V.S : 0u;
    const u32 binc = wave_incl_scan_u32(Sb);
    const u32 nbtask = readlane_u32(binc, 63);
    Q.tbb[lane] = (uint16_t)(binc - Sb);
    if (lane == 63) Q.tbb[64] = (uint16_t)nbtask;
    if (patch) {
      u32 tb = 0, ts = 0;
      u64 oc[4] = {0, 0, 0, 0};
      for (u32 j = 0; j < V.nocc; j++) {
        const u32 e = occ[j * VS_BLOCK], key = e & 1023u;
#pragma unroll
        for (u32 tt = 0; tt < VS_TMAX; tt++)
          if (tt < V.nt && ((u32)(V.tk >> (10 * tt)) & 1023u) == key) { tb |= 1u << j; ts |= tt << (2 * j); }
#pragma unroll
        for (u32 k = 0; k < 4; k++)
          if (j / 4u == k) oc[k] |= (u64)e << (16 * (j & 3u));
      }
      const u32 u0 = Q.u0[lane];
      u64* d = a.vrec + base;
      d[0] = Q.uhdr[lane];
      d[1] = Q.upst[lane];
      d[2] = V.tk | ((u64)V.nt << 40) | ((u64)V.S << 44) | ((u64)V.L << 49) | ((u64)(u0 & 15u) << 56);
      d[3] = (u64)V.tr | ((u64)((u0 >> 8) & 255u) << 20) | ((u64)V.nocc << 28);
      d[4] = (u64)Q.uP[lane] | ((u64)Q.ub0[lane] << 32);
      d[5] = (u64)tb | ((u64)ts << 16);
#pragma unroll
      for (u32 k = 0; k < 4; k++) d[6 + k] = oc[k];
    }
    WAVE_SYNC();
    // ---- build pass: records and metas at the word's base ----
    for (u32 t0 = 0; t0 < nbtask; t0 += 64) {
      const u32 t = t0 + lane;
      if (t < nbtask) {
        VsWord W;
        u32 l, s;
        task_word(Q.tbb, t, W, l, s);
        const u32 ts = Q.tbase[l] + s;  // (the sub-word's task in the record layout)
        const unsigned long long wb = Q.base[l];
        if (wb != ~0ull && !(VS_ABL & 1)) {
          const u32 wl = wv * 64 + l;
          u32 ro = 0;
          for (u32 t2 = Q.tbase[l]; t2 < ts; t2++) ro += Q.tinfo[t2] >> 4;
          const u32 ti = Q.tinfo[ts], np = ti & 15u, rs0 = ti >> 4;
          u64* rb = a.vrec + wb;
          u32 rs = 0;
          u64 cnt = 0, byt = 0;
          if (np) {
            VsRecSink sk;
            sk.g = gbuf + tid; sk.rec = rb + ro; sk.np = np;
            // (greedy big pieces: balanced ones as k_keyspace_thread builds measured +-0 here,
            // profiles/r05g_ab_mode_items_grid_c5.txt -- sub-words rarely pass 64 combinations)
            Planner<true, LWord, VsRecSink, VS_GCAP> pb(lw, T, sk, 0u);
            CountAcc A;
            count_init(A, 0);
            const u32 Ls = vs_build<SLOT>(T, W, wsl + wl * WSLOT, sub, occ0 + wl, s, a.rmode, pb, A);
            pb.finish(Ls);
            const Plan& P = pb.P;
            if (!Ls || !vs_fast(A, P, Ls, s == 0 ? cmin : 0u, rs, cnt, byt) || P.np != np || rs != rs0)
              atomicOr(a.err, A5X_DERR_STATE);
            rb[ro] = fr_hdr(P.np, P.ng, P.ne, P.maxl, P.nbig, P.bstarts, P.bRp);
          }
          rb[Q.rtot[l] + s] = cnt | ((u64)rs << 24) | (byt << 32);
        }
      }
    }
    // ---- word lane: results ----
    if (room) {
      a.count[w] = ctot;
      a.bytes[w] = btot;
      a.flags[w] = A5X_WF_FAST | A5X_WF_VIRT | (patch ? A5X_WF_VFIX : 0u);
      a.rnseg[w] = 1;
      a.roff[w] = (u32)base;
      a.vn[w] = V.S - 1u;
      a.vrsz[w] = rtot;
    }
    const bool lng = lngw || lngs;
    const bool left = valid && !ok && !lng;  // (ok without room: undecided, the host reruns)
    const u32 mi = wave_append(left, a.vout_n);
    if (left) a.vout_list[mi] = (u32)w;
    if (SMALL) {
      const u32 li = wave_append(lng, a.vlong_n);
      if (lng) a.vlong_list[li] = (u32)w;
    }
    WAVE_SYNC();  // (Q is rewritten by the next words)
  }
}

// k_expand_fast over a batch with virtual words runs on the virtual word list: every word
// one entry (mode-engine words as holes, flags 0), a virtual word one entry per sub-word;
// records in one area in list order (each window one contiguous copy).
struct VwArgs {
  const u32* flags;
  const u64* cand_off;
  const u64* byte_off;  // (null: the fused digest, no layout)
  const u32* roff;
  const u64* rec;
  const u64* vrec;
  const u64* vpre;   // exclusive scan of vn: entry of word w = w + vpre[w]
  const u64* vrpre;  // exclusive scan of vrsz: record u64 of word w in vrec2
  u64 nw;
  u64* vcand_off;
  u64* vbyte_off;
  u32* vflags;
  u32* vroff;
  u32* vmap;    // entry -> word
  u32* vobase;  // entry -> its first candidate's index in the word
  u64* vrec2;
  // fixed-width virtual words (A5X_WF_VFIX): the table and the words
  const uint8_t* table;
  u32 table_bytes;
  int rmode;
  u32 rcmin;
  const uint8_t* words;
  const u64* woff;
};

// record u64 of the words that are not virtual (virtual words: k_keyspace_vsub)
__global__ void __launch_bounds__(256) k_vwords_sizes(const u32* flags, const u64* cand_off, u64 nw, u64* vn,
                                                      u64* vrsz) {
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 w = (u64)blockIdx.x * blockDim.x + threadIdx.x; w < nw; w += stride) {
    const u32 f = flags[w];
    if (f & A5X_WF_VIRT) continue;
    vn[w] = 0;
    vrsz[w] = (f & A5X_WF_FAST) && cand_off[w + 1] > cand_off[w] ? ff_rsize(f) : 0ull;
  }
}

// A fixed-width virtual word (k_keyspace_vsub's descriptor d, VS_DESC u64): d0 the sub-words'
// record header, d1 their piece starts (7 bits each), d2 tk | nt << 40 | S << 44 | L << 49 |
// np << 56, d3 tr | rfull << 20 | nocc << 28, d4 P | (bytes of a sub-word s >= 1) << 32, d5 tied
// occurrences (bit j) | their tied pattern << 16 (2 bits each), d6..d9 the occurrences (u16 q << 10 | key).
struct FvWord {
  u64 hdr, pst, tk;
  u32 nt, S, L, np, tr, rfull, nocc, P, b0, tbits, tsel;
  u64 oc0, oc1, oc2, oc3;  // (named, not an array: a dynamic index would put the struct in scratch)
  __device__ __forceinline__ void load(const u64* d) {
    hdr = d[0]; pst = d[1];
    const u64 d2 = d[2], d3 = d[3], d4 = d[4], d5 = d[5];
    tk = d2 & 0xFFFFFFFFFFull; nt = (u32)(d2 >> 40) & 7u; S = (u32)(d2 >> 44) & 31u; L = (u32)(d2 >> 49) & 127u;
    np = (u32)(d2 >> 56) & 15u;
    tr = (u32)d3 & 0xFFFFFu; rfull = (u32)(d3 >> 20) & 255u; nocc = (u32)(d3 >> 28) & 31u;
    P = (u32)d4; b0 = (u32)(d4 >> 32);
    tbits = (u32)d5 & 0xFFFFu; tsel = (u32)(d5 >> 16);
    oc0 = d[6]; oc1 = d[7]; oc2 = d[8]; oc3 = d[9];
  }
  __device__ __forceinline__ u32 oc(u32 j) const {
    const u32 k = j >> 2;  // (value masks, not a select of members: that becomes a dynamic index)
    const u64 o = (oc0 & (0ull - (u64)(k == 0))) | (oc1 & (0ull - (u64)(k == 1))) | (oc2 & (0ull - (u64)(k == 2))) |
                  (oc3 & (0ull - (u64)(k == 3)));
    return (u32)(o >> (16 * (j & 3u))) & 0xFFFFu;
  }
};

// Sub-word s's record of a fixed-width word at rd.  Its pieces are sub-word 0's (the count pass
// planned it) and every choice is as long as its pattern, so piece p's entry a is the sub-word's
// bytes [pst_p, pst_p + len_p) (tied choices in, '\n' at L) with each of the piece's units (at
// most two: R_p <= VS_GCAP) at a nonzero digit of a (first unit least significant) XORed from
// its key to that choice -- the planner's entry, descriptor and meta.  sub: FV_SLOT bytes of LDS;
// wd: the word's bytes (global).
static_assert(VS_GCAP <= 4, "fixed-width sub-words: at most two units per piece");
__device__ __forceinline__ void fv_subword(const Tab& T, const FvWord& F, const uint8_t* wd, u32 s, int rmode, uint8_t* sub, u64* rd) {
  // the tied patterns' choices (digits of s, first tied pattern least significant; s < 16)
  u32 ch0 = 0, ch1 = 0, ch2 = 0, ch3 = 0;
  {
    u32 x = s;
#pragma unroll
    for (u32 tt = 0; tt < VS_TMAX; tt++) {
      const u32 R = tt < F.nt ? (F.tr >> (5 * tt)) & 31u : 1u;
      const u32 q = (u32)((float)x * __builtin_amdgcn_rcpf((float)R) + 0.03125f);  // (x < 16: exact)
      const u32 c = T.keys[(u32)(F.tk >> (10 * tt)) & 1023u].choice_base + (x - q * R);
      x = q;
      if (tt == 0) ch0 = c; else if (tt == 1) ch1 = c; else if (tt == 2) ch2 = c; else ch3 = c;
    }
  }
  // the word's bytes (aligned dwords, shifted into place; the words buffer has 16 readable
  // bytes past the last word), tied choices written over their occurrences, '\n' at L
  u32* sd = (u32*)sub;
  {
    const u64 a0 = (u64)wd;
    const u32* src = (const u32*)(a0 & ~3ull);
    const u32 sh = (u32)(a0 & 3u), nd = F.L / 4u + 1u;
    u32 lo = src[0];
    for (u32 q = 0; q < nd; q++) {
      const u32 hi = src[q + 1];
      sd[q] = __builtin_amdgcn_alignbyte(hi, lo, sh);
      lo = hi;
    }
  }
  for (u32 tb = F.tbits; tb; tb &= tb - 1u) {
    const u32 j = __builtin_ctz(tb), tt = (F.tsel >> (2 * j)) & 3u;
    const u32 e = F.oc(j), q = e >> 10, key = e & 1023u;
    const u32 ci = tt == 0 ? ch0 : tt == 1 ? ch1 : tt == 2 ? ch2 : ch3;
    if (ci == T.keys[key].choice_base) continue;  // (choice 0: the pattern itself)
    const u32 kl = T.keys[key].klen, sh = 8u * (q & 3u);  // (kl <= 4)
    const u64 msk = (((1ull << (8 * kl)) - 1ull) << sh), cv = (u64)(u32)T.cval[ci] << sh;
    const u32 w0 = sd[q / 4u], w1 = sd[q / 4u + 1u];
    const u64 nv = ((((u64)w1 << 32) | w0) & ~msk) | (cv & msk);
    sd[q / 4u] = (u32)nv;
    sd[q / 4u + 1u] = (u32)(nv >> 32);
  }
  sub[F.L] = (uint8_t)10;
  rd[0] = F.hdr;
  u32 j = 0, eb = 0;
  for (u32 p = 0; p < F.np; p++) {
    const u32 ps = (u32)(F.pst >> (7 * p)) & 127u;
    const u32 pe = p + 1 < F.np ? (u32)(F.pst >> (7 * (p + 1))) & 127u : F.L + 1u;
    const u64 lm = (1ull << (8 * (pe - ps))) - 1ull;  // (len <= 7)
    const u64 base = ((u64)lds_ld4(sub, ps) | ((u64)lds_ld4(sub, ps + 4u) << 32)) & lm;
    // the piece's units: the untied occurrences in [ps, pe)
    u32 nu = 0, R0 = 1, R1 = 1, o0 = 0, o1 = 0, c0 = 0, c1 = 0;
    for (; j < F.nocc; j++) {
      const u32 e = F.oc(j), q = e >> 10;
      if (q >= pe) break;
      if ((F.tbits >> j) & 1u) continue;
      const A5xKey K = T.keys[e & 1023u];
      const u32 R = rmode == 2 ? (u32)K.nvals + 1u : 2u;
      if (nu == 0) { R0 = R; o0 = 8u * (q - ps); c0 = K.choice_base; }
      else { R1 = R; o1 = 8u * (q - ps); c1 = K.choice_base; }
      nu++;
    }
    const u32 R = R0 * R1;
    rd[1 + p] = fr_desc(R, eb);
    const u64 meta = fw_meta(pe - ps, R);
    const u32 k0 = (u32)T.cval[c0], k1 = (u32)T.cval[c1];
    u64* re = rd + 1 + F.np + eb;
    for (u32 d1 = 0; d1 < R1; d1++) {
      const u64 v1 = d1 ? base ^ ((u64)(k1 ^ (u32)T.cval[c1 + d1]) << o1) : base;
      for (u32 d0 = 0; d0 < R0; d0++) {
        const u64 v = d0 ? v1 ^ ((u64)(k0 ^ (u32)T.cval[c0 + d0]) << o0) : v1;
        re[d1 * R0 + d0] = (v & lm) | meta;
      }
    }
    eb += R;
  }
}

struct FvWave {
  uint16_t tb[65];  // first fixed-width sub-word task of each lane's word (+ total)
  u32 d[64];        // its descriptor (vrec offset)
  unsigned long long r0[64];  // its first record u64 in vrec2
  unsigned long long ws[64];  // its first byte in the words buffer
};
static size_t vwords_fill_lds(u32 table_bytes) { return ((table_bytes + 15u) & ~15u) + 256 * FV_SLOT + 4 * sizeof(FvWave); }

__global__ void __launch_bounds__(256) k_vwords_fill(VwArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const u32 tbytes = (a.table_bytes + 15u) & ~15u;
  if (a.table) load_table(smem, a.table, a.table_bytes);
  __syncthreads();
  const Tab T = tab_view(smem);
  uint8_t* sub = smem + tbytes + threadIdx.x * FV_SLOT;
  FvWave& Q = ((FvWave*)(smem + tbytes + 256 * FV_SLOT))[threadIdx.x / 64];
  const u32 lane = lane_id();
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 wb = (u64)blockIdx.x * blockDim.x + (threadIdx.x & ~63u); wb < a.nw; wb += stride) {
    const u64 w = wb + lane;
    const bool valid = w < a.nw;
    const u32 f = valid ? a.flags[w] : 0u;
    const u64 v0 = valid ? w + a.vpre[w] : 0ull, r0 = valid ? a.vrpre[w] : 0ull;
    const u64 c0 = valid ? a.cand_off[w] : 0ull, b0 = valid && a.byte_off ? a.byte_off[w] : 0ull;
    u32 nrec = valid ? (u32)(a.vrpre[w + 1] - r0) : 0u;
    const bool fix = valid && (f & A5X_WF_VFIX);
    u64 src = 0;  // (address of the word's records)
    if (valid && !(f & A5X_WF_VIRT)) {
      a.vcand_off[v0] = c0; a.vbyte_off[v0] = b0; a.vflags[v0] = nrec ? f : 0u; a.vroff[v0] = (u32)r0;
      a.vmap[v0] = (u32)w; a.vobase[v0] = 0;
      if (nrec) src = (u64)(a.rec + a.roff[w]);
    } else if (fix) {
      // every sub-word: the same layout; sub-word 0 without the all-keep word when min >= 1
      const u64* d = a.vrec + a.roff[w];
      const u64 hdr = d[0], d2 = d[2], d3 = d[3], d4 = d[4];
      const u32 S = (u32)(d2 >> 44) & 31u, Ls1 = ((u32)(d2 >> 49) & 127u) + 1u, rs = (u32)(d3 >> 20) & 255u;
      const u32 P = (u32)d4, bs = (u32)(d4 >> 32);
      const u32 vf = A5X_WF_FAST | A5X_WF_RADIX | (frh_ng(hdr) << 10) | (frh_ne(hdr) << 16) | (frh_np(hdr) << 24);
      u64 co = 0, bo = 0;
      for (u32 s = 0; s < S; s++) {
        const u64 v = v0 + s;
        a.vcand_off[v] = c0 + co; a.vbyte_off[v] = b0 + bo; a.vflags[v] = vf; a.vroff[v] = (u32)(r0 + (u64)s * rs);
        a.vmap[v] = (u32)w; a.vobase[v] = (u32)co;
        const u32 cut = s == 0 ? a.rcmin : 0u;
        co += P - cut; bo += bs - (cut ? Ls1 : 0u);
      }
      nrec = 0;  // (written below, not copied)
    } else if (valid) {
      const u64* vr = a.vrec + a.roff[w];
      src = (u64)vr;
      const u32 S = (u32)(a.vpre[w + 1] - a.vpre[w]) + 1u;
      u64 co = 0, bo = 0;
      u32 ro = 0;
      for (u32 s = 0; s < S; s++) {
        const u64 m = vr[nrec + s];
        const u32 cnt = (u32)m & 0xFFFFFFu, rs = (u32)(m >> 24) & 255u;
        u32 vf = 0;
        if (rs) {
          const u64 h = vr[ro];
          vf = A5X_WF_FAST | A5X_WF_RADIX | (frh_ng(h) << 10) | (frh_ne(h) << 16) | (frh_np(h) << 24);
        }
        const u64 v = v0 + s;
        a.vcand_off[v] = c0 + co; a.vbyte_off[v] = b0 + bo; a.vflags[v] = vf; a.vroff[v] = (u32)(r0 + ro);
        a.vmap[v] = (u32)w; a.vobase[v] = (u32)co;
        co += cnt; bo += m >> 32; ro += rs;
      }
    }
    if (valid && w + 1 == a.nw) {
      const u64 ve = a.nw + a.vpre[a.nw];
      a.vcand_off[ve] = a.cand_off[a.nw];
      a.vbyte_off[ve] = a.byte_off ? a.byte_off[a.nw] : 0ull;
    }
    // the fixed-width words' sub-words as tasks over the wave's lanes
    const u32 Sf = fix ? (u32)(a.vpre[w + 1] - a.vpre[w]) + 1u : 0u;
    const u32 finc = wave_incl_scan_u32(Sf), nft = readlane_u32(finc, 63);
    if (nft) {
      Q.tb[lane] = (uint16_t)(finc - Sf);
      if (lane == 63) Q.tb[64] = (uint16_t)nft;
      Q.d[lane] = valid ? a.roff[w] : 0u;
      Q.r0[lane] = r0;
      Q.ws[lane] = fix ? a.woff[w] : 0ull;
      WAVE_SYNC();
      for (u32 t0 = 0; t0 < nft; t0 += 64) {
        const u32 t = t0 + lane;
        if (t < nft) {
          const u32 l = vs_owner(Q.tb, t), s = t - Q.tb[l];
          FvWord F;
          F.load(a.vrec + Q.d[l]);
          fv_subword(T, F, a.words + Q.ws[l], s, a.rmode, sub, a.vrec2 + Q.r0[l] + (u64)s * F.rfull);
        }
      }
      WAVE_SYNC();  // (Q is rewritten by the next words)
    }
    // the other records: the wave copies its lanes' ranges in lane order (contiguous ones merged)
    u64 cs = 0, cd = 0;
    u32 cn = 0;
    auto copy = [&]() {
      const u64* sp = (const u64*)cs;
      for (u32 k = lane; k < cn; k += 64) a.vrec2[cd + k] = sp[k];
    };
    for (u32 l = 0; l < 64; l++) {
      const u32 ln = readlane_u32(nrec, l);
      if (!ln) continue;
      const u64 ls = readlane_u64(src, l), ld = readlane_u64(r0, l);
      if (cn && ls == cs + 8ull * cn && ld == cd + cn) { cn += ln; continue; }
      copy();
      cs = ls; cd = ld; cn = ln;
    }
    copy();
  }
}

#define KC_SLOT 48  // k_keyspace_cplx: per-lane LDS word slot (words <= KC_SLOT - 12 bytes)

// The complex words of k_keyspace_thread (overlapping keys, long keys, oversize
// tiles), one lane per listed word: the general unit walk (next_unit) on global
// bytes; FAST records go to fixed slots after the tile regions.
__global__ void __launch_bounds__(256) k_keyspace_cplx(KsArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const u32 tb = (a.table_bytes + 15u) & ~15u;
  u64* gbuf = (u64*)(smem + tb);
  load_table(smem, a.table, a.table_bytes);
  __syncthreads();
  const Tab T = tab_view(smem);
  uint8_t* wst = (uint8_t*)(gbuf + 2 * 256 * FW_UMAXR);  // KC_SLOT bytes per lane
  const u32 n = *a.cplx_n;
  for (u32 i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const u64 w = a.cplx_list[i];
    const u64 s = a.woff[w], L64 = a.woff[w + 1] - s;
    WordClass C;
    C.flags = 0; C.count = 0; C.bytes = 0; C.ovf = false; C.clusters = false;
    u32 f;
    u64* const rec = a.rec + a.cplx_base + (u64)i * FW_RMAX;
    const bool fits = i < a.cplx_cap;
    if (L64 + 12 <= KC_SLOT) {
      // the word in this lane's LDS slot (all byte loads in flight together): the unit
      // walks below re-read every byte many times
      const uint8_t* gp = a.words + s;
      u32* sl = (u32*)(wst + threadIdx.x * KC_SLOT);
#pragma unroll
      for (u32 q = 0; q < KC_SLOT / 4; q++) {
        u32 v = 0;
#pragma unroll
        for (u32 b = 0; b < 4; b++)
          if (4 * q + b < L64) v |= (u32)gp[4 * q + b] << (8 * b);
        sl[q] = v;
      }
      LWord lw;
      lw.base = wst; lw.off = threadIdx.x * KC_SLOT;
      f = ks_classify(lw, L64, T, a, C);
      if ((f & A5X_WF_FAST) && C.count > 0 && fits) ks_build(lw, (u32)L64, T, a, f, C.count, rec, gbuf + threadIdx.x);
    } else {
      GWord gw;
      gw.p = a.words + s;
      f = ks_classify(gw, L64, T, a, C);
      if ((f & A5X_WF_FAST) && C.count > 0 && fits) ks_build(gw, (u32)L64, T, a, f, C.count, rec, gbuf + threadIdx.x);
    }
    if ((f & A5X_WF_FAST) && C.count > 0) {
      if (fits) a.roff[w] = (u32)(a.cplx_base + (u64)i * FW_RMAX);
      else f = C.clusters ? A5X_WF_DEFER : (f & (A5X_WF_RADIX | A5X_WF_BIN));
    }
    if (f & A5X_WF_DEFER) a.defer_list[atomicAdd(a.defer_n, 1u)] = (u32)w;
    else if (!(f & (A5X_WF_FAST | A5X_WF_ERR_OVF))) a.slow_list[atomicAdd(a.nslow, 1u)] = (u32)w;
    a.count[w] = (f & A5X_WF_DEFER) ? 0 : C.count;
    a.bytes[w] = (f & A5X_WF_DEFER) ? 0 : C.bytes;
    a.flags[w] = f;
  }
}

// ---------------------------------------------------------------------------
// Wave-level word setup shared by k_keyspace_wave and k_expand
// ---------------------------------------------------------------------------
struct Slot {            // radix slot (one disjoint single-key match)
  uint16_t pos, klen;
  u32 R;                 // nvals + 1
  u32 choice_base;       // choices[cb] = key ("keep"), [cb + d] = value d-1
  u32 magic, shift;      // branch-free u32 division by R (libdivide form)
  int delta1;            // |value 0| - klen (radix-2 words)
  u64 Q;                 // product of R over earlier slots (digit weight)
};

// Key matches are kept per "event" = a position where at least one key matches.
// Between events every position is a forced keep, so the DP runs over events
// only: (events+1) x W entries instead of (L+1) x W.
template <int LMAX, int MLMAX, int DPENT>
struct WaveLds {
  static constexpr int SMAX = LMAX < MLMAX ? LMAX : MLMAX;
  uint8_t wbuf[LMAX + 16];
  uint16_t evidx[LMAX + 2];    // number of events at positions < p, p in [0, L]
  uint16_t evpos[SMAX + 1];    // event -> position; evpos[m] = L
  u32 evm[SMAX];               // event -> (mstart << 8) | match count
  uint16_t mlist[MLMAX];       // matching key ids, grouped by event
  union {
    Slot slots[SMAX];
    struct { u64 G[DPENT]; u64 H[DPENT]; } dp;
  };
};

struct WordInfo {
  u32 L, nmatch, nslots;
  u32 cls;         // A5X_WF_RADIX [| A5X_WF_BIN] or A5X_WF_GENERAL; 0 = no candidates
  u32 fits;        // 1: the word's setup fit this pass's LDS budget
  u32 freew, W, Cc;
  int lo;
  u32 maxlen;      // upper bound on (candidate length + 1)
  int udelta;      // radix-2: common |v|-klen of all slots, or INT_MIN
  u64 count, bytes;
  u32 ovf;
  u32 nev;         // events (positions with a key match)
  u32 why;         // diagnostics when !fits: 1 long, 2 matches, 3 columns, 4 DP size
};

__device__ __forceinline__ u32 fastdiv(u32 n, u32 magic, u32 shift) {
  u32 q = __umulhi(n, magic);
  return (q + ((n - q) >> 1)) >> shift;
}

// One wave sets up word w: bytes -> wbuf, key matches grouped by event, class,
// and either radix slots or the event DP tables.  Returned fields are uniform.
template <int LMAX, int MLMAX, int DPENT>
__device__ WordInfo wave_setup(WaveLds<LMAX, MLMAX, DPENT>& S, const Tab& T, const uint8_t* words,
                               const u64* woff, u64 w, int mn, int mx) {
  typedef WaveLds<LMAX, MLMAX, DPENT> LdsT;
  WordInfo I;
  const u32 lane = lane_id();
  const u64 s = woff[w];
  const u64 L64 = woff[w + 1] - s;
  I.L = (u32)min(L64, (u64)0xffffffffu);
  I.cls = 0; I.fits = 1; I.nslots = 0; I.count = 0; I.bytes = 0; I.ovf = 0; I.nev = 0;
  I.maxlen = 0; I.udelta = INT32_MIN; I.freew = 1; I.W = 2; I.Cc = 1; I.lo = 1; I.nmatch = 0; I.why = 0;
  if (mx < 1 || L64 == 0) return I;
  const u32 L = I.L;
  const bool stored = L64 <= (u64)LMAX;
  const uint8_t* wp = words + s;
  if (stored) {
    for (u32 p = lane; p < L + 16 && p < LMAX + 16; p += 64) S.wbuf[p] = p < L ? wp[p] : 0;
  }
  ws_sync<LMAX>();
  // ---- matches: positions in chunks of 64 lanes ----
  u32 base = 0, evbase = 0, prev_end = 0;  // running matches / events / max match end
  bool conflict = false, multi = false, room = true;
  u32 maxadd = 0;
  for (u32 p0 = 0; p0 < L; p0 += 64) {
    const u32 p = p0 + lane;
    u32 nm = 0, kmax = 0, dmax = 0;
    if (p < L) {
      const u32 b = stored ? S.wbuf[p] : wp[p];
      const u32 ks = T.bucket[b], ke = T.bucket[b + 1];
      for (u32 k = ks; k < ke; k++) {
        const A5xKey key = T.keys[k];
        if (p + key.klen > L || !key_match_global(wp, p, key, T)) continue;
        nm++;
        kmax = max(kmax, (u32)key.klen);
        if (key.maxdelta > 0) dmax = max(dmax, (u32)key.maxdelta);
      }
    }
    // overlap: a match at p conflicts if an earlier match (any position < p) ends after p
    const u32 endp = nm ? p + kmax : 0;
    u32 pre = endp;  // inclusive max-scan
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      u32 y = __shfl_up((int)pre, d);
      if ((int)lane >= d) pre = max(pre, y);
    }
    u32 before = __shfl_up((int)pre, 1);
    if (lane == 0) before = 0;
    before = max(before, prev_end);
    if (nm && before > p) conflict = true;
    if (nm > 1) multi = true;
    const u32 incl = wave_incl_scan_u32(nm);
    const u32 mstart = base + incl - nm;
    const u64 bal = __ballot(nm > 0);
    const u32 ev = evbase + (u32)__popcll(bal & ((1ull << lane) - 1ull));
    const u32 nev_after = evbase + (u32)__popcll(bal);
    const u32 nm_after = base + __shfl((int)incl, 63);
    if (stored && nev_after <= (u32)LdsT::SMAX && nm_after <= (u32)MLMAX) {
      if (p < L) S.evidx[p] = (uint16_t)ev;
      if (nm) {
        S.evpos[ev] = (uint16_t)p;
        S.evm[ev] = (mstart << 8) | min(nm, 255u);
        const u32 b = S.wbuf[p];
        const u32 ks = T.bucket[b], ke = T.bucket[b + 1];
        u32 j = 0;
        for (u32 k = ks; k < ke; k++) {
          const A5xKey key = T.keys[k];
          if (p + key.klen > L || !key_match_global(wp, p, key, T)) continue;
          S.mlist[mstart + j++] = (uint16_t)k;
        }
      }
    } else {
      room = false;
    }
    maxadd += (u32)wave_sum_u64(dmax);
    base = nm_after;
    evbase = nev_after;
    prev_end = max(prev_end, (u32)__shfl((int)pre, 63));
  }
  conflict = wave_or_u32(conflict) != 0;
  multi = wave_or_u32(multi) != 0;
  I.nmatch = base;
  I.nev = evbase;
  I.maxlen = L + 1 + maxadd;
  if (base == 0) return I;                                  // no candidates
  I.freew = (mn <= 1) && ((i64)base <= (i64)mx);
  I.lo = mn <= 1 ? 1 : mn;
  if (!stored || !room) { I.fits = 0; I.why = stored ? 2 : 1; I.cls = A5X_WF_GENERAL; return I; }
  if (lane == 0) { S.evidx[L] = (uint16_t)evbase; S.evpos[evbase] = (uint16_t)L; }
  ws_sync<LMAX>();
  const u32 m = evbase;

  if (!conflict && !multi && I.freew) {
    // ---- radix slots: one per event, digit weights Q ----
    for (u32 i = lane; i < m; i += 64) {
      const A5xKey key = T.keys[S.mlist[S.evm[i] >> 8]];
      Slot sl;
      sl.pos = S.evpos[i]; sl.klen = key.klen; sl.R = (u32)key.nvals + 1u;
      sl.choice_base = key.choice_base;
      divmagic(sl.R, sl.magic, sl.shift);
      sl.delta1 = (int)T.ch[key.choice_base + 1].len - (int)key.klen;
      sl.Q = 0;
      S.slots[i] = sl;
    }
    I.nslots = m;
    ws_sync<LMAX>();
    // digit weights (serial; nslots is small) and P
    u64 P = 1;
    bool ovf = false, bin = true;
    int ud = S.slots[0].delta1;
    for (u32 i = 0; i < m; i++) {
      const u32 R = S.slots[i].R;
      if (lane == 0) S.slots[i].Q = P;
      P = mul_ovf(P, R, ovf);
      if (R != 2) bin = false;
      if (S.slots[i].delta1 != ud) ud = INT32_MIN;
    }
    ws_sync<LMAX>();
    if (!ovf && P <= (1ull << 32)) {
      // bytes = (P-1)(L+1) + sum_slots (P/R) sum_v delta   (lanes over slots)
      i64 part = 0;
      for (u32 i = lane; i < m; i += 64) {
        const Slot sl = S.slots[i];
        i64 sd = 0;
        for (u32 v = 1; v < sl.R; v++) sd += (i64)T.ch[sl.choice_base + v].len - (i64)sl.klen;
        part += (i64)(P / sl.R) * sd;
      }
      const i64 dsum = wave_sum_i64(part);
      I.cls = A5X_WF_RADIX | (bin ? A5X_WF_BIN : 0u);
      I.count = P - 1;
      I.bytes = (P - 1) * (u64)(L + 1) + (u64)dsum;
      I.udelta = bin ? ud : INT32_MIN;
      return I;
    }
    I.nslots = 0;
    // overflowing radix words go through the DP (same counts, u64 walk)
  }
  // ---- general: DP over events with a count window ----
  // G[e][c]: completions from event e having made c substitutions (c clamped to 1 in
  // the free window); H[e][c]: their bytes from position evpos[e] on, newline incl.
  I.cls = A5X_WF_GENERAL;
  u32 C = I.freew ? 1u : (u32)min((i64)mx, (i64)base);
  I.Cc = C;
  I.W = C + 1;
  if (I.W > 64 || (u64)(m + 1) * I.W > (u64)DPENT) { I.fits = 0; I.why = I.W > 64 ? 3 : 4; return I; }
  const u32 W = I.W, c = lane;
  bool ovf = false;
  for (int e = (int)m; e >= 0; --e) {
    if (c < W) {
      u64 g, h;
      if (e == (int)m) {
        g = I.freew ? (c == 1 ? 1u : 0u) : ((int)c >= I.lo ? 1u : 0u);
        h = g;
      } else {
        const u32 q = S.evpos[e], qn = S.evpos[e + 1];
        g = S.dp.G[(e + 1) * W + c];
        h = add_ovf(S.dp.H[(e + 1) * W + c], mul_ovf(g, qn - q, ovf), ovf);
        const u32 em = S.evm[e], ms = em >> 8, mc = em & 255u;
        const u32 nc = I.freew ? 1u : c + 1u;
        if (nc <= C) {
          for (u32 j = 0; j < mc; j++) {
            const A5xKey key = T.keys[S.mlist[ms + j]];
            const u32 p2 = q + key.klen, e2 = S.evidx[p2], lit = S.evpos[e2] - p2;
            const u64 gs = S.dp.G[e2 * W + nc];
            const u64 hs = S.dp.H[e2 * W + nc];
            g = add_ovf(g, mul_ovf(gs, key.nvals, ovf), ovf);
            const u64 per = (u64)key.sumlen + (u64)key.nvals * lit;
            h = add_ovf(h, add_ovf(mul_ovf(hs, key.nvals, ovf), mul_ovf(gs, per, ovf), ovf), ovf);
          }
        }
      }
      S.dp.G[e * W + c] = g;
      S.dp.H[e * W + c] = h;
    }
    ws_sync<LMAX>();
  }
  I.ovf = wave_or_u32(ovf) != 0;
  I.count = S.dp.G[0];
  bool o2 = false;
  I.bytes = add_ovf(S.dp.H[0], mul_ovf(S.dp.G[0], S.evpos[0], o2), o2);  // + literal prefix
  if (o2) I.ovf = 1;
  return I;
}

// ---------------------------------------------------------------------------
// Keyspace for deferred words: one wave per word (pass-B budget)
// ---------------------------------------------------------------------------
typedef WaveLds<A5X_LMAX_B, A5X_MLMAX_B, A5X_DPENT_B> LdsB;
static_assert(FW_RMAX * 8 <= sizeof(WaveLds<A5X_LMAX_B, A5X_MLMAX_B, A5X_DPENT_B>), "k_locate stages a record in LdsB");
typedef WaveLds<A5X_LMAX_A, A5X_MLMAX_A, A5X_DPENT_A> LdsA;

__global__ void __launch_bounds__(64) k_keyspace_wave(KsArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  load_table(smem, a.table, a.table_bytes);
  __syncthreads();
  const Tab T = tab_view(smem);
  LdsB& S = *(LdsB*)(smem + ((a.table_bytes + 15u) & ~15u));
  const u32 n = *a.defer_n;
  for (u32 i = blockIdx.x; i < n; i += gridDim.x) {
    const u32 w = a.defer_list[i];
    WordInfo I = wave_setup<A5X_LMAX_B, A5X_MLMAX_B, A5X_DPENT_B>(S, T, a.words, a.woff, w, a.mn, a.mx);
    if (lane_id() == 0) {
      u32 f = I.cls ? I.cls : (u32)(A5X_WF_RADIX | A5X_WF_FAST);
      // beyond the LDS budget (long line, many matches, big DP or long candidates):
      // pass G (k_keyspace_g) sizes it in HBM scratch and puts it on the BIG list
      const bool glob = I.cls && (!I.fits || I.maxlen > A5X_RING_B - 16) && I.why != 3;
      // would pass A (smaller LDS budget) handle it?
      bool fitsA = I.L <= A5X_LMAX_A && I.nmatch <= A5X_MLMAX_A && I.maxlen <= A5X_RING_A - 16 &&
                   (I.cls != A5X_WF_GENERAL || (u64)(I.nev + 1) * I.W <= A5X_DPENT_A);
      if (glob) {
        f = A5X_WF_BIG | A5X_WF_GLOB;
        a.glob_list[atomicAdd(a.glob_n, 1u)] = w;
      } else if (I.cls && !fitsA) {
        f |= A5X_WF_BIG;
        a.big_list[atomicAdd(a.nbig, 1u)] = w;
      } else if (I.cls) {
        a.slow_list[atomicAdd(a.nslow, 1u)] = w;
      }
      if (!glob && I.cls && (!I.fits || I.maxlen > A5X_RING_B - 16)) {  // W > 64 count columns
        f |= A5X_WF_ERR_BIG | ((I.fits ? 5u : I.why) << 16) | (min(I.W, 255u) << 24);
        atomicOr(a.err, A5X_DERR_BIG);
      }
      if (I.ovf) { f |= A5X_WF_ERR_OVF; atomicOr(a.err, A5X_DERR_OVF); }
      const bool bad = glob || (f & (A5X_WF_ERR_BIG | A5X_WF_ERR_OVF)) != 0;
      a.count[w] = bad ? 0 : I.count;
      a.bytes[w] = bad ? 0 : I.bytes;
      a.flags[w] = f;
    }
    WAVE_SYNC();
  }
}

// ---------------------------------------------------------------------------
// Pass G: words beyond the pass-B LDS budget (lines up to 64 KiB, more matches,
// bigger DP tables, candidates up to A5X_RING_G - 16 bytes).  The same wave_setup /
// expand_word code on a WaveLds and ring in HBM scratch, one slot per workgroup.
// ---------------------------------------------------------------------------
typedef WaveLds<A5X_LMAX_G, A5X_MLMAX_G, A5X_DPENT_G> LdsG;
#define GSLOT_BYTES ((u64)A5X_RING_G + (((u64)sizeof(LdsG) + 255ull) & ~255ull))

__global__ void __launch_bounds__(64) k_keyspace_g(KsArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  load_table(smem, a.table, a.table_bytes);
  __syncthreads();
  const Tab T = tab_view(smem);
  LdsG& S = *(LdsG*)(a.gscr + (u64)blockIdx.x * GSLOT_BYTES + A5X_RING_G);
  const u32 n = *a.glob_n;
  for (u32 i = blockIdx.x; i < n; i += gridDim.x) {
    const u32 w = a.glob_list[i];
    WordInfo I = wave_setup<A5X_LMAX_G, A5X_MLMAX_G, A5X_DPENT_G>(S, T, a.words, a.woff, w, a.mn, a.mx);
    if (lane_id() == 0) {
      u32 f = (I.cls ? I.cls : (u32)A5X_WF_RADIX) | A5X_WF_BIG | A5X_WF_GLOB;
      bool bad = false;
      if (I.cls && (!I.fits || I.maxlen > A5X_RING_G - 16)) {
        f |= A5X_WF_ERR_BIG | ((I.fits ? 5u : I.why) << 16) | (min(I.W, 255u) << 24);
        atomicOr(a.err, A5X_DERR_BIG);
        bad = true;
      } else if (I.cls) {
        a.big_list[atomicAdd(a.nbig, 1u)] = w;
      }
      if (I.ovf) { f |= A5X_WF_ERR_OVF; atomicOr(a.err, A5X_DERR_OVF); bad = true; }
      a.count[w] = bad ? 0 : I.count;
      a.bytes[w] = bad ? 0 : I.bytes;
      a.flags[w] = f;
    }
    ws_sync<A5X_LMAX_G>();
  }
}

// ---------------------------------------------------------------------------
// Exclusive scan of (count, bytes) pairs: n -> n+1 entries (last = totals)
// ---------------------------------------------------------------------------
#define SCAN_ITEMS 8
#define SCAN_BLOCK 256
#define SCAN_TILE (SCAN_ITEMS * SCAN_BLOCK)

__device__ __forceinline__ void block_excl_scan2(u64& a, u64& b, u64& ta, u64& tb, u32* errp) {
  __shared__ u64 sa[SCAN_BLOCK / 64], sb[SCAN_BLOCK / 64];
  const u32 lane = lane_id(), wv = threadIdx.x / 64;
  u64 ia = a, ib = b;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    u64 ya = shfl_up_u64(ia, d), yb = shfl_up_u64(ib, d);
    if ((int)lane >= d) { ia += ya; ib += yb; }
  }
  if (lane == 63) { sa[wv] = ia; sb[wv] = ib; }
  __syncthreads();
  u64 oa = 0, ob = 0;
  for (u32 k = 0; k < wv; k++) { oa += sa[k]; ob += sb[k]; }
  ta = 0; tb = 0;
  for (u32 k = 0; k < SCAN_BLOCK / 64; k++) { ta += sa[k]; tb += sb[k]; }
  a = oa + ia - a;
  b = ob + ib - b;
  __syncthreads();
}

__global__ void __launch_bounds__(SCAN_BLOCK) k_scan_reduce(const u64* ca, const u64* cb, u64 n, u64* sa, u64* sb,
                                                             u32* err) {
  const u64 base = (u64)blockIdx.x * SCAN_TILE;
  u64 a = 0, b = 0;
  for (u32 j = 0; j < SCAN_ITEMS; j++) {
    const u64 i = base + (u64)j * SCAN_BLOCK + threadIdx.x;
    if (i < n) {
      const u64 x = ca[i], y = cb[i];
      a += x; b += y;
      if (a < x || b < y) atomicOr(err, A5X_DERR_SCANOVF);
    }
  }
  u64 ta, tb;
  block_excl_scan2(a, b, ta, tb, err);
  if (threadIdx.x == 0) { sa[blockIdx.x] = ta; sb[blockIdx.x] = tb; }
}

// out[i] = exclusive prefix (+ block offset); out[n] = total when this block is last
__global__ void __launch_bounds__(SCAN_BLOCK) k_scan_down(const u64* ca, const u64* cb, u64 n, const u64* oa,
                                                           const u64* ob, u64* outa, u64* outb, u32* err) {
  __shared__ u64 la[SCAN_TILE], lb[SCAN_TILE];
  const u64 base = (u64)blockIdx.x * SCAN_TILE;
  for (u32 j = 0; j < SCAN_ITEMS; j++) {
    const u32 t = j * SCAN_BLOCK + threadIdx.x;
    const u64 i = base + t;
    la[t] = i < n ? ca[i] : 0;
    lb[t] = i < n ? cb[i] : 0;
  }
  __syncthreads();
  u64 a = 0, b = 0;
  for (u32 j = 0; j < SCAN_ITEMS; j++) { a += la[threadIdx.x * SCAN_ITEMS + j]; b += lb[threadIdx.x * SCAN_ITEMS + j]; }
  u64 ta, tb;
  u64 ea = a, eb = b;
  block_excl_scan2(ea, eb, ta, tb, err);
  u64 ra = (oa ? oa[blockIdx.x] : 0) + ea, rb = (ob ? ob[blockIdx.x] : 0) + eb;
  for (u32 j = 0; j < SCAN_ITEMS; j++) {
    const u32 t = threadIdx.x * SCAN_ITEMS + j;
    const u64 x = la[t], y = lb[t];
    la[t] = ra; lb[t] = rb;
    ra += x; rb += y;
  }
  // totals: the thread holding element n-1 (tile-local) ends with the inclusive sum
  // (items past n are zero-padded); read before anything is overwritten in place.
  const bool last_blk = base + SCAN_TILE >= n;
  if (last_blk && threadIdx.x == (u32)((n - 1 - base) / SCAN_ITEMS)) {
    outa[n] = ra; outb[n] = rb;
  }
  __syncthreads();
  for (u32 j = 0; j < SCAN_ITEMS; j++) {
    const u32 t = j * SCAN_BLOCK + threadIdx.x;
    const u64 i = base + t;
    if (i < n) { outa[i] = la[t]; outb[i] = lb[t]; }
  }
}

// ---------------------------------------------------------------------------
// Chunk planner: chunk c covers global candidates [c*CH, (c+1)*CH)
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_plan(const u64* cand_off, u64 nw, u64 CH, u32* chunk_w0) {
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 w = (u64)blockIdx.x * blockDim.x + threadIdx.x; w < nw; w += stride) {
    const u64 a = cand_off[w], b = cand_off[w + 1];
    if (b <= a) continue;
    for (u64 c = (a + CH - 1) / CH; c * CH < b; c++) chunk_w0[c] = (u32)w;
  }
}

// Segments of the listed (slow or BIG) words: word w's candidates inside the call's
// range [cb, ce), cut into pieces of CH; item = w | s << 32 (order is irrelevant).
__global__ void __launch_bounds__(256) k_segments(const u32* list, const u32* list_n, const u64* cand_off, u64 cb,
                                                  u64 ce, u64 CH, u64* segs, u32* nsegs) {
  const u32 n = *list_n;
  const u32 stride = gridDim.x * blockDim.x;
  const u32 i0 = blockIdx.x * blockDim.x + threadIdx.x;
  for (u32 ib = i0 - lane_id(); ib < n; ib += stride) {  // whole waves (wave_append)
    const u32 i = ib + lane_id();
    u64 k = 0;
    u32 w = 0;
    if (i < n) {
      w = list[i];
      const u64 lo = max(cb, cand_off[w]), hi = min(ce, cand_off[w + 1]);
      k = hi > lo ? (hi - lo + CH - 1) / CH : 0;
    }
    // per-wave base: exclusive scan of k (k < 2^32 since a word has < 2^32 candidates)
    const u32 incl = wave_incl_scan_u32((u32)k);
    u32 base = 0;
    if (lane_id() == 63 && incl) base = atomicAdd(nsegs, incl);
    base = readlane_u32(base, 63);
    const u32 o = base + incl - (u32)k;
    for (u64 t = 0; t < k; t++) segs[o + t] = (u64)w | (t << 32);
  }
}

// ---------------------------------------------------------------------------
// Expansion
// ---------------------------------------------------------------------------
struct ExpArgs {
  const uint8_t* table;
  u32 table_bytes;
  const uint8_t* words;
  const u64* woff;
  u64 nw;
  const u64* cand_off;   // n+1, exclusive prefix of counts
  const u64* byte_off;   // n+1, exclusive prefix of bytes
  const u32* flags;
  const u32* chunk_w0;
  const u64* segs;       // k_expand_slow / k_expand_b work items (k_segments)
  const u32* nsegs;
  u64 cand_begin, cand_end;  // global candidate range of this call
  u64 CH;
  u64 SEG;               // candidates per k_segments item
  uint8_t* out;
  u64 out_base;          // byte_off value that maps to out[0]
  u64 out_cap;           // bytes writable at out
  int mn, mx;
  u32* err;
  u64* dbg;              // 8-word debug record of the first tripped guard
  const u64* rec;        // FAST plan records (k_keyspace_thread)
  const u32* roff;       // per word: record offset into rec
  u64 rec_n;             // u64 in rec
  // fused digest (k_expand_fast_dig): target set (a5x_md.h md_probe) and hits
  const u32* dg_bitmap;
  u32 dg_bm_mask, dg_has_zero, dg_hit_cap;
  const uint4* dg_table;
  u64 dg_tmask;
  A5xHitRaw* dg_hits;    // (word, candidate in word, digest)
  u32* dg_nhits;
  uint8_t* gscr;         // pass G scratch slots (k_expand_g, k_locate)
  u32 gslots;
  const u32* vmap;       // virtual word list (k_vwords_fill; null: words): entry -> word,
  const u32* vobase;     // and its first candidate's index in the word (hit records)
};

// a fused-digest hit of candidate c of list entry e as (word, candidate in word)
__device__ __forceinline__ void hit_word(const ExpArgs& a, u64 e, u64 c, A5xHitRaw& r) {
  r.blk = a.vmap ? (u64)a.vmap[e] : e;
  r.idx = a.vmap ? c + a.vobase[e] : c;
}

// Record the first tripped guard (code + context) and flag the call as failed.
// Takes the two pointers (not the argument struct) so the kernel arguments are
// never spilled to scratch.
__device__ __forceinline__ void guard_trip2(u32* err, u64* dbg, u64 code, u64 x0, u64 x1, u64 x2, u64 x3) {
  atomicOr(err, A5X_DERR_GUARD);
  if (atomicCAS((unsigned long long*)dbg, 0ull, (unsigned long long)code) == 0ull) {
    dbg[1] = x0; dbg[2] = x1; dbg[3] = x2; dbg[4] = x3;
    dbg[5] = blockIdx.x; dbg[6] = threadIdx.x;
  }
}
#define guard_trip(A, code, x0, x1, x2, x3) guard_trip2((A).err, (A).dbg, code, x0, x1, x2, x3)

// Per-lane byte emitter: bytes are OR-ed into an all-zero LDS ring at their
// final positions (ring index = byte offset relative to the run base).
struct Emit {
  u64 acc;
  u32 n;   // pending bytes in acc
  u32 dw;  // dword index (relative to run base) of acc's low dword
};

template <u32 RING>
__device__ __forceinline__ void em_put(Emit& e, u32* ring, u32 piece, u32 plen) {
  e.acc |= (u64)piece << (8u * e.n);
  e.n += plen;
  if (e.n >= 4) {
    atomicOr(&ring[e.dw & (RING / 4 - 1)], (u32)e.acc);
    e.dw++;
    e.acc >>= 32;
    e.n -= 4;
  }
}
template <u32 RING>
__device__ __forceinline__ void em_bytes(Emit& e, u32* ring, const uint8_t* src, u32 off, u32 len) {
  for (u32 k = 0; k < len; k += 4) {
    const u32 m = min(4u, len - k);
    em_put<RING>(e, ring, keep_bytes(lds_ld4(src, off + k), m), m);
  }
}
template <u32 RING>
__device__ __forceinline__ void em_choice(Emit& e, u32* ring, const Tab& T, u32 ci) {
  const A5xChoice c = T.ch[ci];
  if (c.len <= 4) em_put<RING>(e, ring, c.first4, c.len);
  else em_bytes<RING>(e, ring, T.blob, c.blob_off, c.len);
}
template <u32 RING>
__device__ __forceinline__ void em_finish(Emit& e, u32* ring) {
  if (e.n) atomicOr(&ring[e.dw & (RING / 4 - 1)], (u32)e.acc);
}

// Global byte range of one "run" (contiguous output) staged through the ring.
struct Run {
  u64 base;     // 16-aligned global byte position (relative to out_base) of ring origin
  u64 lo;       // first byte owned by this wave
  u64 pos;      // next byte to be produced
  u64 flushed;  // bytes < flushed are in HBM (16-aligned, >= base)
  bool open;
};

__device__ __forceinline__ void store_block(const ExpArgs& a, u64 X, uint4 v, u64 lo, u64 hi) {
  // block [X, X+16) restricted to bytes [lo, hi); never beyond out_cap
  if (hi > a.out_cap || X + 16 <= lo) {
    guard_trip(a, 1, X, lo, hi, a.out_cap);
    return;
  }
  if (X >= lo && X + 16 <= hi) {
    *(uint4*)(a.out + X) = v;
  } else {
    const u32 wv[4] = {v.x, v.y, v.z, v.w};
    for (u32 b = 0; b < 16; b++) {
      const u64 Y = X + b;
      if (Y >= lo && Y < hi) a.out[Y] = (uint8_t)(wv[b >> 2] >> (8 * (b & 3)));
    }
  }
}

// stream complete blocks [flushed, upto) (upto 16-aligned) and zero them in the ring
template <u32 RING>
__device__ __forceinline__ void run_flush(Run& R, u32* ring, const ExpArgs& a, u64 upto, u64 hi) {
  const u32 lane = lane_id();
  const u64 nb = (upto - R.flushed) / 16;
  for (u64 b = lane; b < nb; b += 64) {
    const u64 X = R.flushed + b * 16;
    uint4* rp = (uint4*)ring + (((X - R.base) / 16) & (RING / 16 - 1));
    uint4 v;
    if constexpr (RING > A5X_RING_B) {  // pass G: the ring is HBM scratch, filled by atomics
      u32* q = (u32*)rp;
      v = make_uint4(atomicExch(q, 0u), atomicExch(q + 1, 0u), atomicExch(q + 2, 0u), atomicExch(q + 3, 0u));
    } else {
      v = *rp;
      *rp = make_uint4(0, 0, 0, 0);
    }
    store_block(a, X, v, R.lo, hi);
  }
  R.flushed = upto;
  ws_sync<(RING > A5X_RING_B ? A5X_LMAX_G : 0)>();
}

template <u32 RING>
__device__ __forceinline__ void run_close(Run& R, u32* ring, const ExpArgs& a) {
  if (!R.open) return;
  const u64 full = R.pos & ~15ull;
  if (full > R.flushed) run_flush<RING>(R, ring, a, full, R.pos);
  if (R.pos > R.flushed) run_flush<RING>(R, ring, a, R.flushed + 16, R.pos);  // partial tail block
  R.open = false;
}

template <u32 RING>
__device__ __forceinline__ void run_open(Run& R, u64 pos) {
  R.base = pos & ~15ull;
  R.lo = pos;
  R.pos = pos;
  R.flushed = R.base;
  R.open = true;
}

// prefix bytes of candidates [0, r) of a radix word (candidate r <-> idx r+1)
template <int LMAX, int MLMAX, int DPENT>
__device__ u64 radix_prefix_bytes(const WaveLds<LMAX, MLMAX, DPENT>& S, const Tab& T, const WordInfo& I, u64 r) {
  if (r == 0) return 0;
  const u64 Y = r + 1;  // idx in [0, Y) minus idx 0
  i64 part = 0;
  for (u32 i = lane_id(); i < I.nslots; i += 64) {
    const Slot sl = S.slots[i];
    const u64 QR = sl.Q * sl.R, full = Y / QR, rem = Y % QR;
    for (u32 v = 1; v < sl.R; v++) {
      const u64 lo = (u64)v * sl.Q;
      const u64 cnt = full * sl.Q + (rem > lo ? min(sl.Q, rem - lo) : 0);
      part += ((i64)T.ch[sl.choice_base + v].len - (i64)sl.klen) * (i64)cnt;
    }
  }
  return (u64)((i64)(r * (u64)(I.L + 1)) + wave_sum_i64(part));
}

// General DP walk for candidate rank r: returns length (incl. newline); emits if EMIT.
template <bool EMIT, u32 RING, int LMAX, int MLMAX, int DPENT>
__device__ u32 dp_walk(const WaveLds<LMAX, MLMAX, DPENT>& S, const Tab& T, const WordInfo& I, u64 r, Emit& e,
                       u32* ring) {
  const u32 W = I.W, m = I.nev;
  u32 p = 0, c = 0, len = 1;
  for (;;) {
    const u32 ev = S.evidx[p], q = S.evpos[ev];
    if (q > p) {  // forced keeps up to the next event
      if (EMIT) em_bytes<RING>(e, ring, S.wbuf, p, q - p);
      len += q - p;
    }
    if (ev >= m) break;
    const u64 gk = S.dp.G[(ev + 1) * W + c];
    if (r < gk) {
      if (EMIT) em_put<RING>(e, ring, S.wbuf[q], 1);
      len++;
      p = q + 1;
      continue;
    }
    r -= gk;
    const u32 em = S.evm[ev], ms = em >> 8, mc = em & 255u;
    const u32 nc = I.freew ? 1u : c + 1u;
    u32 choice = 0, kl = 1;
    for (u32 j = 0; j < mc && nc <= I.Cc; j++) {
      const A5xKey key = T.keys[S.mlist[ms + j]];
      const u64 gs = S.dp.G[S.evidx[q + key.klen] * W + nc];
      if (gs == 0) continue;
      u64 qv;
      if (key.nvals <= 8) {
        qv = 0;
        while (qv < key.nvals && r >= gs) { r -= gs; qv++; }
        if (qv < key.nvals) { choice = key.choice_base + 1 + (u32)qv; kl = key.klen; break; }
      } else {
        qv = r / gs;
        if (qv < key.nvals) { r -= qv * gs; choice = key.choice_base + 1 + (u32)qv; kl = key.klen; break; }
        r -= gs * key.nvals;
      }
    }
    // choice == 0 cannot happen for r < G[ev][c]
    if (EMIT) em_choice<RING>(e, ring, T, choice);
    len += T.ch[choice].len;
    p = q + kl;
    c = nc;
  }
  if (EMIT) em_put<RING>(e, ring, '\n', 1);
  return len;
}

// byte offset of candidate r inside its word's output (general words; any lane)
template <int LMAX, int MLMAX, int DPENT>
__device__ u64 dp_prefix_bytes(const WaveLds<LMAX, MLMAX, DPENT>& S, const Tab& T, const WordInfo& I, u64 r) {
  const u32 W = I.W, m = I.nev;
  u32 p = 0, c = 0;
  u64 pl = 0, acc = 0;
  for (;;) {
    const u32 ev = S.evidx[p], q = S.evpos[ev];
    pl += q - p;
    if (ev >= m) break;
    const u32 qn = S.evpos[ev + 1];
    const u64 gk = S.dp.G[(ev + 1) * W + c];
    if (r < gk) { pl++; p = q + 1; continue; }
    r -= gk;
    acc += S.dp.H[(ev + 1) * W + c] + (pl + (qn - q)) * gk;
    const u32 em = S.evm[ev], ms = em >> 8, mc = em & 255u;
    const u32 nc = I.freew ? 1u : c + 1u;
    u32 choice = 0, kl = 1;
    for (u32 j = 0; j < mc && nc <= I.Cc; j++) {
      const A5xKey key = T.keys[S.mlist[ms + j]];
      const u32 p2 = q + key.klen, e2 = S.evidx[p2], lit = S.evpos[e2] - p2;
      const u64 gs = S.dp.G[e2 * W + nc];
      const u64 hs = S.dp.H[e2 * W + nc];
      bool found = false;
      for (u32 v = 0; v < key.nvals; v++) {
        const u32 ci = key.choice_base + 1 + v;
        if (r < gs) { choice = ci; kl = key.klen; found = true; break; }
        r -= gs;
        acc += hs + (pl + T.ch[ci].len + lit) * gs;
      }
      if (found) break;
    }
    pl += T.ch[choice].len;
    p = q + kl;
    c = nc;
  }
  return acc;
}

// One word (any class) through the per-word path: wave_setup in LDS, then rounds of
// up to 64 candidates (radix digits or the DP walk).  Candidates [r, r+nhere).
template <int LMAX, int MLMAX, int DPENT, u32 RING>
__device__ bool expand_word(WaveLds<LMAX, MLMAX, DPENT>& S, u32* ring, const Tab& T, const ExpArgs& a, Run& R,
                            u64 w, u64 r, u64 nhere, u64 cnt) {
  const u32 lane = lane_id();
  WordInfo I = wave_setup<LMAX, MLMAX, DPENT>(S, T, a.words, a.woff, w, a.mn, a.mx);
  if (!I.fits || I.count != cnt || I.maxlen > RING - 16) {
    if (lane == 0) atomicOr(a.err, A5X_DERR_STATE);
    return false;
  }
  u64 pos = a.byte_off[w] - a.out_base;
  if (r) {
    if (I.cls & A5X_WF_RADIX) pos += radix_prefix_bytes(S, T, I, r);
    else pos += uniform64(dp_prefix_bytes(S, T, I, r));
  }
  if (!R.open || R.pos != pos) {
    run_close<RING>(R, ring, a);
    run_open<RING>(R, pos);
  }
  // lanes per round: the ring holds at most RING-16 unflushed bytes
  const u32 nl = min(64u, (RING - 16) / I.maxlen);
  const u64 rend = r + nhere;
  for (u64 rr = r; rr < rend; rr += nl) {
    const bool act = lane < nl && rr + lane < rend;
    const u64 rk = rr + lane;
    u32 len = 0;
    Emit e;
    if (I.cls & A5X_WF_RADIX) {
      const u32 idx = (u32)(rk + 1);
      if (act) {
        int l = (int)I.L + 1;
        u32 n = idx;
        for (u32 i = 0; i < I.nslots; i++) {
          const Slot& sl = S.slots[i];
          const u32 q = fastdiv(n, sl.magic, sl.shift);
          const u32 d = n - q * sl.R;
          n = q;
          if (d) l += (int)T.ch[sl.choice_base + d].len - (int)sl.klen;
        }
        len = (u32)l;
      }
      const u32 incl = wave_incl_scan_u32(len);
      const u32 tot = lane63(incl);
      const u64 off = R.pos + incl - len - R.base;
      if (act) {
        e.acc = 0; e.n = (u32)off & 3u; e.dw = (u32)(off >> 2);
        u32 prev = 0, n = idx;
        for (u32 i = 0; i < I.nslots; i++) {
          const Slot& sl = S.slots[i];
          const u32 q = fastdiv(n, sl.magic, sl.shift);
          const u32 d = n - q * sl.R;
          n = q;
          if (sl.pos > prev) em_bytes<RING>(e, ring, S.wbuf, prev, sl.pos - prev);
          em_choice<RING>(e, ring, T, sl.choice_base + d);
          prev = sl.pos + sl.klen;
        }
        if (I.L > prev) em_bytes<RING>(e, ring, S.wbuf, prev, I.L - prev);
        em_put<RING>(e, ring, '\n', 1);
        em_finish<RING>(e, ring);
      }
      R.pos += tot;
    } else {
      if (act) len = dp_walk<false, RING>(S, T, I, rk, e, ring);
      const u32 incl = wave_incl_scan_u32(len);
      const u32 tot = lane63(incl);
      const u64 off = R.pos + incl - len - R.base;
      if (act) {
        e.acc = 0; e.n = (u32)off & 3u; e.dw = (u32)(off >> 2);
        dp_walk<true, RING>(S, T, I, rk, e, ring);
        em_finish<RING>(e, ring);
      }
      R.pos += tot;
    }
    ws_sync<LMAX>();
    const u64 full = R.pos & ~15ull;
    if (full > R.flushed) run_flush<RING>(R, ring, a, full, R.pos);
  }
  ws_sync<LMAX>();
  return true;
}

// ---------------------------------------------------------------------------
// k_expand_fast: one wave per CH-candidate chunk; windows of consecutive FAST
// words of one keyspace tile.
//
// The plan records (a5x_plan.h) were built by k_keyspace_thread, packed in word
// order per tile, so a window's records are ONE contiguous HBM range: the window
// setup is a 16-B-per-lane copy into LDS plus one metadata load per word.
// Rounds of <= 64 consecutive candidates span word boundaries (lane = candidate):
//   pass 1  one u64 LDS read + one umulhi per group -> length + per-piece digits;
//   scan    DPP wave prefix sum of the lengths -> byte offsets;
//   pass 2  one entry read per piece, bytes appended to whole aligned dwords of a
//           per-wave LDS ring (fw_pass2: plain ds_write_b32, no atomics, no
//           zeroing; a dword shared by two candidates is completed by the earlier
//           lane with the later lane's head bytes, the round's last partial dword
//           is carried into the next round in a register);
//   flush   complete 16-B ring blocks -> global_store_dwordx4 (1 KiB per wave
//           instruction, consecutive lanes consecutive addresses).
// Non-FAST words are holes, written by k_expand_slow / k_expand_b.
// ---------------------------------------------------------------------------
#ifndef FX_RING
#define FX_RING 4096  // per-wave linear output staging (bytes)
#endif
                      // during the window setup bytes [16, 16 + 8 FX_WREC) hold the window's
                      // small records (ring block 0 keeps the run's partial block)
#ifndef FX_SWZ
#define FX_SWZ 0      // ring stored XOR-swizzled at 16-B-block granularity inside 128-B bank rows
#endif                // (a5x_ring.h fx7_swz; A/B variant, the ring then starts 1 KiB aligned)
#ifndef FX_BATCH
#define FX_BATCH 0    // flush: all ring reads issued before the stores (A/B variant)
#endif
#ifndef FX_SADDR
#define FX_SADDR 0    // flush stores addressed as scalar base + 32-bit lane offset (A/B variant)
#endif
#ifndef FX_DRAIN
#define FX_DRAIN 0    // diagnostic: s_waitcnt vmcnt(0) after every flush (A/B variant)
#endif
#ifndef FX_GRID
#define FX_GRID 0     // flush store instructions on the output's 128-B line grid (A/B variant)
#endif
#ifndef FX_TRASH
#if FX_SWZ
#define FX_TRASH 0
#else
#define FX_TRASH 256  // (unused gap in front of the ring; keeps the measured LDS layout)
#endif
#endif
// physical ring block of logical block b (FX_SWZ: fx7_swz on a 1 KiB-aligned ring)
__device__ __forceinline__ u32 fx_pb(u32 b) { return FX_SWZ ? b ^ ((b >> 3) & 7u) : b; }
#ifndef FX_WW
#define FX_WW 32      // window words
#endif
#ifndef FX_NBE
#define FX_NBE 256    // big entries per window (16 B each); [FX_ZBE] is the empty piece
#endif
#define FX_ZBE (FX_NBE - 1)
#define FX6_ZBE FX_ZBE
// window records: ring bytes [16, FX_RING) during the setup; the last u64 is the zero slot
#ifndef FX_LALIGN
#define FX_LALIGN 0   // flush whole 128-B output lines only, the rest carried to the ring front (A/B)
#endif
// first ring block of the window records during the setup: behind the carried partial
// block (FX_LALIGN: behind up to 8 carried blocks + the partial one)
#define FX_RBLK (FX_LALIGN ? 9 : 1)
#define FX_RZ ((FX_RING - 16 * FX_RBLK) / 8 - 1)
#ifndef FX_K
#define FX_K 4        // candidates per lane run (a5x_fx6.h)
#endif
#ifndef FX_ABL
#define FX_ABL 0      // timing ablations (variant builds only; output is garbage when set):
                      // 4 no global stores, 8 no rounds, 16 no big entries, 32 no prefix,
                      // 64 no placement ORs, 128 no ring re-zeroing
#endif
#ifndef FX_DABL
#define FX_DABL 0     // fused-digest ablations (variant builds, wrong hits): 1 no MD rounds, 2 no probe
#endif

// The window's small-piece records live in the ring (from byte 16) during the window
// setup (rec[FX_ZSLOT] = 0); the rounds then reuse those bytes as output staging.
struct FXWin {
  uint4 be[FX_NBE];        // big entries: 15 content bytes, length in byte 15
  uint4 wq[FX_WW][2];      // per word (a5x_fx6.h): magics; R - 1 | entry bases | first run
  u32 rb[FX_WW + 4];       // first rank of the word inside the window
  u32 re[FX_WW + 4];       // rank end of the word inside the window
  u32 mag[FB_RMAX + 4];    // fr_magic(R), R <= FB_RMAX
};
static_assert(FW_RMAX < FX_RZ && FB_EMAX < FX_ZBE, "a FAST record must fit a window");
#ifndef FX_WPE
#define FX_WPE 4  // 16 waves per CU: <= 128 VGPRs, <= 10 KiB LDS per wave
#endif
static_assert(FX_RING + FX_TRASH + sizeof(FXWin) <= 163840 / (4 * FX_WPE), "4 FX_WPE waves per CU must fit the 160 KiB of LDS");

// Closed-form bytes of candidates [0, r) of a FAST word (candidate r <-> index r + 1
// in the piece mixed radix, piece 0 least significant).  rec = the word's record
// (LDS).  Wave-collective: lanes over the word's pieces (np <= FW_PMAX).
__device__ u64 fast_prefix_bytes(const u64* rec, u64 r) {
  const u32 lane = lane_id();
  const u32 np = frh_np(rec[0]);
  const u32 Y = (u32)r + 1u;  // <= P <= FW_PMAX_CNT: 32-bit arithmetic throughout
  u32 Rl = 1;
  u64 G = 0;
  if (lane < np) { G = rec[1 + lane]; Rl = frd_R(G); }
  u32 inc = Rl;  // inclusive prefix product of R over pieces (one DPP row: np <= 16)
  inc *= (u32)__builtin_amdgcn_update_dpp(1, (int)inc, 0x111, 0xf, 0xf, false);
  inc *= (u32)__builtin_amdgcn_update_dpp(1, (int)inc, 0x112, 0xf, 0xf, false);
  inc *= (u32)__builtin_amdgcn_update_dpp(1, (int)inc, 0x114, 0xf, 0xf, false);
  inc *= (u32)__builtin_amdgcn_update_dpp(1, (int)inc, 0x118, 0xf, 0xf, false);
  i64 part = 0, base0 = 0;
  if (lane < np) {
    const u64* ent = rec + 1 + np + frd_ebase(G);
    const u32 Q = inc / Rl, full = Y / inc, rem = Y - full * inc;
    const int l0 = (int)fw_len(ent[0]);
    base0 = l0;
    for (u32 v = 1; v < Rl; v++) {
      const u32 lo = v * Q;
      const u32 cnt = full * Q + (rem > lo ? min(Q, rem - lo) : 0u);
      part += (i64)((int)fw_len(ent[v]) - l0) * (i64)cnt;
    }
  }
  // every candidate = the digit-0 piece lengths + deltas
  return (u64)((i64)r * wave_sum_i64(base0) + wave_sum_i64(part));
}

// Staging state of one wave (uniform): ring byte 0 <-> global byte B (16-aligned,
// relative to out_base); bytes [lo, pos) belong to this wave's current run.
struct FxRun {
  u64 B, lo, pos;
  u32 carry;  // bytes [pos & ~3, pos) of the unfinished dword
  bool open;
};

// Stream the complete 16-B blocks of [B, pos) and move the partial last block to
// ring block 0.  The first block of a run may start before lo: byte-exact.
// (nontemporal: the stream is written once; plain stores measured +4-8 % expansion time,
// profiles/r05ce_ab_chunk_stores_occupancy_c3.txt)
#ifndef FX_ST
#define FX_ST 0  // output stores: 0 nontemporal, 1 plain (write-back), 2 sc1 (write-through), 3 the cache-policy
#endif           // bits FX_STPOL ("sc0 nt", ...) -- A/B variants
#ifndef FX_STPOL
#define FX_STPOL "nt"
#endif
__device__ __forceinline__ void fx_store16(uint8_t* p, const uint4 v) {
  typedef u32 v4u __attribute__((ext_vector_type(4)));
  v4u x = {v.x, v.y, v.z, v.w};
  if (FX_ST == 1) *(v4u*)p = x;
  else if (FX_ST == 2) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(x) : "memory");
  else if (FX_ST == 3) asm volatile("global_store_dwordx4 %0, %1, off " FX_STPOL ::"v"(p), "v"(x) : "memory");
  else __builtin_nontemporal_store(x, (v4u*)p);
}

#if FX_LALIGN
// Whole 128-B output lines only: the complete blocks up to the last line boundary are
// stored (every store instruction then starts on a line once the run's first flush has
// reached one) and the rest -- up to 8 blocks + the partial one -- moves to the ring front.
// ALL: every complete block (the run's end).
template <bool ALL = false>
__device__ __forceinline__ void fx_flush(FxRun& R, u32* ring, const ExpArgs& a) {
  const u32 lane = lane_id();
  const u32 nb = uniform((u32)((R.pos - R.B) >> 4));
  if (nb == 0) return;
  const u64 B = uniform64(R.B);
  const u32 nf = ALL ? nb : (u32)(((((B + 16ull * nb) & ~127ull) > B ? ((B + 16ull * nb) & ~127ull) : B) - B) >> 4);
  if (nf == 0) return;
  if (B + 16ull * nf > a.out_cap) { guard_trip(a, 1, B, R.lo, R.pos, a.out_cap); R.B = B + 16ull * nf; return; }
  uint4* r4 = (uint4*)ring;
  const uint4 z = make_uint4(0, 0, 0, 0);
  if (B >= R.lo) {
    for (u32 b = lane; b < nf; b += 64) {
      if (!(FX_ABL & 4)) fx_store16(a.out + B + 16ull * b, r4[b]);
      r4[b] = z;
    }
  } else {
    for (u32 b = lane; b < nf; b += 64) {
      if (!(FX_ABL & 4)) store_block(a, B + 16ull * b, r4[b], R.lo, R.pos);
      r4[b] = z;
    }
  }
  // carry blocks [nf, nb] to [0, nc): all reads before the writes (one instruction each)
  const u32 nc = nb - nf + 1u;  // <= 9
  uint4 t = z;
  if (lane < nc) t = r4[nf + lane];
  WAVE_SYNC();
  if (lane < nc) r4[lane] = t;
  if (lane < nc && nf + lane >= nc) r4[nf + lane] = z;  // sources not overwritten by the carry
  R.B = B + 16ull * nf;
  WAVE_SYNC();
}
#else
template <bool ALL = false>
__device__ __forceinline__ void fx_flush(FxRun& R, u32* ring, const ExpArgs& a) {
  const u32 lane = lane_id();
  const u32 nb = uniform((u32)((R.pos - R.B) >> 4));
  if (nb == 0) return;
  const u64 B = uniform64(R.B);
  if (B + 16ull * nb > a.out_cap) { guard_trip(a, 1, B, R.lo, R.pos, a.out_cap); R.B = B + 16ull * nb; return; }
  uint4* r4 = (uint4*)ring;
  // (OR placement: every flushed block is zeroed again behind its read)
  if (B >= R.lo) {
#if FX_GRID
    // store instructions on the 128-B line grid of the output: instruction i covers the
    // 64 blocks from line (B & ~127) + 1 KiB i; lanes before B or past the flush idle
    const u32 d = (u32)(B >> 4) & 7u;
    for (u32 i = lane; i < nb + d; i += 64) {
      if (i >= d) {
        const u32 b = i - d;
        if (!(FX_ABL & 4)) fx_store16(a.out + B + 16ull * b, r4[fx_pb(b)]);
        if (!(FX_ABL & 128)) r4[fx_pb(b)] = make_uint4(0, 0, 0, 0);
      }
    }
#elif FX_BATCH
    // every ring read of the flush (and the partial block nb) issued before the first wait:
    // one LDS round trip per flush instead of one per KiB (the loop below waits for each
    // read before its store)
    static_assert(FX_RING <= 4096, "batched flush: at most 4 blocks per lane");
    const u32 nq = (nb + 63u) >> 6;  // uniform, 1..4
    uint4 v0, v1 = make_uint4(0, 0, 0, 0), v2 = v1, v3 = v1;
    v0 = r4[fx_pb(min(lane, nb))];  // (clamped: lanes past the flush re-read block nb)
    if (nq > 1) v1 = r4[fx_pb(min(lane + 64u, nb))];
    if (nq > 2) v2 = r4[fx_pb(min(lane + 128u, nb))];
    if (nq > 3) v3 = r4[fx_pb(min(lane + 192u, nb))];
    const uint4 t = r4[fx_pb(nb)];
    uint8_t* o = a.out + B + 16ull * lane;
    if (!(FX_ABL & 4)) {
      if (lane < nb) fx_store16(o, v0);
      if (nq > 1 && lane + 64u < nb) fx_store16(o + 1024, v1);
      if (nq > 2 && lane + 128u < nb) fx_store16(o + 2048, v2);
      if (nq > 3 && lane + 192u < nb) fx_store16(o + 3072, v3);
    }
    // blocks [0, nb] back to zero (nb: the partial block, moved to block 0)
    const uint4 z = make_uint4(0, 0, 0, 0);
    const u32 nz = (nb >> 6) + 1u;  // uniform, 1..4 (nb < FX_RING / 16)
    if (lane <= nb) r4[fx_pb(lane)] = z;
    if (nz > 1 && lane + 64u <= nb) r4[fx_pb(lane + 64u)] = z;
    if (nz > 2 && lane + 128u <= nb) r4[fx_pb(lane + 128u)] = z;
    if (nz > 3 && lane + 192u <= nb) r4[fx_pb(lane + 192u)] = z;
    if (lane == 0) r4[0] = t;  // after lane 0's own zero write of block 0 (a lane's LDS ops stay in order)
    R.B = B + 16ull * nb;
    WAVE_SYNC();
    return;
#elif FX_SADDR
    // scalar base + 32-bit lane offset (global_store ... saddr): 4 B of address per lane to
    // the vector memory pipeline instead of 8
    typedef u32 gv4u __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(1))) gv4u gv4;
    typedef __attribute__((address_space(1))) uint8_t gu8;
    gu8* const ob = (gu8*)(uintptr_t)uniform64((u64)(uintptr_t)(a.out + B));
    for (u32 b = lane; b < nb; b += 64) {
      const uint4 v = r4[fx_pb(b)];
      const gv4u x = {v.x, v.y, v.z, v.w};
      if (!(FX_ABL & 4)) __builtin_nontemporal_store(x, (gv4*)(ob + 16u * b));
      if (!(FX_ABL & 128)) r4[fx_pb(b)] = make_uint4(0, 0, 0, 0);
    }
#else
    for (u32 b = lane; b < nb; b += 64) {
      if (!(FX_ABL & 4)) fx_store16(a.out + B + 16ull * b, r4[fx_pb(b)]);
      if (!(FX_ABL & 128)) r4[fx_pb(b)] = make_uint4(0, 0, 0, 0);
    }
#endif
  } else {
    for (u32 b = lane; b < nb; b += 64) {
      if (!(FX_ABL & 4)) store_block(a, B + 16ull * b, r4[fx_pb(b)], R.lo, R.pos);
      if (!(FX_ABL & 128)) r4[fx_pb(b)] = make_uint4(0, 0, 0, 0);
    }
  }
  if (lane == 0) {
    const uint4 t = r4[fx_pb(nb)];
    r4[fx_pb(nb)] = make_uint4(0, 0, 0, 0);
    r4[0] = t;
  }
#if FX_DRAIN  // (diagnostic A/B: wait for every store of the flush, as the window setup's loads do)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  R.B = B + 16ull * nb;
  WAVE_SYNC();
}
#endif

// flush everything up to pos (tail block byte-exact)
__device__ __forceinline__ void fx_close(FxRun& R, u32* ring, const ExpArgs& a) {
  if (!R.open) return;
  fx_flush<true>(R, ring, a);
  if (R.pos > R.B && lane_id() == 0) {  // (block 0 is physical block 0 under FX_SWZ too)
    store_block(a, R.B, ((const uint4*)ring)[0], max(R.lo, R.B), R.pos);
    ((uint4*)ring)[0] = make_uint4(0, 0, 0, 0);
  }
  WAVE_SYNC();
  R.open = false;
}

#define FX6_KMAX FX_K
#define FX6_SWZ FX_SWZ
#define FX6_ABL FX_ABL
#include "a5x_fx6.h"
#include "a5x_md.h"

// Window metadata of words w .. w + FX_WW - 1 (lane j <-> word w + j, same keyspace
// tile), all loads issued together.  (No prefetch across the rounds: the registers it
// holds cost a wave per SIMD, and occupancy hides these loads better.)
struct FxMeta {
  u64 c0, c1, bo;
  u32 fl, roff;
};
__device__ __forceinline__ FxMeta fx_meta(const ExpArgs& a, u64 w) {
  const u32 lane = lane_id();
  const u64 wl = w + lane;
  const bool inb = lane < FX_WW && wl < a.nw && wl / FW_TILE == w / FW_TILE;
  FxMeta m;
  m.c0 = inb ? a.cand_off[wl] : ~0ull;
  m.c1 = inb ? a.cand_off[wl + 1] : ~0ull;
  m.fl = inb ? a.flags[wl] : 0u;
  m.roff = inb ? a.roff[wl] : 0u;
  m.bo = (lane == 0 && w < a.nw) ? a.byte_off[w] : 0;
  return m;
}

// ring flush for a5x_fx6.h rounds
struct FxFlush {
  static constexpr bool DIGEST = false;
  u32* ring;
  const ExpArgs* a;
  u64 wbase;
  __device__ __forceinline__ void operator()(FxRun& R) { fx_flush(R, ring, *a); }
  __device__ __forceinline__ void digest(const FxLaneRun&) {}
};

// Fused digest (main.go:66's candidates hashed where they are built):
// after a round's placement every lane MD5s its run's candidates straight out of the
// LDS ring and probes the target set; nothing goes to HBM but the hits, which carry
// (word, candidate in word) directly.  The ring is then zeroed for the next round.
template <bool MD5>
struct FxDigest {
  static constexpr bool DIGEST = true;
  u32* ring;
  const ExpArgs* a;
  u64 wbase;  // global index of window word 0
  __device__ __forceinline__ void operator()(FxRun& R) {
    const u32 lane = lane_id();
    const u32 nb = (u32)(R.pos - R.B + 31u) / 16u;  // the round's bytes + the ORs' zero overhang
    for (u32 b = lane; b < nb; b += 64) ((uint4*)ring)[b] = make_uint4(0, 0, 0, 0);
    R.B = R.pos = R.lo = 0;
    WAVE_SYNC();
  }
  __device__ __forceinline__ void digest(const FxLaneRun& lr) {
    const uint8_t* base = (const uint8_t*)ring;
    u32 off = lr.off;
#pragma unroll 1
    for (u32 c = 0; c < FX6_KMAX; c++) {
      u32 l = lr.clen[0];
#pragma unroll
      for (u32 q = 1; q < FX6_KMAX; q++) l = c == q ? lr.clen[q] : l;
      const bool on = c < lr.nc;
      if (!__builtin_amdgcn_ballot_w64(on)) break;  // runs are filled from candidate 0
      u32 d[4];
#if FX_DABL & 1  // (ablation: no MD rounds -- a cheap stand-in digest)
      d[0] = off * 0x9E3779B9u + l; d[1] = d[0] ^ 0x85EBCA6Bu; d[2] = d[0] * 3u; d[3] = d[1] + c;
#else
      if constexpr (MD5) md_lds<true>(base, off, on ? l - 1u : 0u, d);  // the candidate without its '\n'
      else ntlm_lds(base, off, on ? l - 1u : 0u, d);
#endif
#if FX_DABL & 2  // (ablation: no target probe -- the digest kept live by a never-true test)
      const bool hit = (d[0] ^ d[1] ^ d[2] ^ d[3]) == 0x7A5A5A5Au && d[0] == 0x13579BDFu;
#else
      const bool hit = md_probe(a->dg_bitmap, a->dg_bm_mask, a->dg_table, a->dg_tmask, a->dg_has_zero != 0, d);
#endif
      if (on && hit) {
        const u32 h = atomicAdd(a->dg_nhits, 1u);
        if (h < a->dg_hit_cap) {
          A5xHitRaw r;
          hit_word(*a, wbase + lr.j, lr.st + c, r);
          r.d[0] = d[0]; r.d[1] = d[1]; r.d[2] = d[2]; r.d[3] = d[3];
          a->dg_hits[h] = r;
        }
      }
      off += l;
    }
  }
};

// ---------------------------------------------------------------------------
// Fused digest with one candidate per 64-B message slot (windows whose candidates fit
// one MD block, FXD_MAXL bytes with the '\n'): lane L's candidate is OR-placed at ring
// byte 64 L and its '\n' turned into the 0x80 pad byte (one ds_xor), so the slot IS the
// MD5 / MD4 message block -- four 16-B LDS reads, no per-word keep / pad masks, the bit
// length in M[14].  NTLM windows carry big entries already converted to UTF-16LE
// (fx_utf16_entry), so the slot holds the UTF-16LE message and MD4 runs on it directly;
// the UTF-8 walk of ntlm_stream is left to windows that cannot take the slots.
// ---------------------------------------------------------------------------
#define FXD_MAXL 56u  // slot path: candidate + '\n' (NTLM: UTF-16LE bytes + "\n\0") <= 56 B
#ifndef FXD_NWSPEC
#define FXD_NWSPEC 1  // slot rounds specialised by the window's message words (8 / 12 / 14)
#endif


// One rune of Go's utf8.DecodeRune from the 4 bytes x (avail of them belong to the
// string): r, its byte size sz (invalid: U+FFFD, 1 byte), cut = a valid lead byte whose
// sequence runs past the available bytes (decoded here it differs from the decoding in
// the longer string).
__device__ __forceinline__ void utf8_rune(u32 x, u32 avail, u32& r, u32& sz, bool& cut) {
  const u32 b0 = x & 255u, b1 = (x >> 8) & 255u, b2 = (x >> 16) & 255u, b3 = x >> 24;
  r = b0; sz = 1; cut = false;
  if (b0 < 0x80u) return;
  r = 0xFFFDu;
  u32 size = 0, lo = 0x80u, hi = 0xBFu;
  if (b0 >= 0xC2u && b0 <= 0xDFu) size = 2;
  else if (b0 >= 0xE0u && b0 <= 0xEFu) { size = 3; lo = b0 == 0xE0u ? 0xA0u : 0x80u; hi = b0 == 0xEDu ? 0x9Fu : 0xBFu; }
  else if (b0 >= 0xF0u && b0 <= 0xF4u) { size = 4; lo = b0 == 0xF0u ? 0x90u : 0x80u; hi = b0 == 0xF4u ? 0x8Fu : 0xBFu; }
  cut = size > avail;
  const bool c2 = b2 >= 0x80u && b2 <= 0xBFu, c3 = b3 >= 0x80u && b3 <= 0xBFu;
  if (size && size <= avail && b1 >= lo && b1 <= hi && (size < 3 || c2) && (size < 4 || c3)) {
    sz = size;
    r = size == 2 ? ((b0 & 0x1Fu) << 6) | (b1 & 0x3Fu)
      : size == 3 ? ((b0 & 0x0Fu) << 12) | ((b1 & 0x3Fu) << 6) | (b2 & 0x3Fu)
                  : ((b0 & 0x07u) << 18) | ((b1 & 0x3Fu) << 12) | ((b2 & 0x3Fu) << 6) | (b3 & 0x3Fu);
  }
}

// A big entry (<= 15 UTF-8 bytes) as UTF-16LE (Go []rune + utf16.Encode of the piece).
// The candidate's UTF-16LE is the concatenation of its pieces' when no piece ends inside
// a rune: ok = false for an entry cut inside a rune or longer than 15 bytes as UTF-16LE.
__device__ __forceinline__ uint4 fx_utf16_entry(const uint4 e, bool& ok) {
  typedef unsigned __int128 u128;
  u128 in = (u128)((u64)e.x | ((u64)e.y << 32)) | ((u128)((u64)e.z | ((u64)(e.w & 0xFFFFFFu) << 32)) << 64);
  const u32 n = e.w >> 24;
  u128 out = 0;
  u32 i = 0, o = 0;
  bool good = true;
  for (u32 it = 0; it < 15u && i < n; it++) {
    u32 r, sz;
    bool cut;
    utf8_rune((u32)in, n - i, r, sz, cut);
    good = good && !cut;
    if (r >= 0x10000u) {
      const u32 v = r - 0x10000u;
      const u32 pair = (0xD800u + (v >> 10)) | ((0xDC00u + (v & 0x3FFu)) << 16);
      if (o < 16u) out |= (u128)pair << (8u * o);
      o += 4;
    } else {
      if (o < 16u) out |= (u128)r << (8u * o);
      o += 2;
    }
    in >>= 8u * sz;
    i += sz;
  }
  ok = good && o <= 15u;
  const u64 lo = (u64)out, hi = (u64)(out >> 64);
  return make_uint4((u32)lo, (u32)(lo >> 32), (u32)hi, ((u32)(hi >> 32) & 0xFFFFFFu) | ((o <= 15u ? o : 0u) << 24));
}

// One round of the slot path: lane L < nr takes window candidate rr + L (one candidate
// per run), places it at ring + 64 L, hashes the slot and probes the target set.  NW:
// message words that can be non-zero (the window's longest message, with its pad byte,
// fits 4 NW bytes): words NW .. 13 are compile-time zeros, so their MD adds fold away
// and their slot quads are neither read nor cleared.
template <int NB, bool MD5, int NW>
__device__ __forceinline__ void fxd_round(const uint4* be, const uint4 (*wq)[2], const u32* rb, const u32* re, u32 ring,
                                          u32 rr, u32 j, bool act, const ExpArgs& a, u64 wbase) {
  const u32 lane = lane_id();
  const uint4 q0 = wq[j][0], q1 = wq[j][1];
  const u32 st = act ? rr + lane - q1.w + rb[j] : 0u;  // the candidate's rank in its word
  const bool on = act && st < re[j];
  u32 d[4];
  fx6_digits<NB>(st + 1u, q0, q1.x, d);
  uint4 ent[NB];
  u32 len = 0;
#pragma unroll
  for (int b = 0; b < NB; b++) {
    ent[b] = be[on ? fx6_eb(q1, b) + d[b] : (u32)FX6_ZBE];
    len += ent[b].w >> 24;
  }
  const u32 slot = ring + 64u * lane;
  u32 P = slot;
#pragma unroll
  for (int b = 0; b < NB; b++) fx7_put(ent[b], P);
  constexpr u32 TL = MD5 ? 1u : 2u;  // the '\n' ("\n\0" in UTF-16LE) becomes the 0x80 pad
  if (on) {
    const u32 pb = slot + len - TL;
    fx7_xor(pb & ~3u, 0x8Au << (8u * (pb & 3u)));
  }
  WAVE_SYNC();
  static_assert(NW == 8 || NW == 12 || NW == 14, "message word classes");
  constexpr int NQ = (NW + 3) / 4;  // slot quads that can hold message bytes
  u32 M[16];
#pragma unroll
  for (int q = 0; q < NQ; q++) {
    const uint4 v = fx6_ld16(slot + 16u * q);
    M[4 * q] = v.x; M[4 * q + 1] = v.y; M[4 * q + 2] = v.z; M[4 * q + 3] = v.w;
  }
#pragma unroll
  for (int q = NW; q < 14; q++) M[q] = 0u;
  M[14] = on ? (len - TL) << 3 : 0u;
  M[15] = 0u;
#pragma unroll
  for (int q = 0; q < NQ; q++) fx6_st16(slot + 16u * q, make_uint4(0, 0, 0, 0));  // zero again for the next round
  u32 h[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
#if FX_DABL == 0
  // (early rejection: a wave whose candidates all miss the prefilter on digest words 0 / 3
  // skips the last two MD steps and the table probe -- md_block_probe)
  const bool hit = md_block_probe<MD5>(M, on, a.dg_bitmap, a.dg_bm_mask, a.dg_table, a.dg_tmask, a.dg_has_zero != 0, h);
#else
#if FX_DABL & 1
  h[0] ^= M[0] + M[14]; h[1] ^= M[1]; h[2] ^= M[2]; h[3] ^= M[3];
#else
  if constexpr (MD5) md5_block(h, M);
  else md4_block(h, M);
#endif
#if FX_DABL & 2
  const bool hit = (h[0] ^ h[1] ^ h[2] ^ h[3]) == 0x7A5A5A5Au && h[0] == 0x13579BDFu;
#else
  const bool hit = md_probe(a.dg_bitmap, a.dg_bm_mask, a.dg_table, a.dg_tmask, a.dg_has_zero != 0, h);
#endif
#endif
  if (on && hit) {
    const u32 k = atomicAdd(a.dg_nhits, 1u);
    if (k < a.dg_hit_cap) {
      A5xHitRaw r;
      hit_word(a, wbase + j, st, r);
      r.d[0] = h[0]; r.d[1] = h[1]; r.d[2] = h[2]; r.d[3] = h[3];
      a.dg_hits[k] = r;
    }
  }
  WAVE_SYNC();
}

// The window's candidates (T of them) in rounds of 64 on the slot path.
template <bool MD5, int NW>
__device__ __forceinline__ void fxd_rounds(FXWin& F, u32* ring, const ExpArgs& a, u64 wbase, u32 T, u32 k, u32 rw,
                                           u64 m2, u64 m3, u64 m4) {
  const u32 lane = lane_id();
  const u32 ringa = fx6_addr(ring);
  u32 jcur = 0;
  for (u32 rr = 0; rr < T; rr += 64u) {
    const u32 nr = min(64u, T - rr);
    const u32 j = fx6_word(rw, k, rr, nr, jcur);
    const bool act = lane < nr;
    const u32 jl = readlane_u32(j, nr - 1u);
    const u64 span = ((2ull << (jl - jcur)) - 1ull) << jcur;  // words jcur .. jl
    if (span & m4) fxd_round<4, MD5, NW>(F.be, F.wq, F.rb, F.re, ringa, rr, j, act, a, wbase);
    else if (span & m3) fxd_round<3, MD5, NW>(F.be, F.wq, F.rb, F.re, ringa, rr, j, act, a, wbase);
    else if (span & m2) fxd_round<2, MD5, NW>(F.be, F.wq, F.rb, F.re, ringa, rr, j, act, a, wbase);
    else fxd_round<1, MD5, NW>(F.be, F.wq, F.rb, F.re, ringa, rr, j, act, a, wbase);
  }
}

// The window's rounds: T runs of K candidates, nl runs per round; each round takes
// the largest big-piece count among the words it spans (m2 / m3 / m4: window words
// with >= 2 / 3 / 4 big pieces).
template <int K, class FL>
__device__ __forceinline__ void fx_rounds(FXWin& F, u32* ring, FxRun& R, FL& fl, u32 T, u32 k, u32 rw, u64 m2,
                                          u64 m3, u64 m4) {
  const u32 lane = lane_id();
  const u32 ringa = fx6_addr(ring);
  const u32 cap = FX_RING - 32u;
  u32 jcur = 0;
  for (u32 rr = 0; rr < T;) {
    const u32 nr = min(64u, T - rr);
    const u32 j = fx6_word(rw, k, rr, nr, jcur);
    const bool act = lane < nr;
    const u32 jl = readlane_u32(j, nr - 1u);
    const u64 span = ((2ull << (jl - jcur)) - 1ull) << jcur;  // words jcur .. jl
    u32 took;
    FxLaneRun lr;
    if (span & m4) took = fx7_round<4, K>(F.be, F.wq, F.rb, F.re, ringa, cap, R, rr, j, act, fl, lr);
    else if (span & m3) took = fx7_round<3, K>(F.be, F.wq, F.rb, F.re, ringa, cap, R, rr, j, act, fl, lr);
    else if (span & m2) took = fx7_round<2, K>(F.be, F.wq, F.rb, F.re, ringa, cap, R, rr, j, act, fl, lr);
    else took = fx7_round<1, K>(F.be, F.wq, F.rb, F.re, ringa, cap, R, rr, j, act, fl, lr);
    if constexpr (FL::DIGEST) {
      fl.digest(lr);
      fl(R);
    }
    rr += took;
  }
}

// Big entry (a5x_plan.h fb_entry, same bytes): combination c of the span <= FB_SPAN small
// pieces whose descriptors are rec[d0 ..], entries rec[wbe ..]; the loop runs smax
// (wave-uniform) iterations instead of FB_SPAN.
//
// Three LDS trips per entry, not two per small piece: every descriptor read is issued
// at once, the digits are a VALU chain, then every small entry read is issued at once
// (the descriptors do not depend on the digits; read in turn, each piece waited for
// its descriptor and then its entry, s_waitcnt lgkmcnt(0) each: 2 smax serial trips).
__device__ __forceinline__ uint4 fx_entry(const u64* rec, u32 d0, u32 wbe, u32 span, u32 smax, u32 c) {
  u64 lo64 = 0, hi64 = 0;
  u32 off = 0;
  u64 G[FB_SPAN], EV[FB_SPAN];
#pragma unroll
  for (u32 i = 0; i < FB_SPAN; i++)
    if (i < smax) G[i] = rec[i < span ? d0 + i : (u32)FX_RZ];
  u32 ei[FB_SPAN];
#pragma unroll
  for (u32 i = 0; i < FB_SPAN; i++) {
    if (i < smax) {
      const u32 ghi = (u32)(G[i] >> 32);
      u32 q = __umulhi(c, (u32)G[i]);
      q += c & (u32)((int)ghi >> 31);  // R = 1: q = c
      const u32 d = c - q * (((ghi >> 8) & 31u) + 1u);
      c = q;
      ei[i] = i < span ? wbe + (ghi & 255u) + d : (u32)FX_RZ;
    }
  }
#pragma unroll
  for (u32 i = 0; i < FB_SPAN; i++)
    if (i < smax) EV[i] = rec[ei[i]];
#pragma unroll
  for (u32 i = 0; i < FB_SPAN; i++) {
    if (i >= smax) break;
    const u64 ev = EV[i];
    const u64 cv = ev & FW_M56;
    const u32 sh = 8u * off;
    const u64 x = cv << (sh & 63u), y = cv >> ((64u - sh) & 63u);
    lo64 |= off < 8u ? x : 0ull;
    hi64 |= off < 8u ? (off ? y : 0ull) : x;
    off += fw_len(ev);
  }
  return make_uint4((u32)lo64, (u32)(lo64 >> 32), (u32)hi64, ((u32)(hi64 >> 32) & 0xFFFFFFu) | (off << 24));
}

// DIG: 0 = write the stream, 1 = fused MD5, 2 = fused NTLM
template <int DIG>
__device__ __forceinline__ void expand_chunk_fast(FXWin& F, u32* ring, const ExpArgs& a, u64 chunk) {
  const u32 lane = lane_id();
  u64* const rec = (u64*)(ring + 4 * FX_RBLK);  // ring bytes [16 FX_RBLK, 16 FX_RBLK + 8 FX_WREC)
  const u64 g0 = max(a.cand_begin, chunk * a.CH);
  const u64 g1 = min(a.cand_end, (chunk + 1) * a.CH);
  if (g0 >= g1) return;
  u64 w = a.chunk_w0[chunk];
  if (w >= a.nw) { guard_trip(a, 2, chunk, w, g0, a.nw); return; }
  while (w < a.nw && a.cand_off[w + 1] <= g0) w++;
  if (w >= a.nw) { guard_trip(a, 3, chunk, w, g0, a.nw); return; }
  if (lane == 0) F.be[FX_ZBE] = make_uint4(0, 0, 0, 0);
  for (u32 i = lane; i < FX_RING / 16; i += 64) ((uint4*)ring)[i] = make_uint4(0, 0, 0, 0);
  F.mag[lane] = fr_magic(lane);
  if (lane == 0) F.mag[FB_RMAX] = fr_magic(FB_RMAX);
  u64 g = g0;
  FxRun R;
  R.open = false; R.B = 0; R.lo = 0; R.pos = 0; R.carry = 0;
  typename std::conditional<DIG != 0, FxDigest<DIG == 1>, FxFlush>::type fl;
  fl.ring = ring; fl.a = &a; fl.wbase = 0;
  FxMeta M = fx_meta(a, w);
  STAMP_DECL
  while (g < g1) {
    if (w >= a.nw) { guard_trip(a, 4, chunk, w, g, g1); break; }
    // ---- window: lane j <-> word w + j ----
    const u64 c0 = M.c0, c1 = M.c1;
    const u32 fl_ = M.fl;
    const bool hasc = c1 > c0 && c0 != ~0ull;
    const bool fast = (fl_ & A5X_WF_FAST) && c0 < g1;
    const u32 rs = (fast && hasc) ? ff_rsize(fl_) : 0u;
    const u32 incR = wave_incl_scan_u32(rs);
    // records must be one contiguous range (complex words have slots elsewhere; a
    // gathered per-word copy that let them join windows measured 8.81 vs 8.65 ms on C3)
    const u64 rm = __ballot(rs > 0);
    const u32 rbase = readlane_u32(M.roff, rm ? (u32)__builtin_ctzll(rm) : 0u);
    const bool contig = rs == 0 || M.roff == rbase + (incR - rs);
    const bool ok = fast && incR + 1u < FX_RZ && contig;  // (+1: the copy's alignment shift)
    const u64 badm = __ballot(!ok);
    u32 k = badm ? (u32)__builtin_ctzll(badm) : 64u;
    STAMP(0);
    if (k == 0) {  // (A/B: one hole word per step)
      const u64 w0c1 = uniform64(c1);
      if (w0c1 > g && w0c1 != ~0ull) {
        if (!DIG) fx_close(R, ring, a);
        g = min(w0c1, g1);
      }
      w++;
      M = fx_meta(a, w);
      continue;
    }
    // ---- small records -> LDS (one contiguous range) ----
    const u64 fm = __ballot(lane < k && rs > 0);
    if (fm == 0) {  // only words without candidates: skip them
      w += k;
      M = fx_meta(a, w);
      continue;
    }
    const u32 jf = (u32)__builtin_ctzll(fm);
    const u64 src0 = (u64)readlane_u32(M.roff, jf);
    const u32 ntot = readlane_u32(incR, k - 1);
    // Every load of the copy issued before the first LDS store: one global round trip
    // (a load-store loop waited vmcnt(0) per KiB -- a trip each, and each behind the
    // wave's outstanding output stores, which share the counter).  16-B loads from the
    // aligned-down source: record u64 src0 lands at rec[sh].
    const u32 sh = (u32)(src0 & 1u);
    {
      static_assert((FX_RZ + 1) / 2 <= 4 * 64, "window records: at most 4 uint4 per lane");
      const uint4* src = (const uint4*)(a.rec + (src0 - sh));
      const u32 nq = (ntot + sh + 1u) / 2u;
      // (clamped, unconditional loads: the excess lanes re-read the last quad)
      const u32 nq1 = nq - 1u;
      const uint4 v0 = src[min(lane, nq1)], v1 = src[min(lane + 64u, nq1)];
      const uint4 v2 = src[min(lane + 128u, nq1)], v3 = src[min(lane + 192u, nq1)];
      uint4* r4 = (uint4*)rec;
      if (lane < nq) r4[lane] = v0;
      if (lane + 64u < nq) r4[lane + 64u] = v1;
      if (lane + 128u < nq) r4[lane + 128u] = v2;
      if (lane + 192u < nq) r4[lane + 192u] = v3;
    }
    const u32 rb = incR - rs + sh;
    const u64 bo = M.bo;
    if (lane == 0) rec[FX_RZ] = 0;
    WAVE_SYNC();
    STAMP(4);
    // ---- big pieces per word: R = product of the spanned small R ----
    u64 hdr = 0;
    u32 nbw = 0, R0 = 1, R1 = 1, R2 = 1, R3 = 1;
    if (lane < k && rs) {
      hdr = rec[rb];
      nbw = frh_nbig(hdr);
      R0 = frh_R(hdr, 0);
      R1 = frh_R(hdr, 1);
      R2 = frh_R(hdr, 2);
      R3 = frh_R(hdr, 3);
    }
    const u32 E = R0 + R1 + R2 + R3 - (FB_NMAX - nbw);  // fb_R = 1 past the last big piece
    const u32 incE = wave_incl_scan_u32(E);
    const u64 over = __ballot(lane < k && incE > FX_ZBE);
    if (over) k = (u32)__builtin_ctzll(over);  // the window ends where the big entries do not fit
    if (k == 0) { guard_trip(a, 6, chunk, w, E, incE); break; }
    const bool inw = lane < k;
    const u32 maxl = inw ? frh_maxl(hdr) : 0u;
    const u32 winmax = wave_max_u32(maxl);
    const u64 m2 = __ballot(inw && nbw >= 2), m3 = __ballot(inw && nbw >= 3), m4 = __ballot(inw && nbw >= 4);
    const u32 ebase = incE - E;
    // ---- per-word info: magics, R - 1, entry bases (pieces past the count: R 1, the
    // empty entry), the word's ranks inside [g, g1) and its runs ----
    // candidates per run: a round always takes at least one run (K (longest) <= ring);
    // the fused digest's slot path (fxd_rounds): one candidate per run
    bool dslot = false;
    if constexpr (DIG != 0) dslot = (DIG == 1 ? winmax : 2u * winmax) <= FXD_MAXL;
    u32 K = dslot ? 1u : (FX_K * winmax + 16u <= FX_RING - 32u ? FX_K : 1u);
    const u64 wc0 = uniform64(c0);
    const u32 rbw = lane == 0 ? (u32)(g - wc0) : 0u;
    const u32 rew = inw ? (u32)(min(c1, g1) - c0) : 0u;
    u32 nrun = inw && rs ? (rew - rbw + K - 1u) / K : 0u;
    u32 incr = wave_incl_scan_u32(nrun);
    u32 rw = inw ? incr - nrun : 0xffffffffu;
    u32 T = readlane_u32(incr, k - 1);
    if (inw) {
      const u32 b1 = ebase + R0, b2 = b1 + R1, b3 = b2 + R2;
      const u32 e1 = nbw > 1 ? b1 : (u32)FX_ZBE, e2 = nbw > 2 ? b2 : (u32)FX_ZBE, e3 = nbw > 3 ? b3 : (u32)FX_ZBE;
      const u32 rmk = (R0 - 1u) | ((R1 - 1u) << 6) | ((R2 - 1u) << 12) | ((R3 - 1u) << 18);
      F.wq[lane][0] = make_uint4(F.mag[R0], F.mag[R1], F.mag[R2], F.mag[R3]);
      F.wq[lane][1] = make_uint4(rmk, (nbw ? ebase : (u32)FX_ZBE) | (e1 << 16), e2 | (e3 << 16), rw);
      F.rb[lane] = rbw;
      F.re[lane] = rew;
    }
    WAVE_SYNC();
    STAMP(5);
    // ---- build the big entries: lanes over the window's entries (conv: as UTF-16LE, the
    // NTLM slot path; returns whether an entry could not be converted) ----
    auto build_entries = [&](bool conv) -> bool {
      bool bad = false;
      const u32 etot = readlane_u32(incE, k - 1);
      const u32 est = lane < k ? ebase : 0xffffffffu;
      u32 jb = 0;  // word of the pass's first entry (uniform)
      for (u32 t0 = 0; t0 < etot; t0 += 64) {
        const u32 t = t0 + lane;
        u32 j = jb;
        for (;;) {
          const u32 jn = uniform(jb + 1);
          if (jn >= k) break;
          const u32 sj = uniform(readlane_u32(est, jn));
          if (sj >= t0 + 64) break;
          jb = jn;
          j += (t >= sj) ? 1u : 0u;
        }
        // (cross-lane reads with every lane active: a bpermute from an inactive lane is garbage)
        const u32 wrb = (u32)__shfl((int)rb, (int)j);
        const u32 u = t - (u32)__shfl((int)ebase, (int)j);
        const u32 nbj = (u32)__shfl((int)nbw, (int)j);
        const bool on = t < etot;
        // big piece b of word j holding entry u, the combination c, its small pieces
        const uint4 q1 = F.wq[on ? j : 0][1];
        const u32 b0 = q1.y & 0xFFFFu;
        const u32 s1 = (q1.y >> 16) - b0, s2 = (q1.z & 0xFFFFu) - b0, s3 = (q1.z >> 16) - b0;
        u32 b = 0, cb = 0;
        if (nbj > 1 && u >= s1) { b = 1; cb = s1; }
        if (nbj > 2 && u >= s2) { b = 2; cb = s2; }
        if (nbj > 3 && u >= s3) { b = 3; cb = s3; }
        const u64 h = rec[on ? wrb : (u32)FX_RZ];
        const u32 np = frh_np(h), nbh = frh_nbig(h);
        const u32 sp0 = frh_bstart(h, b), sp1 = b + 1 < nbh ? frh_bstart(h, b + 1) : np;
        const u32 span = on ? sp1 - sp0 : 0u;
        uint4 e = fx_entry(rec, wrb + 1u + sp0, wrb + 1u + np, span, wave_max_u32(span), u - cb);
        if (DIG == 2 && conv) {
          bool ok = true;
          e = fx_utf16_entry(e, ok);
          bad = bad || (on && !ok);
        }
        if (on) F.be[t] = e;
      }
      return wave_or_u32(bad ? 1u : 0u) != 0u;
    };
    if (!(FX_ABL & 16) && build_entries(DIG == 2 && dslot)) {
      // an entry cut inside a rune (or too long as UTF-16LE): UTF-8 entries, K-candidate runs
      WAVE_SYNC();
      dslot = false;
      (void)build_entries(false);
      K = FX_K * winmax + 16u <= FX_RING - 32u ? FX_K : 1u;
      nrun = inw && rs ? (rew - rbw + K - 1u) / K : 0u;
      incr = wave_incl_scan_u32(nrun);
      rw = inw ? incr - nrun : 0xffffffffu;
      T = readlane_u32(incr, k - 1);
      if (inw) F.wq[lane][1].w = rw;
    }
    WAVE_SYNC();
    STAMP(1);
    // ---- run position of g (the fused digest writes nothing: its ring restarts at 0) ----
    if (!DIG) {
      const u64 r0 = g - wc0;
      u64 pos = uniform64(bo) - a.out_base;
      if (!(FX_ABL & 32))
      if (r0) pos += fast_prefix_bytes(rec + readlane_u32(rb, 0), r0);
      if (!R.open || R.pos != pos) {
        fx_close(R, ring, a);
        R.B = pos & ~15ull; R.lo = pos; R.pos = pos; R.carry = 0; R.open = true;
      }
    }
    fl.wbase = w;
    // the records' ring bytes [16, 16 + 8 ntot) back to zero for the OR rounds
    for (u32 i = FX_RBLK + lane; i < FX_RBLK + (ntot + sh + 2) / 2; i += 64) ((uint4*)ring)[i] = make_uint4(0, 0, 0, 0);
    WAVE_SYNC();
    STAMP(2);
    // the next window's metadata, loaded under this window's rounds (the window's own
    // metadata registers are dead from here on)
    const u64 gnext = min(g1, uniform64(shfl_u64(c1, (int)k - 1)));
    M = fx_meta(a, w + k);
    // ---- rounds ----
    if (!(FX_ABL & 8))
    {
      if (DIG != 0 && dslot) {
        // message bytes of the window's longest candidate ('\n' -> pad; NTLM: UTF-16LE)
        const u32 mb = FXD_NWSPEC ? (DIG == 1 ? winmax : 2u * winmax) : FXD_MAXL;
        if (mb <= 32u) fxd_rounds<DIG == 1, 8>(F, ring, a, w, T, k, rw, m2, m3, m4);
        else if (mb <= 48u) fxd_rounds<DIG == 1, 12>(F, ring, a, w, T, k, rw, m2, m3, m4);
        else fxd_rounds<DIG == 1, 14>(F, ring, a, w, T, k, rw, m2, m3, m4);
      }
      else if (K == FX_K) fx_rounds<FX_K>(F, ring, R, fl, T, k, rw, m2, m3, m4);
      else fx_rounds<1>(F, ring, R, fl, T, k, rw, m2, m3, m4);
    }
    STAMP(3);
    g = gnext;
    w += k;
    WAVE_SYNC();
  }
  if (!DIG) fx_close(R, ring, a);
  STAMP(6);
  STAMP_FLUSH();
}

__device__ __forceinline__ u32 lds_per_wave_fast() { return (FX_RING + FX_TRASH + (u32)sizeof(FXWin) + 15u) & ~15u; }

template <int DIG>
__device__ __forceinline__ void expand_fast_body(const ExpArgs& a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const u32 wv = threadIdx.x / 64, nwv = blockDim.x / 64;
  uint8_t* mine = smem + wv * lds_per_wave_fast();
  u32* ring = (u32*)(mine + FX_TRASH);
  FXWin& F = *(FXWin*)(mine + FX_TRASH + FX_RING);
  const u64 chunk = a.cand_begin / a.CH + (u64)blockIdx.x * nwv + wv;
  if (chunk * a.CH >= a.cand_end) return;
  if (FX_SWZ && DIG == 0 && (fx6_addr(ring) & 1023u)) { guard_trip(a, 7, fx6_addr(ring), 0, 0, 0); return; }
  expand_chunk_fast<DIG>(F, ring, a, chunk);
}

__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(FX_WPE))) k_expand_fast(ExpArgs a) {
  expand_fast_body<0>(a);
}

// the same chunks, hashed (MD5) and probed in the ring instead of written (FxDigest)
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(FX_WPE))) k_expand_fast_md5(ExpArgs a) {
  expand_fast_body<1>(a);
}

// the same chunks, NTLM (MD4 over Go's UTF-16LE of each candidate, converted as the
// message blocks are filled) hashed and probed in the ring
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(FX_WPE))) k_expand_fast_ntlm(ExpArgs a) {
  expand_fast_body<2>(a);
}

// k_expand_slow / k_expand_b: one k_segments item (a slow or BIG word's run of <= CH
// candidates inside the call's range) per wave, through wave_setup.
template <int LMAX, int MLMAX, int DPENT, u32 RING>
__device__ void expand_segment(WaveLds<LMAX, MLMAX, DPENT>& S, u32* ring, const Tab& T, const ExpArgs& a, u64 item) {
  const u64 w = (u32)item, s = item >> 32;
  if (w >= a.nw) { guard_trip(a, 2, item, w, s, a.nw); return; }
  const u64 c0 = a.cand_off[w], c1 = a.cand_off[w + 1];
  const u64 lo = max(a.cand_begin, c0) + s * a.SEG;
  const u64 hi = min(min(a.cand_end, c1), lo + a.SEG);
  if (lo >= hi) { guard_trip(a, 3, item, w, lo, hi); return; }
  Run R;
  R.open = false;
  expand_word<LMAX, MLMAX, DPENT, RING>(S, ring, T, a, R, w, lo - c0, hi - lo, c1 - c0);
  run_close<RING>(R, ring, a);
}

__device__ __forceinline__ u32 lds_per_wave_slow() { return (A5X_RING_A + (u32)sizeof(LdsA) + 15u) & ~15u; }

__global__ void __launch_bounds__(256) k_expand_slow(ExpArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const u32 wv = threadIdx.x / 64, nwv = blockDim.x / 64;
  if (blockIdx.x * nwv >= *a.nsegs) return;  // idle workgroup (uniform): release its LDS at once
  load_table(smem, a.table, a.table_bytes);
  const u32 tb = (a.table_bytes + 15u) & ~15u;
  uint8_t* mine = smem + tb + wv * lds_per_wave_slow();
  u32* ring = (u32*)mine;
  LdsA& S = *(LdsA*)(mine + A5X_RING_A);
  for (u32 i = lane_id(); i < A5X_RING_A / 16; i += 64) ((uint4*)ring)[i] = make_uint4(0, 0, 0, 0);
  __syncthreads();
  const Tab T = tab_view(smem);
  const u32 n = *a.nsegs;
  for (u32 i = blockIdx.x * nwv + wv; i < n; i += gridDim.x * nwv)
    expand_segment<A5X_LMAX_A, A5X_MLMAX_A, A5X_DPENT_A, A5X_RING_A>(S, ring, T, a, a.segs[i]);
}

__global__ void __launch_bounds__(64) k_expand_b(ExpArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  if (blockIdx.x >= *a.nsegs) return;  // idle workgroup: release its 160 KB of LDS at once
  load_table(smem, a.table, a.table_bytes);
  const u32 tb = (a.table_bytes + 15u) & ~15u;
  u32* ring = (u32*)(smem + tb);
  LdsB& S = *(LdsB*)(smem + tb + A5X_RING_B);
  for (u32 i = lane_id(); i < A5X_RING_B / 16; i += 64) ((uint4*)ring)[i] = make_uint4(0, 0, 0, 0);
  __syncthreads();
  const Tab T = tab_view(smem);
  const u32 n = *a.nsegs;
  for (u32 i = blockIdx.x; i < n; i += gridDim.x) {
    const u64 item = a.segs[i];
    if (a.flags[(u32)item] & A5X_WF_GLOB) continue;  // pass G (k_expand_g)
    expand_segment<A5X_LMAX_B, A5X_MLMAX_B, A5X_DPENT_B, A5X_RING_B>(S, ring, T, a, item);
  }
}

// pass G: the GLOB words' segments of the BIG list, one scratch slot per workgroup
__global__ void __launch_bounds__(64) k_expand_g(ExpArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  load_table(smem, a.table, a.table_bytes);
  __syncthreads();
  const Tab T = tab_view(smem);
  uint8_t* slot = a.gscr + (u64)blockIdx.x * GSLOT_BYTES;
  u32* ring = (u32*)slot;  // zero between flushes (a5x_host zeroes it once)
  LdsG& S = *(LdsG*)(slot + A5X_RING_G);
  const u32 n = *a.nsegs;
  for (u32 i = blockIdx.x; i < n; i += gridDim.x) {
    const u64 item = a.segs[i];
    if (!(a.flags[(u32)item] & A5X_WF_GLOB)) continue;
    expand_segment<A5X_LMAX_G, A5X_MLMAX_G, A5X_DPENT_G, A5X_RING_G>(S, ring, T, a, item);
  }
}

// ---------------------------------------------------------------------------
// Locate: global byte offset of candidate indices (range starts for partial calls)
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(64) k_locate(ExpArgs a, const u64* cands, u32 n, u64* out_bytes) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  load_table(smem, a.table, a.table_bytes);
  __syncthreads();
  const Tab T = tab_view(smem);
  LdsB& S = *(LdsB*)(smem + ((a.table_bytes + 15u) & ~15u));
  for (u32 i = blockIdx.x; i < n; i += gridDim.x) {  // one wave per query
    const u64 g = cands[i];
    if (g >= a.cand_off[a.nw]) { if (lane_id() == 0) out_bytes[i] = a.byte_off[a.nw]; continue; }
    // largest w with cand_off[w] <= g (that word has count > 0)
    u64 lo = 0, hi = a.nw;  // invariant cand_off[lo] <= g < cand_off[hi]
    while (hi - lo > 1) {
      const u64 mid = (lo + hi) / 2;
      if (a.cand_off[mid] <= g) lo = mid; else hi = mid;
    }
    const u64 w = lo, r = g - a.cand_off[w];
    u64 pos = a.byte_off[w];
    if (r && (a.flags[w] & A5X_WF_FAST)) {
      // FAST words: the group radix order of k_expand_fast (record from HBM)
      u64* rec = (u64*)&S;
      const u32 rs = ff_rsize(a.flags[w]);
      for (u32 i2 = lane_id(); i2 < rs; i2 += 64) rec[i2] = a.rec[a.roff[w] + i2];
      WAVE_SYNC();
      pos += fast_prefix_bytes(rec, r);
    } else if (r && (a.flags[w] & A5X_WF_GLOB)) {
      // pass G word: its setup in this workgroup's scratch slot (the host limits the grid)
      if (blockIdx.x >= a.gslots) { if (lane_id() == 0) atomicOr(a.err, A5X_DERR_STATE); return; }
      LdsG& SG = *(LdsG*)(a.gscr + (u64)blockIdx.x * GSLOT_BYTES + A5X_RING_G);
      WordInfo I = wave_setup<A5X_LMAX_G, A5X_MLMAX_G, A5X_DPENT_G>(SG, T, a.words, a.woff, w, a.mn, a.mx);
      if (!I.fits) { if (lane_id() == 0) atomicOr(a.err, A5X_DERR_STATE); return; }
      if (I.cls & A5X_WF_RADIX) pos += radix_prefix_bytes(SG, T, I, r);
      else pos += uniform64(dp_prefix_bytes(SG, T, I, r));
    } else if (r) {
      WordInfo I = wave_setup<A5X_LMAX_B, A5X_MLMAX_B, A5X_DPENT_B>(S, T, a.words, a.woff, w, a.mn, a.mx);
      if (!I.fits) { if (lane_id() == 0) atomicOr(a.err, A5X_DERR_STATE); return; }
      if (I.cls & A5X_WF_RADIX) pos += radix_prefix_bytes(S, T, I, r);
      else pos += uniform64(dp_prefix_bytes(S, T, I, r));
    }
    if (lane_id() == 0) out_bytes[i] = pos;
    WAVE_SYNC();
  }
}

// ---------------------------------------------------------------------------
// Verification digest: per word {count, bytes, sum h, sum h^2}, h = fmix64(fnv1a64)
// (same definition as oracle/a5_oracle.c a5o_cand_hash).  One lane per word.
// ---------------------------------------------------------------------------
__device__ __forceinline__ u64 fmix64(u64 k) {
  k ^= k >> 33; k *= 0xff51afd7ed558ccdULL;
  k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ULL;
  k ^= k >> 33;
  return k;
}

__global__ void __launch_bounds__(256) k_digest(const uint8_t* out, const u64* byte_off, u64 out_base, u64 nw,
                                                u64* dig) {
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 w = (u64)blockIdx.x * blockDim.x + threadIdx.x; w < nw; w += stride) {
    const u64 s = byte_off[w] - out_base, e = byte_off[w + 1] - out_base;
    u64 cnt = 0, hs = 0, hq = 0, h = 1469598103934665603ULL;
    for (u64 i = s; i < e; i++) {
      const u32 b = out[i];
      if (b == '\n') {
        const u64 f = fmix64(h);
        cnt++; hs += f; hq += f * f;
        h = 1469598103934665603ULL;
      } else {
        h ^= b; h *= 1099511628211ULL;
      }
    }
    dig[4 * w + 0] = cnt; dig[4 * w + 1] = e - s; dig[4 * w + 2] = hs; dig[4 * w + 3] = hq;
  }
}

// ---------------------------------------------------------------------------
// host-visible launch helpers (C++ linkage; used by a5x_host.cpp)
// ---------------------------------------------------------------------------
#include "a5x_launch.h"

static inline u32 blocks_for(u64 n, u32 bs, u32 cap) {
  u64 b = (n + bs - 1) / bs;
  if (b < 1) b = 1;
  return (u32)(b < cap ? b : cap);
}

hipError_t a5x_launch_keyspace(const A5xKsLaunch& L, hipStream_t st) {
  KsArgs a;
  a.table = L.table; a.table_bytes = L.table_bytes; a.words = L.words; a.woff = L.woff; a.nw = L.nw;
  a.mn = L.mn; a.mx = L.mx; a.count = L.count; a.bytes = L.bytes; a.flags = L.flags;
  a.defer_list = L.defer_list; a.defer_n = L.defer_n; a.nbig = L.nbig; a.nslow = L.nslow; a.err = L.err;
  a.big_list = L.big_list; a.slow_list = L.slow_list;
  a.rec = L.rec; a.roff = L.roff;
  a.cplx_list = L.cplx_list; a.cplx_n = L.cplx_n; a.cplx_cap = L.cplx_cap; a.cplx_base = L.cplx_base;
  a.glob_list = L.glob_list; a.glob_n = L.glob_n; a.gscr = L.gscr;
  a.rmode = L.rmode; a.rcmin = L.rcmin; a.rnseg = L.rnseg; a.rseg = L.rseg; a.vocc = L.vocc;
  a.hiflag = L.hiflag;
  const dim3 kg(blocks_for(L.nw, FW_TILE, 65536));
  if (L.hiflag) {  // the table's keys start on UTF-8 lead bytes only: the walk by the batch's bytes
    hipLaunchKernelGGL(k_hibytes, dim3(256), dim3(256), 0, st, L.words, L.woff, L.nw, L.hiflag);
    // (the full grid: a resident one striding over the tiles measured slower on C5 -s, 19.3 vs
    // 17.9 ms keyspace; on an ASCII batch every workgroup returns at once)
    hipLaunchKernelGGL(k_keyspace_thread<true>, kg, dim3(FW_TILE), a5x_keyspace_thread_lds(L.table_bytes), st, a);
  }
  hipLaunchKernelGGL(k_keyspace_thread<false>, kg, dim3(FW_TILE), a5x_keyspace_thread_lds(L.table_bytes), st, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (L.rmode) {  // -r / -s / -s -r FAST probe: k_keyspace_thread + the words it listed
    hipLaunchKernelGGL(k_keyspace_rprobe, dim3(L.defer_blocks), dim3(256), a5x_keyspace_rprobe_lds(L.table_bytes), st,
                       a);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_keyspace_cplx, dim3(L.defer_blocks), dim3(256),
                     ((L.table_bytes + 15u) & ~15u) + 2 * 256 * FW_UMAXR * 8 + 256 * KC_SLOT, st, a);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  const size_t lds = ((L.table_bytes + 15u) & ~15u) + sizeof(LdsB);
  hipLaunchKernelGGL(k_keyspace_wave, dim3(L.defer_blocks), dim3(64), lds, st, a);
  return hipGetLastError();
}

uint64_t a5x_gslot_bytes() { return GSLOT_BYTES; }

hipError_t a5x_launch_keyspace_g(const A5xKsLaunch& L, hipStream_t st) {
  KsArgs a;
  memset(&a, 0, sizeof a);
  a.table = L.table; a.table_bytes = L.table_bytes; a.words = L.words; a.woff = L.woff; a.nw = L.nw;
  a.mn = L.mn; a.mx = L.mx; a.count = L.count; a.bytes = L.bytes; a.flags = L.flags;
  a.nbig = L.nbig; a.err = L.err; a.big_list = L.big_list;
  a.glob_list = L.glob_list; a.glob_n = L.glob_n; a.gscr = L.gscr;
  hipLaunchKernelGGL(k_keyspace_g, dim3(L.gslots), dim3(64), (L.table_bytes + 15u) & ~15u, st, a);
  return hipGetLastError();
}

size_t a5x_keyspace_thread_lds(u32 table_bytes) {
  return ((table_bytes + 15u) & ~15u) + FW_TILE * KS_GCAP * 8 + 64 + KS_WB + 32 + FW_TILE * KS_ULOG * 2;
}

size_t a5x_keyspace_rprobe_lds(u32 table_bytes) {
  return ((table_bytes + 15u) & ~15u) + 256 * KS_GCAP * 8 + 256 * RP_SLOT;
}

static size_t vsub_lds(u32 table_bytes, u32 wslot, u32 slot) {
  return ((table_bytes + 15u) & ~15u) + VS_BLOCK * (VS_GCAP * 8 + wslot + slot + VS_OCC * 2) +
         (VS_BLOCK / 64) * sizeof(VsWave);
}
size_t a5x_keyspace_vsub_lds(u32 table_bytes) { return vsub_lds(table_bytes, VS_WSLOT, VS_SLOT); }

hipError_t a5x_launch_vsub(const A5xKsLaunch& L, hipStream_t st) {
  KsArgs a;
  memset(&a, 0, sizeof a);
  a.table = L.table; a.table_bytes = L.table_bytes; a.words = L.words; a.woff = L.woff; a.nw = L.nw;
  a.mn = L.mn; a.mx = L.mx; a.count = L.count; a.bytes = L.bytes; a.flags = L.flags; a.err = L.err;
  a.defer_list = L.defer_list; a.defer_n = L.defer_n; a.roff = L.roff;
  a.rmode = L.rmode; a.rcmin = L.rcmin; a.rnseg = L.rnseg; a.rseg = L.rseg;
  a.vout_list = L.vout_list; a.vout_n = L.vout_n; a.vn = L.vn; a.vrsz = L.vrsz;
  a.vrec = L.vrec; a.vrec_n = (unsigned long long*)L.vrec_n; a.vrec_cap = L.vrec_cap; a.vocc = L.vocc;
  const dim3 grid(L.defer_blocks * (256 / VS_BLOCK));
  if (L.vlong_list) {
    // small lane slots first (more waves per CU); the words they cannot hold go to the
    // large instantiation through vlong_list
    a.vlong_list = L.vlong_list; a.vlong_n = L.vlong_n;
    hipLaunchKernelGGL((k_keyspace_vsub<VS_WSLOT_S, VS_SLOT_S, true>), grid, dim3(VS_BLOCK),
                       vsub_lds(L.table_bytes, VS_WSLOT_S, VS_SLOT_S), st, a);
    a.defer_list = L.vlong_list; a.defer_n = L.vlong_n;
    a.vlong_list = nullptr; a.vlong_n = nullptr;
  }
  hipLaunchKernelGGL((k_keyspace_vsub<VS_WSLOT, VS_SLOT, false>), grid, dim3(VS_BLOCK),
                     vsub_lds(L.table_bytes, VS_WSLOT, VS_SLOT), st, a);
  return hipGetLastError();
}

hipError_t a5x_launch_vwords_sizes(const uint32_t* flags, const uint64_t* cand_off, uint64_t nw, uint64_t* vn,
                                   uint64_t* vrsz, hipStream_t st) {
  hipLaunchKernelGGL(k_vwords_sizes, dim3(blocks_for(nw, 256, 8192)), dim3(256), 0, st, flags, cand_off, nw, vn, vrsz);
  return hipGetLastError();
}

hipError_t a5x_launch_vwords_fill(const A5xVwLaunch& L, hipStream_t st) {
  VwArgs a;
  a.flags = L.flags; a.cand_off = L.cand_off; a.byte_off = L.byte_off; a.roff = L.roff; a.rec = L.rec;
  a.vrec = L.vrec; a.vpre = L.vpre; a.vrpre = L.vrpre; a.nw = L.nw;
  a.vcand_off = L.vcand_off; a.vbyte_off = L.vbyte_off; a.vflags = L.vflags; a.vroff = L.vroff;
  a.vmap = L.vmap; a.vobase = L.vobase; a.vrec2 = L.vrec2;
  a.table = L.table; a.table_bytes = L.table_bytes; a.rmode = L.rmode; a.rcmin = L.rcmin; a.words = L.words;
  a.woff = L.woff;
  hipLaunchKernelGGL(k_vwords_fill, dim3(blocks_for(L.nw, 256, 8192)), dim3(256), vwords_fill_lds(L.table_bytes), st, a);
  return hipGetLastError();
}

size_t a5x_keyspace_wave_lds(u32 table_bytes) { return ((table_bytes + 15u) & ~15u) + sizeof(LdsB); }

// recursive exclusive scan of pairs; tmp must hold a5x_scan_tmp_elems(n) u64
u64 a5x_scan_tmp_elems(u64 n) {
  u64 t = 0;
  while (n > SCAN_TILE) { n = (n + SCAN_TILE - 1) / SCAN_TILE; t += 2 * (n + 1); }
  return t + 2;
}

hipError_t a5x_launch_scan(const u64* ca, const u64* cb, u64 n, u64* outa, u64* outb, u64* tmp, u32* err,
                           hipStream_t st) {
  if (n <= SCAN_TILE) {
    hipLaunchKernelGGL(k_scan_down, dim3(1), dim3(SCAN_BLOCK), 0, st, ca, cb, n, (const u64*)nullptr,
                       (const u64*)nullptr, outa, outb, err);
    return hipGetLastError();
  }
  const u64 nb = (n + SCAN_TILE - 1) / SCAN_TILE;
  u64* sa = tmp;
  u64* sb = tmp + (nb + 1);
  hipLaunchKernelGGL(k_scan_reduce, dim3((u32)nb), dim3(SCAN_BLOCK), 0, st, ca, cb, n, sa, sb, err);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  // scan the block sums in place (into the same arrays, n+1 layout)
  e = a5x_launch_scan(sa, sb, nb, sa, sb, tmp + 2 * (nb + 1), err, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_scan_down, dim3((u32)nb), dim3(SCAN_BLOCK), 0, st, ca, cb, n, (const u64*)sa,
                     (const u64*)sb, outa, outb, err);
  return hipGetLastError();
}

hipError_t a5x_launch_plan(const u64* cand_off, u64 nw, u64 CH, u32* chunk_w0, hipStream_t st) {
  hipLaunchKernelGGL(k_plan, dim3(blocks_for(nw, 256, 65536)), dim3(256), 0, st, cand_off, nw, CH, chunk_w0);
  return hipGetLastError();
}

hipError_t a5x_launch_segments(const u32* list, const u32* list_n, u32 n_bound, const u64* cand_off, u64 cb, u64 ce,
                               u64 CH, u64* segs, u32* nsegs, hipStream_t st) {
  hipLaunchKernelGGL(k_segments, dim3(blocks_for(n_bound, 256, 4096)), dim3(256), 0, st, list, list_n, cand_off, cb,
                     ce, CH, segs, nsegs);
  return hipGetLastError();
}

static ExpArgs exp_args(const A5xExpLaunch& L) {
  ExpArgs a;
  a.table = L.table; a.table_bytes = L.table_bytes; a.words = L.words; a.woff = L.woff; a.nw = L.nw;
  a.cand_off = L.cand_off; a.byte_off = L.byte_off; a.flags = L.flags; a.chunk_w0 = L.chunk_w0;
  a.segs = L.segs; a.nsegs = L.nsegs; a.cand_begin = L.cand_begin; a.cand_end = L.cand_end; a.CH = L.CH; a.SEG = L.SEG; a.out = L.out;
  a.out_base = L.out_base; a.out_cap = L.out_cap; a.mn = L.mn; a.mx = L.mx; a.err = L.err; a.dbg = L.dbg;
  a.rec = L.rec; a.roff = L.roff; a.rec_n = L.rec_n;
  a.dg_bitmap = L.dg_bitmap; a.dg_bm_mask = L.dg_bm_mask; a.dg_has_zero = L.dg_has_zero; a.dg_hit_cap = L.dg_hit_cap;
  a.dg_table = L.dg_table; a.dg_tmask = L.dg_tmask; a.dg_hits = L.dg_hits; a.dg_nhits = L.dg_nhits;
  a.gscr = L.gscr; a.gslots = L.gslots;
  a.vmap = L.vmap; a.vobase = L.vobase;
  return a;
}

size_t a5x_expand_lds(u32 table_bytes, int kind, u32 waves) {
  const size_t tb = (table_bytes + 15u) & ~15u;
  if (kind == 2) return tb + ((A5X_RING_B + sizeof(LdsB) + 15u) & ~(size_t)15u);
  if (kind == 1) return tb + waves * ((A5X_RING_A + sizeof(LdsA) + 15u) & ~(size_t)15u);
  return waves * ((FX_RING + FX_TRASH + sizeof(FXWin) + 15u) & ~(size_t)15u);
}

// waves per workgroup a kernel admits: its compiled maxThreadsPerBlock / 64 (>= 1)
u32 a5x_max_waves(const void* fn) {
  hipFuncAttributes at;
  if (hipFuncGetAttributes(&at, fn) != hipSuccess || at.maxThreadsPerBlock < 64) return 1u;
  return (u32)at.maxThreadsPerBlock / 64u;
}

// kind 0: k_expand_fast, 1: k_expand_slow, 2: k_expand_b, 3 / 5: k_expand_fast_md5 / _ntlm (fused digest)
hipError_t a5x_launch_expand(const A5xExpLaunch& L, int kind, hipStream_t st) {
  ExpArgs a = exp_args(L);
  const u64 c0 = L.cand_begin / L.CH, c1 = (L.cand_end + L.CH - 1) / L.CH;
  const u64 nchunks = c1 - c0;
  if (nchunks == 0) return hipSuccess;
  u32 waves = kind == 0 ? L.waves_per_block_fast : L.waves_per_block;
  // (A5X_WAVES beyond what the layout fits in a workgroup's 64 KiB of dynamic LDS: fewer waves)
  const int lk = kind == 1 ? 1 : kind == 2 ? 2 : 0;
  while (waves > 1 && a5x_expand_lds(L.table_bytes, lk, waves) > 65536) waves--;
  // ... and never more threads than the kernel was compiled for (its __launch_bounds__):
  // a larger workgroup fails to launch ("unspecified launch failure")
  const void* fn = kind == 0 ? (const void*)k_expand_fast : kind == 3 ? (const void*)k_expand_fast_md5
                 : kind == 5 ? (const void*)k_expand_fast_ntlm : kind == 1 ? (const void*)k_expand_slow
                 : kind == 2 ? (const void*)k_expand_b : (const void*)k_expand_g;
  const u32 wmax = a5x_max_waves(fn);
  if (waves > wmax) waves = wmax;
  const u64 nb = (nchunks + waves - 1) / waves;
  if (kind == 0)
    hipLaunchKernelGGL(k_expand_fast, dim3((u32)nb), dim3(64 * waves), a5x_expand_lds(L.table_bytes, 0, waves), st, a);
  else if (kind == 3)
    hipLaunchKernelGGL(k_expand_fast_md5, dim3((u32)nb), dim3(64 * waves), a5x_expand_lds(L.table_bytes, 0, waves), st,
                       a);
  else if (kind == 5)
    hipLaunchKernelGGL(k_expand_fast_ntlm, dim3((u32)nb), dim3(64 * waves), a5x_expand_lds(L.table_bytes, 0, waves), st,
                       a);
  else if (kind == 1)  // (the bound counts the range's candidates, not the slow words' segments:
                       // workgroups past *nsegs exit before they stage anything.  A grid capped at
                       // 2 workgroups per CU measured 2-3 % slower on C3: its grid-stride waves
                       // held their LDS beside k_expand_fast for the whole slow-word work)
    hipLaunchKernelGGL(k_expand_slow, dim3(blocks_for(L.nsegs_bound, waves, 65536)), dim3(64 * waves),
                       a5x_expand_lds(L.table_bytes, 1, waves), st, a);
  else if (kind == 2)
    hipLaunchKernelGGL(k_expand_b, dim3(blocks_for(L.nsegs_bound, 1, 65536)), dim3(64), a5x_expand_lds(L.table_bytes, 2, 1),
                       st, a);
  else if (kind == 4)
    hipLaunchKernelGGL(k_expand_g, dim3(L.gslots), dim3(64), (L.table_bytes + 15u) & ~15u, st, a);
  return hipGetLastError();
}

hipError_t a5x_launch_locate(const A5xExpLaunch& L, const u64* cands, u32 n, u64* out_bytes, hipStream_t st) {
  ExpArgs a = exp_args(L);
  u32 grid = n < 1024 ? (n ? n : 1) : 1024;
  if (L.gscr && L.gslots) grid = grid < L.gslots ? grid : L.gslots;  // one pass G slot per workgroup
  hipLaunchKernelGGL(k_locate, dim3(grid), dim3(64), a5x_keyspace_wave_lds(L.table_bytes), st, a, cands, n, out_bytes);
  return hipGetLastError();
}

// The word of each global candidate g[i] (largest w with cand_off[w] <= g[i]) and its
// index in that word; g[i] >= cand_off[nw] -> (nw, 0).  One lane per target
// (a5x_split_device: one launch instead of a host binary search of device reads).
__global__ void __launch_bounds__(256) k_word_of(const u64* cand_off, u64 nw, const u64* g, u32 nt, u64* word,
                                                 u64* ciw) {
  const u32 i = blockIdx.x * 256u + threadIdx.x;
  if (i >= nt) return;
  const u64 x = g[i];
  if (x >= cand_off[nw]) { word[i] = nw; ciw[i] = 0; return; }
  u64 a = 0, b = nw;  // cand_off[a] <= x < cand_off[b]
  while (b - a > 1) {
    const u64 m = a + (b - a) / 2;
    if (cand_off[m] <= x) a = m; else b = m;
  }
  word[i] = a;
  ciw[i] = x - cand_off[a];
}

hipError_t a5x_launch_word_of(const u64* cand_off, u64 nw, const u64* g, uint32_t nt, u64* word, u64* ciw,
                              hipStream_t st) {
  if (nt) hipLaunchKernelGGL(k_word_of, dim3((nt + 255) / 256), dim3(256), 0, st, cand_off, nw, g, nt, word, ciw);
  return hipGetLastError();
}

hipError_t a5x_launch_digest(const uint8_t* out, const u64* byte_off, u64 out_base, u64 nw, u64* dig,
                             hipStream_t st) {
  hipLaunchKernelGGL(k_digest, dim3(blocks_for(nw, 256, 65536)), dim3(256), 0, st, out, byte_off, out_base, nw, dig);
  return hipGetLastError();
}

int a5x_read_stamps(unsigned long long* out16, int reset) {
#ifdef A5X_STAMPS
  if (hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_a5x_stamps), 16 * 8) != hipSuccess) return -2;
  if (reset) {
    unsigned long long z[16] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_a5x_stamps), z, sizeof z) != hipSuccess) return -2;
  }
  return 0;
#else
  (void)out16; (void)reset;
  return -9;
#endif
}

hipError_t a5x_set_kernel_attrs() {
  hipError_t e = hipFuncSetAttribute((const void*)k_expand_b, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (e != hipSuccess) return e;
  e = hipFuncSetAttribute((const void*)k_keyspace_wave, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (e != hipSuccess) return e;
  e = hipFuncSetAttribute((const void*)k_keyspace_thread<false>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (e != hipSuccess) return e;
  e = hipFuncSetAttribute((const void*)k_keyspace_thread<true>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (e != hipSuccess) return e;
  e = hipFuncSetAttribute((const void*)k_keyspace_cplx, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (e != hipSuccess) return e;
  e = hipFuncSetAttribute((const void*)k_keyspace_rprobe, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (e != hipSuccess) return e;
  e = hipFuncSetAttribute((const void*)k_keyspace_vsub<VS_WSLOT, VS_SLOT, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (e != hipSuccess) return e;
  e = hipFuncSetAttribute((const void*)k_keyspace_vsub<VS_WSLOT_S, VS_SLOT_S, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (e != hipSuccess) return e;
  e = hipFuncSetAttribute((const void*)k_vwords_fill, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (e != hipSuccess) return e;
  e = hipFuncSetAttribute((const void*)k_locate, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (e != hipSuccess) return e;
  e = hipFuncSetAttribute((const void*)k_expand_slow, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (e != hipSuccess) return e;
  return hipFuncSetAttribute((const void*)k_expand_fast, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
}
