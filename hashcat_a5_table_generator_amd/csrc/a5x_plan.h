// a5x_plan.h -- per-word unit scan, keyspace closed form and piece plan of the
// FAST expansion path.  Host + device: the kernels (a5x_kernels.hip) run it per
// lane; the host library runs the same code for a5x_debug_fast_word(), which the
// CPU test suite compares against the oracle (tests/test_plan.py).
//
// Reference semantics (processWord, /root/reference/main.go:168-205): a candidate
// is a set of non-overlapping key matches of the ORIGINAL word plus one value per
// match.  Matches are grouped into *units*: a lone match (R = 1 + nvals choices,
// choice 0 = the key itself) or a *cluster* of overlapping matches (e.g. "s"/"ss"
// over "ss", czech+german), whose choices are all non-overlapping subsets of its
// matches times their values (choice 0 = no match).  Units are disjoint, so the
// candidates are the mixed-radix product of the units minus the all-zero
// (unchanged) combination, whenever the substitution-count window is free
// (min <= 1 and every candidate's count <= max).
#pragma once
#include <stdint.h>

#include "a5x_format.h"

#define A5X_HD __host__ __device__ inline

typedef uint64_t u64;
typedef uint32_t u32;
typedef int64_t i64;

// ---------------------------------------------------------------------------
// the device table (see a5x_format.h)
// ---------------------------------------------------------------------------
struct Tab {
  const A5xTableHdr* hdr;
  const uint16_t* bucket;
  const A5xKey* keys;
  const A5xChoice* ch;
  const uint8_t* blob;
  const u64* kmatch;   // first min(klen, 4) key bytes | klen << 32
  const u32* bucket2;  // bucket[b] | bucket[b + 1] << 16
  const u64* cval;     // choice bytes (<= 7) | len << 56
};

A5X_HD Tab tab_view(const uint8_t* base) {
  Tab t;
  t.hdr = (const A5xTableHdr*)base;
  t.bucket = (const uint16_t*)(base + t.hdr->off_bucket);
  t.keys = (const A5xKey*)(base + t.hdr->off_keys);
  t.ch = (const A5xChoice*)(base + t.hdr->off_choices);
  t.blob = base + t.hdr->off_blob;
  t.kmatch = (const u64*)(base + t.hdr->off_kmatch);
  t.bucket2 = (const u32*)(base + t.hdr->off_bucket2);
  t.cval = (const u64*)(base + t.hdr->off_cval);
  return t;
}

A5X_HD u64 mul_ovf(u64 a, u64 b, bool& ovf) {
  u64 r;
  ovf |= __builtin_mul_overflow(a, b, &r);
  return r;
}
A5X_HD u64 add_ovf(u64 a, u64 b, bool& ovf) {
  u64 r = a + b;
  ovf |= r < a;
  return r;
}
A5X_HD u32 umin32(u32 a, u32 b) { return a < b ? a : b; }
A5X_HD u32 umax32(u32 a, u32 b) { return a > b ? a : b; }

// libdivide u32 branch-free division (d >= 2): l = ceil(log2 d), M = floor(2^32 (2^l - d) / d) + 1
A5X_HD void divmagic(u32 d, u32& magic, u32& shift) {
  const u32 l = 32 - (u32)__builtin_clz(d - 1);
  const u64 m = (((u64)1 << 32) * (((u64)1 << l) - d)) / d + 1;
  magic = (u32)m;
  shift = l - 1;
}
A5X_HD u32 fastdiv_hd(u32 n, u32 magic, u32 shift) {
  const u32 q = (u32)(((u64)n * magic) >> 32);
  return (((n - q) >> 1) + q) >> shift;
}

// ---------------------------------------------------------------------------
// FAST plan records (built once per word by k_keyspace_thread, streamed by
// k_expand_fast).  A record is a run of u64 in HBM:
//   [0]               header  (fr_hdr)
//   [1, 1+np)         piece descriptors, pieces in byte order (fr_desc)
//   [1+np, 1+np+ne)   piece entries: the R entries of a piece consecutive, pieces
//                     in order; entry = 7 content bytes + meta byte (len | (R-1) << 3)
// A word is cut left to right into pieces of <= FW_PLEN bytes: a *group* piece
// holds one or more consecutive substitution units (a key match with its R =
// 1 + nvals choices, or a cluster of overlapping matches) with the literal bytes
// around them, all R_1 x R_2 x ... <= FW_UMAXR combinations precombined; a
// *literal* piece holds plain bytes (R = 1).  Combination a_1 + R_1 (a_2 + ...)
// of a group is the mixed-radix digit order of its units (left unit least
// significant), and pieces are digits of the word's candidate index n = rank + 1
// in the same order, so candidate numbering equals the per-unit radix order of
// the other expansion kernels.
// ---------------------------------------------------------------------------
#define FW_PLEN 7    // bytes per piece
#define FW_UMAXM 8   // matches per cluster unit
#define FW_UMAXR 16  // choices per unit / group (4-bit R-1 fields)
#define FW_PMAX 8    // pieces per word
#define FW_RMAX 250  // record u64 per word (window budget)
#define FW_TILE 256  // words per keyspace tile (one workgroup)
#define FW_TILE_REC (FW_TILE * 40)  // record u64 budget per tile (avg 320 B / word)
#define FW_MAXL 1000 // longest candidate (+ newline) of a FAST word
#define FW_PMAX_CNT (1u << 24)  // candidates per FAST word: exact magic division (n (R-1) < 2^32)
                                // and 24-bit digit products (v_mad_u32_u24)
// big pieces (k_expand_fast window setup): consecutive small pieces combined into
// <= FB_PLEN bytes with <= FB_RMAX combinations, entries of 16 B (15 bytes + length)
#define FB_PLEN 15
#define FB_RMAX 64
#define FB_SPAN 4    // small pieces per big piece
#define FB_NMAX 4    // big pieces per word
#ifndef FB_EMAX
#define FB_EMAX 254  // big entries per word (window budget)
#endif

#define FW_M56 0x00FFFFFFFFFFFFFFull
A5X_HD u64 fw_meta(u32 len, u32 R) { return (u64)(len | ((R - 1u) << 3)) << 56; }
A5X_HD u32 fw_len(u64 e) { return (u32)(e >> 56) & 7u; }
A5X_HD u64 keep_bytes64(u64 v, u32 n) { return n >= 8 ? v : (v & ((1ull << (8 * n)) - 1ull)); }

// header: np | ng << 4 | ne << 8 | maxl << 16 | nbig << 28 | first small piece of
//         big pieces 1..3 << 31 (3 bits each) | R - 1 of big pieces 0..3 << 40 (6 bits
//         each; 0 past nbig, i.e. R = 1)
A5X_HD u64 fr_hdr(u32 np, u32 ng, u32 ne, u32 maxl, u32 nbig, u32 bstarts, u32 bRp) {
  return (u64)np | ((u64)ng << 4) | ((u64)ne << 8) | ((u64)maxl << 16) | ((u64)nbig << 28) | ((u64)bstarts << 31) |
         ((u64)bRp << 40);
}
A5X_HD u32 frh_nbig(u64 h) { return (u32)(h >> 28) & 7u; }
A5X_HD u32 frh_bstart(u64 h, u32 b) { return b == 0 ? 0u : (b > 3 ? 15u : (u32)(h >> (31 + 3 * (b - 1))) & 7u); }
A5X_HD u32 frh_np(u64 h) { return (u32)h & 15u; }
A5X_HD u32 frh_ng(u64 h) { return (u32)(h >> 4) & 15u; }
A5X_HD u32 frh_ne(u64 h) { return (u32)(h >> 8) & 255u; }
A5X_HD u32 frh_maxl(u64 h) { return (u32)(h >> 16) & 4095u; }
A5X_HD u32 frh_R(u64 h, u32 b) { return ((u32)(h >> (40 + 6 * b)) & 63u) + 1u; }  // R of big piece b

// piece descriptor: magic = ceil(2^32 / R) (0 for R = 1) | first entry (relative
// to the entries) << 32 | (R-1) << 40 | (R == 1) << 63.  The digit of n is
// d = n - q R with q = umulhi(n, magic) (+ n when R = 1): exact for n (R - 1) <
// 2^32 (FW_PMAX_CNT bound).
A5X_HD u32 fr_magic(u32 R) { return R > 1 ? 0xFFFFFFFFu / R + 1u : 0u; }  // (= ceil(2^32 / R): a 32-bit division)
A5X_HD u64 fr_desc(u32 R, u32 ebase) {
  return (u64)fr_magic(R) | ((u64)(ebase & 255u) << 32) | ((u64)(R - 1) << 40) | ((u64)(R == 1) << 63);
}
A5X_HD u32 frd_R(u64 G) { return ((u32)(G >> 40) & 31u) + 1u; }
A5X_HD u32 frd_ebase(u64 G) { return (u32)(G >> 32) & 255u; }

// FAST flag fields (written by the keyspace pass): record size = 1 + np + ne
A5X_HD u32 ff_ng(u32 f) { return (f >> 10) & 31u; }
A5X_HD u32 ff_ne(u32 f) { return (f >> 16) & 255u; }
A5X_HD u32 ff_np(u32 f) { return (f >> 24) & 31u; }
A5X_HD u32 ff_rsize(u32 f) { return 1u + ff_np(f) + ff_ne(f); }

// k_expand_fast window: records at wrec[0, FX_ZSLOT), wrec[FX_ZSLOT] = 0 (the
// empty entry every piece past a word's last one reads).
#define FX_WREC 256
#define FX_ZSLOT 255

// A word's bytes in global memory (or host memory).
struct GWord {
  const uint8_t* p;
  A5X_HD u32 at(u32 i) const { return p[i]; }
  A5X_HD u64 ld(u32 i, u32 n) const {  // n <= 7
    u64 v = 0;
    for (u32 k = 0; k < n; k++) v |= (u64)p[i + k] << (8 * k);
    return v;
  }
};

template <class W>
A5X_HD bool key_match_w(const W& wd, u32 p, const A5xKey& key, const Tab& T) {
  const A5xChoice c0 = T.ch[key.choice_base];
  for (u32 i = 1; i < key.klen; i++) {  // byte 0 matched by the bucket
    const u32 kb = i < 4 ? ((c0.first4 >> (8 * i)) & 255u) : T.blob[c0.blob_off + i];
    if (wd.at(p + i) != kb) return false;
  }
  return true;
}

// <= 7 bytes of choice ci as a u64
A5X_HD u64 choice7(const Tab& T, u32 ci) {
  const A5xChoice c = T.ch[ci];
  u64 v = c.first4;
  for (u32 k = 4; k < c.len && k < 8; k++) v |= (u64)T.blob[c.blob_off + k] << (8 * k);
  return v;
}

// ---------------------------------------------------------------------------
// units
// ---------------------------------------------------------------------------
struct Unit {
  u32 s, e;        // byte span [s, e) of the original word
  u32 R;           // choices; choice 0 = the span unchanged
  u32 ml;          // longest choice (bytes)
  u32 mnl;         // shortest choice (bytes)
  u32 spos, sneg;  // sums over choices of max(len - span, 0) and max(span - len, 0)
  int maxd;        // longest choice - span
  u32 nm;          // key matches in the unit (bounds the substitutions of a choice)
  u32 key;         // lone match: its key index
  u32 cb;          // lone match: the key's choice_base (choices cb + a, a < R)
  u32 k;           // cluster: number of matches (0 for a lone match)
  u64 m0, m1;      // cluster matches 0-3 / 4-7, 16 bits each: (pos - s) << 10 | key index
  bool ok;         // cluster fits FW_UMAXM matches, FW_UMAXR choices of <= FW_PLEN bytes
};

A5X_HD u32 unit_mkey(const Unit& U, u32 j) { return (u32)((j < 4 ? U.m0 : U.m1) >> (16 * (j & 3))) & 1023u; }
A5X_HD u32 unit_mpos(const Unit& U, u32 j) { return U.s + ((u32)((j < 4 ? U.m0 : U.m1) >> (16 * (j & 3) + 10)) & 63u); }

// Enumerate the choices of a cluster in a fixed order (match subsets by increasing
// bitmask, then values as an odometer, first match fastest); choice 0 is the empty
// subset.  target -1: statistics only (R, ml, spos, sneg, maxd, ok); target -2:
// also every choice a into content[a * cstride] (bytes | len << 56); else stop at
// choice `target` and return its bytes (len <= FW_PLEN) in *content / *len.
template <class W>
A5X_HD void cluster_choices(const W& wd, Unit& U, const Tab& T, int target, u64* content, u32* len,
                            u32 cstride = 1) {
  const u32 span = U.e - U.s;
  u32 R = 0, ml = 0, mnl = 0xffffffffu, spos = 0, sneg = 0;
  int maxd = -(int)span;
  bool ok = U.ok;
  for (u32 mask = 0; mask < (1u << U.k) && ok; mask++) {
    // valid = chosen matches pairwise disjoint (matches are in position order)
    u32 last = 0, nch = 0;
    bool valid = true;
    for (u32 j = 0; j < U.k; j++) {
      if (!((mask >> j) & 1u)) continue;
      const u32 pj = unit_mpos(U, j);
      if (nch && pj < last) { valid = false; break; }
      last = pj + T.keys[unit_mkey(U, j)].klen;
      nch++;
    }
    if (!valid) continue;
    // value odometer over the chosen matches: 4-bit digit j in [0, nvals_j)
    u32 odo = 0;
    while (true) {
      // bytes of this choice
      u64 v = 0;
      u32 n = 0, cur = U.s;
      for (u32 j = 0; j < U.k; j++) {
        if (!((mask >> j) & 1u)) continue;
        const u32 pj = unit_mpos(U, j);
        const A5xKey key = T.keys[unit_mkey(U, j)];
        for (; cur < pj; cur++, n++) if (n < 8) v |= (u64)wd.at(cur) << (8 * n);
        const u32 ci = key.choice_base + 1u + ((odo >> (4 * j)) & 15u);
        const u32 cl = T.ch[ci].len;
        if (n < 8) v |= choice7(T, ci) << (8 * n);
        n += cl;
        cur = pj + key.klen;
      }
      for (; cur < U.e; cur++, n++) if (n < 8) v |= (u64)wd.at(cur) << (8 * n);
      if (n > FW_PLEN || R >= FW_UMAXR) { ok = false; break; }
      if ((int)R == target) {
        *content = keep_bytes64(v, n);
        *len = n;
        U.ok = true;
        return;
      }
      if (target == -2) content[R * cstride] = keep_bytes64(v, n) | ((u64)n << 56);
      R++;
      ml = umax32(ml, n);
      mnl = umin32(mnl, n);
      if (n > span) spos += n - span; else sneg += span - n;
      maxd = (int)n - (int)span > maxd ? (int)n - (int)span : maxd;
      // next value combination
      u32 j = 0;
      for (; j < U.k; j++) {
        if (!((mask >> j) & 1u)) continue;
        const u32 dj = ((odo >> (4 * j)) & 15u) + 1u;
        odo &= ~(15u << (4 * j));
        if (dj < T.keys[unit_mkey(U, j)].nvals && dj < 16u) { odo |= dj << (4 * j); break; }
      }
      if (j == U.k) break;
    }
  }
  U.R = R; U.ml = ml; U.mnl = mnl; U.spos = spos; U.sneg = sneg; U.maxd = maxd; U.ok = ok;
}

// Next unit at or after p (p advances past it).  Returns false at the end of the word.
template <class W>
A5X_HD bool next_unit(const W& wd, u32 L, u32& p, const Tab& T, Unit& U) {
  for (; p < L; p++) {
    u32 e = p, nmatch = 0, k0 = 0;
    U.m0 = 0; U.m1 = 0;
    U.ok = true;
    // matches at p, then at every position inside the growing span
    for (u32 q = p; q < e || q == p; q++) {
      const u32 b = wd.at(q);
      const u32 ks = T.bucket[b], ke = T.bucket[b + 1];
      for (u32 kk = ks; kk < ke; kk++) {
        const A5xKey key = T.keys[kk];
        if (q + key.klen > L || !key_match_w(wd, q, key, T)) continue;
        if (nmatch < FW_UMAXM && q - p < 64 && kk < 1024) {
          const u64 f = (u64)(((q - p) << 10) | kk) << (16 * (nmatch & 3));
          if (nmatch < 4) U.m0 |= f; else U.m1 |= f;
        } else
          U.ok = false;
        if (nmatch == 0) k0 = kk;
        nmatch++;
        e = umax32(e, q + key.klen);
      }
      if (q == p && nmatch == 0) break;
    }
    if (nmatch == 0) continue;
    U.s = p; U.e = e; U.nm = nmatch;
    if (nmatch == 1) {
      const A5xKey key = T.keys[k0];
      U.key = k0; U.k = 0; U.cb = key.choice_base;
      U.R = key.nvals + 1u; U.ml = key.maxclen; U.mnl = key.minclen;
      U.spos = key.sum_dpos; U.sneg = key.sum_dneg; U.maxd = key.maxdelta;
      U.ok = true;
    } else {
      U.key = ~0u; U.k = nmatch;
      if (U.ok) cluster_choices(wd, U, T, -1, nullptr, nullptr);
    }
    p = e;
    return true;
  }
  return false;
}

// bytes and length of choice a of a unit
template <class W>
A5X_HD u64 unit_choice(const W& wd, const Unit& U, const Tab& T, u32 a, u32& len) {
  if (U.k == 0) {  // (entries hold <= FW_PLEN = 7 bytes: longer choices never get here)
    const u64 e = T.cval[U.cb + a];
    len = (u32)(e >> 56);
    return e & FW_M56;
  }
  Unit V = U;
  u64 v = 0;
  len = 0;
  cluster_choices(wd, V, T, (int)a, &v, &len);
  return v;
}

// unit_choice with a cluster's choices already enumerated into cb (stride cs)
template <class W>
A5X_HD u64 unit_choice_b(const W& wd, const Unit& U, const Tab& T, u32 a, u32& len, const u64* cb, u32 cs) {
  if (U.k == 0) return unit_choice(wd, U, T, a, len);
  const u64 e = cb[a * cs];
  len = (u32)(e >> 56);
  return e & FW_M56;
}

// ---------------------------------------------------------------------------
// piece plan -> record
// ---------------------------------------------------------------------------
struct Plan {
  u32 np, ng, ne, lconst, maxl, minl;
  u32 nbig, bstarts, bent;  // big pieces, their first small pieces (3 bits each), big entries
  u32 bRp;                  // R - 1 of big pieces 0..3 (6 bits each)
  bool ok;
};

// Record sinks.  gld/gst(ne, a): entry a of the open group (R <= FW_UMAXR entries, built in
// place while units merge into it; ne = the entries closed so far); ent(i, v): final entry i; desc(i, v): piece i.
// cbuf / cstride: where a cluster unit's choices are enumerated once (BUILD only).
struct NullSink {
  A5X_HD u64* cbuf() const { return nullptr; }
  A5X_HD u32 cstride() const { return 1; }
  A5X_HD u64 gld(u32, u32) const { return 0; }
  A5X_HD void gst(u32, u32, u64) {}
  A5X_HD void ent(u32, u64) {}
  A5X_HD void desc(u32, u64) {}
};
struct ArraySink {  // host replay / tests: rec[0..] as laid out in HBM
  u64* rec;
  u32 np;
  u64 g[FW_UMAXR], c[FW_UMAXR];
  A5X_HD u64* cbuf() { return c; }
  A5X_HD u32 cstride() const { return 1; }
  A5X_HD u64 gld(u32, u32 a) const { return g[a]; }
  A5X_HD void gst(u32, u32 a, u64 v) { g[a] = v; }
  A5X_HD void ent(u32 i, u64 v) { rec[1 + np + i] = v; }
  A5X_HD void desc(u32 i, u64 v) { rec[1 + i] = v; }
};

#ifndef PL_SPLIT_CAP
#define PL_SPLIT_CAP 4   // groups of <= this many entries merge read-all-then-write-all (registers); larger
                         // ones in place (k_keyspace_thread's 8-entry groups: C3 keyspace 2.19 vs 2.25 ms at 8,
                         // profiles/r06u_ab_vwords_fixed_width_c5.txt)
#endif


// Cut a unit-radix word into pieces (see the record format above), one unit at a
// time (unit() in word order, then finish()).  BUILD: also write the entries and
// piece descriptors through the sink (the header is the caller's: fr_hdr of P).
// Shared by the unit walk (plan_word) and the position-synchronous keyspace kernel.
template <bool BUILD, class W, class S, u32 CAP = FW_UMAXR>
struct Planner {
  const W& wd;
  const Tab& T;
  S& sk;
  Plan P;
  bool open;                    // a group piece is being built
  u32 bR, bl, bspan;            // the big piece being filled
  u32 cR, cmax, cmin, cpi, prev;
  // Balanced big pieces (BUILD walks): a second grouping of the same small pieces with
  // R per big piece capped at acap (0: none).  The greedy grouping fills every big piece
  // up to FB_RMAX combinations, e.g. R 4 4 4 3 -> 64 + 3 = 67 entries; capped near
  // P^(1 / nbig) the same two pieces are 16 + 12 = 28 entries.  k_expand_fast's windows
  // are bounded by their big entries, so fewer entries = more words and candidates per
  // window setup.  pick_balanced() takes it when it has as many big pieces as the greedy.
  u32 acap, aR, al, aspan;
  Plan A;
  // first word byte of pieces 0..7 (7 bits each; k_keyspace_vsub's patched sub-words --
  // dead code for every other user)
  u64 pst;

  A5X_HD Planner(const W& w, const Tab& t, S& s, u32 balanced_cap = 0) : wd(w), T(t), sk(s) {
    P.np = 0; P.ng = 0; P.ne = 0; P.lconst = 0; P.maxl = 0; P.minl = 0; P.ok = true;
    P.nbig = 0; P.bstarts = 0; P.bent = 0; P.bRp = 0;
    open = false; bR = 1; bl = 0; bspan = 0; cR = 1; cmax = 0; cmin = 0; cpi = 0; prev = 0; pst = 0;
    acap = balanced_cap; aR = 1; al = 0; aspan = 0;
    A.nbig = 0; A.bstarts = 0; A.bent = 0; A.bRp = 0;
  }
  static A5X_HD void big_join(Plan& Q, u32& qR, u32& ql, u32& qspan, u32 cap, u32 R, u32 maxlen, u32 pi) {
    if (Q.nbig && ql + maxlen <= FB_PLEN && qR * R <= cap && qspan < FB_SPAN) {
      Q.bent += qR * R - qR;
      qR *= R; ql += maxlen; qspan++;
    } else {
      if (Q.nbig >= 1 && Q.nbig <= 3) Q.bstarts |= (pi & 7u) << (3 * (Q.nbig - 1));
      Q.nbig++;
      Q.bent += R;
      qR = R; ql = maxlen; qspan = 1;
    }
    if (Q.nbig <= FB_NMAX) {
      const u32 sh = 6u * (Q.nbig - 1u);
      Q.bRp = (Q.bRp & ~(63u << sh)) | (((qR - 1u) & 63u) << sh);
    }
  }
  A5X_HD void big_add(u32 R, u32 maxlen, u32 pi) {  // small piece pi (in order) joins a big piece
    big_join(P, bR, bl, bspan, FB_RMAX, R, maxlen, pi);
    if (acap) big_join(A, aR, al, aspan, acap, R, maxlen, pi);
  }
  A5X_HD void pick_balanced() {
    if (acap && A.nbig == P.nbig && A.bent < P.bent) {
      P.bstarts = A.bstarts; P.bRp = A.bRp; P.bent = A.bent;
    }
  }
  A5X_HD void close_group() {
    if constexpr (BUILD) {
      for (u32 a = 0; a < cR; a++)
        if (a < cR) sk.ent(P.ne + a, sk.gld(P.ne, a));
      sk.desc(cpi, fr_desc(cR, P.ne));
    }
    big_add(cR, cmax, cpi);
    P.ne += cR; P.ng++; P.maxl += cmax; P.minl += cmin;
    open = false;
  }
  A5X_HD void piece_at(u32 pi, u32 off) {
    if (pi < 8) pst |= (u64)(off & 127u) << (7 * pi);
  }
  A5X_HD void literal(u32 off, u32 n, bool nl_last) {  // one literal piece of n bytes
    piece_at(P.np, off);
    if constexpr (BUILD) {
      const u32 nb = nl_last ? n - 1 : n;
      u64 v = nb ? wd.ld(off, nb) : 0ull;
      if (nl_last) v |= 10ull << (8 * nb);
      sk.ent(P.ne, v | fw_meta(n, 1));
      sk.desc(P.np, fr_desc(1, P.ne));
    }
    big_add(1, n, P.np);
    P.ne++; P.np++; P.lconst += n; P.maxl += n; P.minl += n;
  }
  A5X_HD void unit(const Unit& U) {
    if (!P.ok) return;
    const u32 Ru = U.R, ml = U.ml, run = U.s - prev;
    if (!U.ok || ml > FW_PLEN || Ru > CAP || Ru < 2) { P.ok = false; return; }
    u64* cb = nullptr;
    u32 cs = 1;
    if constexpr (BUILD) {
      if (U.k) {  // cluster: all choices once (unit_choice would re-enumerate per entry)
        cb = sk.cbuf(); cs = sk.cstride();
        Unit V = U;
        cluster_choices(wd, V, T, -2, cb, nullptr, cs);
      }
    }
    if (open && cmax + run + ml <= FW_PLEN && cR * Ru <= CAP) {
      // merge: entry a1 + cR * a2 = old[a1] ++ run ++ choice a2 (descending: in place;
      // fixed trip count so lanes of a wave stay together)
      const u32 nR = cR * Ru;
      if constexpr (BUILD && CAP <= PL_SPLIT_CAP) {
        // small groups: every old entry and choice read first (one round trip, nothing
        // written yet), then every new entry written -- no read waits behind a write
        const u64 rb = run ? wd.ld(prev, run) : 0ull;
        const u32 inv = (256u + cR - 1u) / cR;  // t / cR = (t * inv) >> 8 for t < 16
        u64 ov[CAP], cv[CAP];
        u32 cl[CAP];
#pragma unroll
        for (u32 t = 0; t < CAP; t++) {
          const u32 a2 = (t * inv) >> 8, a1 = t - a2 * cR;
          cl[t] = 0;
          ov[t] = t < nR ? sk.gld(P.ne, a1) : 0ull;
          cv[t] = t < nR ? unit_choice_b(wd, U, T, a2, cl[t], cb, cs) : 0ull;
        }
#pragma unroll
        for (u32 t = 0; t < CAP; t++) {
          if (t < nR) {
            const u32 ol = fw_len(ov[t]);
            const u64 v = (ov[t] & FW_M56) | (rb << (8 * ol)) | (cv[t] << (8 * (ol + run)));
            sk.gst(P.ne, t, (v & FW_M56) | fw_meta(ol + run + cl[t], nR));
          }
        }
      } else if constexpr (BUILD) {
        const u64 rb = run ? wd.ld(prev, run) : 0ull;
        const u32 inv = (256u + cR - 1u) / cR;  // t / cR = (t * inv) >> 8 for t < 16
        for (int t = nR - 1; t >= 0; t--) {
          if ((u32)t >= nR) continue;
          const u32 a2 = ((u32)t * inv) >> 8, a1 = (u32)t - a2 * cR;
          u32 cl = 0;
          const u64 cv = unit_choice_b(wd, U, T, a2, cl, cb, cs);
          const u64 old = sk.gld(P.ne, a1);
          const u32 ol = fw_len(old);
          const u64 v = (old & FW_M56) | (rb << (8 * ol)) | (cv << (8 * (ol + run)));
          sk.gst(P.ne, (u32)t, (v & FW_M56) | fw_meta(ol + run + cl, nR));
        }
      }
      cR = nR; cmax += run + ml; cmin += run + U.mnl;
    } else {
      if (open) close_group();
      u32 off = prev, rem = run;
      while (rem + ml > FW_PLEN) {  // literal run that does not fit with the unit
        const u32 n = umin32(FW_PLEN, rem);
        literal(off, n, false);
        off += n; rem -= n;
      }
      open = true; cR = Ru; cmax = rem + ml; cmin = rem + U.mnl; cpi = P.np;
      piece_at(cpi, off);
      P.np++;
      if constexpr (BUILD && CAP <= PL_SPLIT_CAP) {  // (read every choice, then write)
        const u64 rb = rem ? wd.ld(off, rem) : 0ull;
        u64 cv[CAP];
        u32 cl[CAP];
#pragma unroll
        for (u32 a = 0; a < CAP; a++) {
          cl[a] = 0;
          cv[a] = a < Ru ? unit_choice_b(wd, U, T, a, cl[a], cb, cs) : 0ull;
        }
#pragma unroll
        for (u32 a = 0; a < CAP; a++)
          if (a < Ru) sk.gst(P.ne, a, ((rb | (cv[a] << (8 * rem))) & FW_M56) | fw_meta(rem + cl[a], Ru));
      } else if constexpr (BUILD) {
        const u64 rb = rem ? wd.ld(off, rem) : 0ull;
        for (u32 a = 0; a < Ru; a++) {
          if (a >= Ru) continue;
          u32 cl = 0;
          const u64 cv = unit_choice_b(wd, U, T, a, cl, cb, cs);
          const u64 v = rb | (cv << (8 * rem));
          sk.gst(P.ne, a, (v & FW_M56) | fw_meta(rem + cl, Ru));
        }
      }
    }
    prev = U.e;
  }
  A5X_HD void finish(u32 L) {  // tail bytes + '\n'
    if (!P.ok) return;
    const u32 run = L - prev, tl = run + 1;
    if (open && cmax + tl <= FW_PLEN) {
      if constexpr (BUILD) {
        const u64 tb = (run ? wd.ld(prev, run) : 0ull) | (10ull << (8 * run));
        for (u32 a = 0; a < cR; a++) {
          if (a >= cR) continue;
          const u64 old = sk.gld(P.ne, a);
          const u32 ol = fw_len(old);
          sk.gst(P.ne, a, ((old | (tb << (8 * ol))) & FW_M56) | fw_meta(ol + tl, cR));
        }
      }
      cmax += tl; cmin += tl;
      close_group();
    } else {
      if (open) close_group();
      u32 off = prev, rem = tl;
      while (rem) {
        const u32 n = umin32(FW_PLEN, rem);
        literal(off, n, n == rem);
        off += n; rem -= n;
      }
    }
  }
};

template <bool BUILD, class W, class S>
A5X_HD Plan plan_word(const W& wd, u32 L, const Tab& T, S& sk, u32 balanced_cap = 0) {
  Planner<BUILD, W, S> pl(wd, T, sk, balanced_cap);
  u32 p = 0;
  Unit U;
  while (pl.P.ok && next_unit(wd, L, p, T, U)) pl.unit(U);
  pl.finish(L);
  pl.pick_balanced();
  return pl.P;
}

// The balanced grouping's cap for a FAST word of P = prod R = count + 1: the fewest big
// pieces nb with FB_RMAX^nb >= P, then about P^(1 / nb) with slack for the
// discreteness of the small pieces' R (slack8 in 1/8 units; 0: no balanced grouping).
#ifndef FB_BAL_SLACK8
#define FB_BAL_SLACK8 0  // off: measured on C3 (A/B, one box) the balanced grouping left the
                         // expansion at 8.78-8.80 ms and cost the keyspace 0.54 ms (3.14 -> 3.68)
#endif
A5X_HD u32 fb_balanced_cap(u64 P, u32 slack8 = FB_BAL_SLACK8) {
  if (!slack8 || P <= FB_RMAX) return 0;
  u32 nb = 1;
  for (u64 x = FB_RMAX; x < P && nb < FB_NMAX; nb++) x *= FB_RMAX;
  u32 r = 2;
  while (r < FB_RMAX) {
    u64 x = 1;
    for (u32 i = 0; i < nb && x < P; i++) x *= r;
    if (x >= P) break;
    r++;
  }
  const u32 c = (r * slack8 + 7u) / 8u;
  return c < r ? r : (c > FB_RMAX ? FB_RMAX : c);
}

// The unit of a lone match of key k at position s (next_unit's single-match case).
A5X_HD void lone_unit(const Tab& T, u32 s, u32 k, Unit& U) {
  const A5xKey key = T.keys[k];
  U.s = s; U.e = s + key.klen; U.nm = 1;
  U.key = k; U.k = 0; U.m0 = 0; U.m1 = 0; U.cb = key.choice_base;
  U.R = key.nvals + 1u; U.ml = key.maxclen; U.mnl = key.minclen;
  U.spos = key.sum_dpos; U.sneg = key.sum_dneg; U.maxd = key.maxdelta;
  U.ok = true;
}

// ---------------------------------------------------------------------------
// keyspace of one word by the unit closed form (k_keyspace_thread)
// ---------------------------------------------------------------------------
struct WordClass {
  u64 count, bytes;
  u32 flags;       // A5X_WF_* (+ FAST fields) or A5X_WF_DEFER
  bool ovf;        // count/bytes overflow u64
  bool clusters;   // the word has overlapping-key units (the slow path needs the DP)
};

// Closed-form keyspace accumulated unit by unit (P = product of R,
// bytes = (P - 1)(L + 1) + signed length deltas), plus the word-shape facts the
// class decision needs.
struct CountAcc {
  u64 P, Dp, Dn;
  u32 nmatch, nunits, maxl;
  bool bin, clusters, ok, ovf;
};
A5X_HD void count_init(CountAcc& A, u32 L) {
  A.P = 1; A.Dp = 0; A.Dn = 0; A.nmatch = 0; A.nunits = 0; A.maxl = L + 1;
  A.bin = true; A.clusters = false; A.ok = true; A.ovf = false;
}
A5X_HD void count_unit(CountAcc& A, const Unit& U) {
  A.nunits++;
  A.nmatch += U.nm;
  if (U.k) {
    A.clusters = true;
    if (!U.ok) A.ok = false;
  }
  const u64 R = U.R;
  // sum over the unit's choices of (|choice| - span), split by sign
  A.Dp = add_ovf(mul_ovf(A.Dp, R, A.ovf), mul_ovf(A.P, U.spos, A.ovf), A.ovf);
  A.Dn = add_ovf(mul_ovf(A.Dn, R, A.ovf), mul_ovf(A.P, U.sneg, A.ovf), A.ovf);
  A.P = mul_ovf(A.P, R, A.ovf);
  if (U.k || U.R != 2) A.bin = false;
  if (U.maxd > 0) A.maxl += (u32)U.maxd;
}

// The class decision from the accumulated units and the piece plan.  ringmax: the
// slow kernel's per-wave ring (a radix word's longest candidate must fit).
A5X_HD WordClass classify_finish(const CountAcc& A, const Plan& PL, u32 L, int mn, int mx, u32 ringmax) {
  WordClass C;
  C.count = 0; C.bytes = 0; C.flags = 0; C.ovf = false; C.clusters = A.clusters;
  if (A.ok && A.nunits == 0) {
    C.flags = A5X_WF_RADIX | A5X_WF_FAST;
    return C;
  }
  const bool freew = (mn <= 1) && ((i64)A.nmatch <= (i64)mx);
  if (!A.ok || !freew || A.ovf || A.P > (1ull << 32) || A.maxl > ringmax) {
    C.flags = A5X_WF_DEFER;
    return C;
  }
  bool o2 = false;
  const u64 cnt = A.P - 1;
  u64 byt = add_ovf(mul_ovf(cnt, (u64)L + 1, o2), A.Dp, o2);
  if (byt < A.Dn) o2 = true;
  byt -= A.Dn;
  if (o2) {
    C.flags = A5X_WF_ERR_OVF;
    C.ovf = true;
    return C;
  }
  C.count = cnt; C.bytes = byt;
  // minl >= 3: a candidate completes the dword that holds its first byte (see
  // fb_put); maxl bounds the per-round ring use
  const bool fast = PL.ok && PL.np <= FW_PMAX && PL.ne <= 255 && 1 + PL.np + PL.ne <= FW_RMAX &&
                    PL.maxl <= FW_MAXL && PL.minl >= 3 && A.P <= FW_PMAX_CNT && PL.nbig <= FB_NMAX &&
                    PL.bent <= FB_EMAX;
  if (fast) {
    C.flags = (A.clusters ? 0u : (A5X_WF_RADIX | (A.bin ? A5X_WF_BIN : 0u))) | A5X_WF_FAST | (PL.ng << 10) |
              (PL.ne << 16) | (PL.np << 24);
  } else {
    // the slow kernel re-derives the word (radix or DP walk); clusters need its DP
    C.flags = A.clusters ? 0u : (A5X_WF_RADIX | (A.bin ? A5X_WF_BIN : 0u));
  }
  return C;
}

// One walk over the units: counts and the piece plan (count mode) together.
template <class W>
A5X_HD WordClass classify_word(const W& wd, u32 L, const Tab& T, int mn, int mx, u32 ringmax) {
  if (mx < 1 || L == 0) {  // processWord emits nothing
    WordClass C;
    C.count = 0; C.bytes = 0; C.ovf = false; C.clusters = false;
    C.flags = A5X_WF_RADIX | A5X_WF_FAST;
    return C;
  }
  CountAcc A;
  count_init(A, L);
  NullSink ns;
  Planner<false, W, NullSink> pl(wd, T, ns);
  u32 p = 0;
  Unit U;
  while (next_unit(wd, L, p, T, U)) {
    count_unit(A, U);
    if (!A.ok) break;
    pl.unit(U);
  }
  pl.finish(L);
  return classify_finish(A, pl.P, L, mn, mx, ringmax);
}

// ---------------------------------------------------------------------------
// k_expand_fast, per candidate (host replay in a5x_debug_plan_word)
// ---------------------------------------------------------------------------
// pass 1 over the window records wrec: word with its np piece descriptors at
// wrec[ga, ga + np) and entries from wrec[wbe]; n = rank in the word + 1.  Each
// piece takes its digit of n and selects its entry e[i].  NPM >= np fixed
// iterations (so the descriptor and entry loads are issued back to back): pieces
// past np select the empty entry wrec[FX_ZSLOT].  Returns the candidate's length
// including '\n'.
template <int NPM>
A5X_HD u32 fw_pass1(const u64* wrec, u32 ga, u32 np, u32 wbe, u32 n, u64* e) {
  u64 G[NPM];
#pragma unroll
  for (int i = 0; i < NPM; i++) G[i] = wrec[ga + i];  // past np: whatever follows (unused)
  u32 idx[NPM];
#pragma unroll
  for (int i = 0; i < NPM; i++) {
    const u32 ghi = (u32)(G[i] >> 32);
    u32 q = (u32)(((u64)n * (u32)G[i]) >> 32);
    q += n & (u32)((int)ghi >> 31);  // R = 1: q = n
    const u32 d = n - q * (((ghi >> 8) & 31u) + 1u);
    n = q;
    idx[i] = (u32)i < np ? wbe + (ghi & 255u) + d : (u32)FX_ZSLOT;
  }
  u32 len = 0;
#pragma unroll
  for (int i = 0; i < NPM; i++) {
    e[i] = wrec[idx[i]];
    len += (u32)(e[i] >> 56) & 7u;
  }
  return len;
}

// pass 2: the candidate's pieces e[0, NPM) appended to the output as whole,
// aligned dwords of a ring, with plain stores and no atomics.  Byte o (ring
// offset) is the candidate's first; acc holds the o & 3 bytes before it: the
// previous candidate's tail for a round's first lane (the carry), zeros otherwise.
// Dword ownership: the dword holding byte o belongs to the PREVIOUS candidate
// unless acc is the carry (has_prev = false): it is returned in *head (zeros below
// o) for the previous lane to merge into its last partial dword, which it writes.
// Requires every candidate to complete that dword (len >= 3, FAST minl).  Stores
// that are not due go to ring[trash] (a per-lane scratch dword): no branches.
// Returns the ring dword of the unfinished last dword; *acc_io / *n_io = its
// bytes / count.
template <int NPM>
A5X_HD u32 fw_pass2(const u64* e, u32 o, u32* ring, u32 trash, bool has_prev, u32* acc_io, u32* n_io, u32* head) {
  u32 acc = *acc_io, n = o & 3u, D = o >> 2;
  bool hp = has_prev && n != 0;
  u32 hd = 0;
#pragma unroll
  for (int i = 0; i < NPM; i++) {
    const u32 ehi = (u32)(e[i] >> 32);
    const u32 t = n + ((ehi >> 24) & 7u);
    const u32 chi = ehi & 0xFFFFFFu;
    const u64 lo = ((((u64)chi << 32) | (u32)e[i]) << (8u * n)) | acc;
    // bytes 8, 9 (only needed when t >= 8, i.e. n >= 1): chi >> (32 - 8n)
#ifdef __HIP_DEVICE_COMPILE__
    const u32 hi = __builtin_amdgcn_alignbyte(0u, chi, 0u - n);
#else
    const u32 hi = (u32)((((u64)chi << 32) >> (32u - 8u * (n & 3u))) >> 32);
#endif
    const bool c4 = t >= 4u, c8 = t >= 8u;
    ring[(c4 && !hp) ? D : trash] = (u32)lo;
    ring[c8 ? D + 1u : trash] = (u32)(lo >> 32);
    hd = (c4 && hp) ? (u32)lo : hd;
    hp = hp && !c4;
    acc = c8 ? hi : (c4 ? (u32)(lo >> 32) : (u32)lo);
    D += t >> 2;
    n = t & 3u;
  }
  *acc_io = acc;
  *n_io = n;
  *head = hd;
  return D;
}

// ---------------------------------------------------------------------------
// Big pieces (k_expand_fast): the small pieces [bstart(b), bstart(b+1)) of a
// word combined into one <= FB_PLEN-byte piece with R_b = product of their R
// combinations (R_b <= FB_RMAX), stored as 16-B entries: bytes 0-14 content (zero
// past the length), byte 15 = length.  Combination c of big piece b is the
// mixed-radix digit vector of its small pieces (first small piece least
// significant), so the big pieces are digits of n in the same order.
// ---------------------------------------------------------------------------
A5X_HD u32 fb_perm(u32 hi, u32 lo, u32 sel) {  // v_perm_b32 for selectors with bytes < 8
#ifdef __HIP_DEVICE_COMPILE__
  return __builtin_amdgcn_perm(hi, lo, sel);
#else
  const u64 v = ((u64)hi << 32) | lo;
  u32 r = 0;
  for (u32 i = 0; i < 4; i++) r |= (u32)((v >> (8 * ((sel >> (8 * i)) & 7u))) & 255u) << (8 * i);
  return r;
#endif
}

// R of big piece b of the word whose record is at wrec[wrb] (header h)
A5X_HD u32 fb_R(const u64* wrec, u32 wrb, u64 h, u32 b) {
  const u32 nb = frh_nbig(h), np = frh_np(h);
  if (b >= nb) return 1;
  const u32 s0 = frh_bstart(h, b), s1 = b + 1 < nb ? frh_bstart(h, b + 1) : np;
  u32 R = 1;
  for (u32 i = s0; i < s1 && i < FW_PMAX; i++) R *= frd_R(wrec[wrb + 1 + i]);
  return R;
}

// entry c of big piece b (x, y, z, w = bytes 0-3, 4-7, 8-11, 12-14 + length)
A5X_HD void fb_entry(const u64* wrec, u32 wrb, u32 b, u32 c, u32 out[4], u32 zslot = FX_ZSLOT) {
  const u64 h = wrec[wrb];
  const u32 nb = frh_nbig(h), np = frh_np(h);
  const u32 sp0 = frh_bstart(h, b), sp1 = b + 1 < nb ? frh_bstart(h, b + 1) : np;
  const u32 wbe = wrb + 1 + np;
  u64 lo64 = 0, hi64 = 0;
  u32 off = 0;
#pragma unroll
  for (u32 i = 0; i < FB_SPAN; i++) {
    const bool valid = sp0 + i < sp1;
    const u64 G = wrec[valid ? wrb + 1 + sp0 + i : zslot];
    const u32 ghi = (u32)(G >> 32);
    u32 q = (u32)(((u64)c * (u32)G) >> 32);
    q += c & (u32)((int)ghi >> 31);  // R = 1: q = c
    const u32 d = c - q * (((ghi >> 8) & 31u) + 1u);
    c = q;
    const u64 ev = wrec[valid ? wbe + (ghi & 255u) + d : zslot];
    const u64 cv = ev & FW_M56;
    if (off < 8) {
      lo64 |= cv << (8 * off);
      if (off) hi64 |= cv >> (64 - 8 * off);
    } else {
      hi64 |= cv << (8 * (off - 8));
    }
    off += fw_len(ev);
  }
  out[0] = (u32)lo64; out[1] = (u32)(lo64 >> 32); out[2] = (u32)hi64;
  out[3] = ((u32)(hi64 >> 32) & 0xFFFFFFu) | (off << 24);
}

// One big piece appended to a candidate's output as whole, aligned dwords of a
// ring: entry e (e[3] byte 3 = length) after the n pending bytes held in the TOP n
// bytes of pv; complete dwords go to ring[D ..].  Dword ownership: the dword
// holding a candidate's first byte belongs to the PREVIOUS candidate unless the
// pending bytes are the carry; while hp is set, the first complete dword is kept in
// hd (zeros below the candidate's first byte) for the previous lane to merge into
// its last partial dword.  Stores that are not due go to ring[T + k] (the lane's 4
// trash dwords): no branches.  acc = the unfinished dword (bottom-aligned n bytes).
A5X_HD void fb_put(const u32 e[4], u32& pv, u32& n, u32& D, bool& hp, u32& hd, u32& acc, u32* ring, u32 T) {
  const u32 sel = (u32)(0x0706050403020100ull >> (32u - 8u * n));  // bytes 4-n .. 7-n of {s_k, s_k-1}
  const u32 s3 = e[3] & 0xFFFFFFu;
  const u32 w0 = fb_perm(e[0], pv, sel);
  const u32 w1 = fb_perm(e[1], e[0], sel);
  const u32 w2 = fb_perm(e[2], e[1], sel);
  const u32 w3 = fb_perm(s3, e[2], sel);
  const u32 w4 = fb_perm(0u, s3, sel);
  const u32 t = n + (e[3] >> 24);
  const bool m1 = t >= 4u, m2 = t >= 8u, m3 = t >= 12u, m4 = t >= 16u;
  ring[(m1 && !hp) ? D : T] = w0;
  ring[(m2 ? D : T) + 1u] = w1;
  ring[(m3 ? D : T) + 2u] = w2;
  ring[(m4 ? D : T) + 3u] = w3;
  hd = (m1 && hp) ? w0 : hd;
  hp = hp && !m1;
  u32 x = m1 ? w1 : w0;
  x = m2 ? w2 : x;
  x = m3 ? w3 : x;
  x = m4 ? w4 : x;
  acc = x;
  n = t & 3u;
  pv = acc << ((32u - 8u * n) & 31u);
  D += t >> 2;
}
