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
};

A5X_HD Tab tab_view(const uint8_t* base) {
  Tab t;
  t.hdr = (const A5xTableHdr*)base;
  t.bucket = (const uint16_t*)(base + t.hdr->off_bucket);
  t.keys = (const A5xKey*)(base + t.hdr->off_keys);
  t.ch = (const A5xChoice*)(base + t.hdr->off_choices);
  t.blob = base + t.hdr->off_blob;
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
// FAST window format (see k_expand_fast)
// ---------------------------------------------------------------------------
#define FW_WB 512   // window word-byte budget
#define FW_WG 64    // window group-piece budget
#define FW_WE 512   // window entry budget (u64 each)
#define FW_WW 32    // window word budget
#define FW_PMAX 20  // pieces per word (6-bit digit|R-1 fields, 10 per u64, two u64)
#define FW_PLEN 7   // bytes per piece
#define FW_RING 4096
#define FW_UMAXM 8  // matches per cluster unit
#define FW_UMAXR 8  // choices per unit / group

static_assert(FW_WE <= 65535 && FW_WG <= 255, "window budgets");

struct FGroup {   // 16 B, one per group piece
  u32 magic;
  uint8_t shift, R, dsh, dhi;   // digit field of piece i: dsh = 6 (i mod 10), dhi = i >= 10
  u32 plen;                     // 4-bit length of entry a at bits 4a
  u32 pad1;
};
struct FWord {    // 32 B
  uint16_t gbase, ng, ebase, np;
  u32 lconst;     // bytes of the literal pieces (digit-independent)
  u32 maxl;       // longest candidate + '\n'
  u64 c0;         // first global candidate index of the word
  u64 pad;
};
struct FWin {
  u32 bytes32[(FW_WB + 32) / 4];
  FGroup groups[FW_WG];
  u64 ent[FW_WE];
  FWord words[FW_WW];
};

#define FW_M56 0x00FFFFFFFFFFFFFFull
A5X_HD u64 fw_meta(u32 len, u32 R) { return (u64)(len | ((R - 1u) << 3)) << 56; }
A5X_HD u32 fw_len(u64 e) { return (u32)(e >> 56) & 7u; }
A5X_HD u64 keep_bytes64(u64 v, u32 n) { return n >= 8 ? v : (v & ((1ull << (8 * n)) - 1ull)); }

// FAST flag fields (written by the keyspace pass)
A5X_HD u32 ff_ng(u32 f) { return (f >> 10) & 31u; }
A5X_HD u32 ff_ne(u32 f) { return (f >> 16) & 255u; }
A5X_HD u32 ff_np(u32 f) { return (f >> 24) & 31u; }

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
  u32 spos, sneg;  // sums over choices of max(len - span, 0) and max(span - len, 0)
  int maxd;        // longest choice - span
  u32 nm;          // key matches in the unit (bounds the substitutions of a choice)
  u32 key;         // lone match: its key index
  u32 k;           // cluster: number of matches (0 for a lone match)
  u64 m0, m1;      // cluster matches 0-3 / 4-7, 16 bits each: (pos - s) << 10 | key index
  bool ok;         // cluster fits FW_UMAXM matches, FW_UMAXR choices of <= FW_PLEN bytes
};

A5X_HD u32 unit_mkey(const Unit& U, u32 j) { return (u32)((j < 4 ? U.m0 : U.m1) >> (16 * (j & 3))) & 1023u; }
A5X_HD u32 unit_mpos(const Unit& U, u32 j) { return U.s + ((u32)((j < 4 ? U.m0 : U.m1) >> (16 * (j & 3) + 10)) & 63u); }

// Enumerate the choices of a cluster in a fixed order (match subsets by increasing
// bitmask, then values as an odometer, first match fastest); choice 0 is the empty
// subset.  target < 0: statistics only (R, ml, spos, sneg, maxd, ok); else stop at
// choice `target` and return its bytes (len <= FW_PLEN) in *content / *len.
template <class W>
A5X_HD void cluster_choices(const W& wd, Unit& U, const Tab& T, int target, u64* content, u32* len) {
  const u32 span = U.e - U.s;
  u32 R = 0, ml = 0, spos = 0, sneg = 0;
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
      R++;
      ml = umax32(ml, n);
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
  U.R = R; U.ml = ml; U.spos = spos; U.sneg = sneg; U.maxd = maxd; U.ok = ok;
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
      U.key = k0; U.k = 0;
      U.R = key.nvals + 1u; U.ml = key.maxclen;
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
  if (U.k == 0) {
    const u32 ci = T.keys[U.key].choice_base + a;
    len = T.ch[ci].len;
    return choice7(T, ci);
  }
  Unit V = U;
  u64 v = 0;
  len = 0;
  cluster_choices(wd, V, T, (int)a, &v, &len);
  return v;
}

// ---------------------------------------------------------------------------
// piece plan
// ---------------------------------------------------------------------------
struct Plan {
  u32 np, ng, ne, lconst, maxl;
  bool ok;
};

// Cut a unit-radix word into pieces (see k_expand_fast).  BUILD also writes the
// window's entries (from entry index e0) and FGroups (from g0).
template <bool BUILD, class W>
A5X_HD Plan plan_word(const W& wd, u32 L, const Tab& T, FWin* F, u32 g0, u32 e0) {
  Plan P;
  P.np = 0; P.ng = 0; P.ne = 0; P.lconst = 0; P.maxl = 0; P.ok = true;
  bool open = false;  // a group piece is being built
  u32 cR = 1, cmax = 0, ceb = 0, cpi = 0, cplen = 0;
  u32 prev = 0, p = 0;
  Unit U;
  while (P.ok && next_unit(wd, L, p, T, U)) {
    const u32 Ru = U.R, ml = U.ml, run = U.s - prev;
    if (!U.ok || ml > FW_PLEN || Ru > FW_UMAXR) { P.ok = false; break; }
    if (open && cmax + run + ml <= FW_PLEN && cR * Ru <= FW_UMAXR) {
      // merge: entry a1 + cR * a2 = old[a1] ++ run ++ choice a2 (descending: in place)
      const u32 nR = cR * Ru;
      if constexpr (BUILD) {
        u32 nplen = 0;
        const u64 rb = run ? wd.ld(prev, run) : 0ull;
        for (int a2 = (int)Ru - 1; a2 >= 0; a2--) {
          u32 cl = 0;
          const u64 cv = unit_choice(wd, U, T, (u32)a2, cl);
          for (int a1 = (int)cR - 1; a1 >= 0; a1--) {
            const u32 ia = ceb + (u32)a1, ib = ceb + (u32)a1 + cR * (u32)a2;
            const u64 old = (ia < FW_WE) ? F->ent[ia] : 0ull;
            const u32 ol = fw_len(old);
            const u32 nl = ol + run + cl;
            const u64 v = (old & FW_M56) | (rb << (8 * ol)) | (cv << (8 * (ol + run)));
            if (ib < FW_WE) F->ent[ib] = (v & FW_M56) | fw_meta(nl, nR);
            nplen |= nl << (4 * ((u32)a1 + cR * (u32)a2));
          }
        }
        cplen = nplen;
      }
      P.ne += nR - cR;
      cR = nR; cmax += run + ml;
    } else {
      if (open) {  // close the group piece
        if constexpr (BUILD) {
          if (g0 + P.ng < FW_WG) {
            FGroup G;
            u32 mg, sh;
            divmagic(cR, mg, sh);
            G.magic = mg; G.shift = (uint8_t)sh; G.R = (uint8_t)cR; G.dsh = (uint8_t)(6 * (cpi % 10));
            G.dhi = (uint8_t)(cpi >= 10); G.plen = cplen; G.pad1 = 0;
            F->groups[g0 + P.ng] = G;
          }
        }
        P.ng++; P.maxl += cmax;
        open = false;
      }
      u32 off = prev, rem = run;
      while (rem + ml > FW_PLEN) {  // literal run that does not fit with the unit
        const u32 n = umin32(FW_PLEN, rem);
        if constexpr (BUILD) {
          if (e0 + P.ne < FW_WE) F->ent[e0 + P.ne] = wd.ld(off, n) | fw_meta(n, 1);
        }
        P.ne++; P.np++; P.lconst += n; P.maxl += n;
        off += n; rem -= n;
      }
      open = true; cR = Ru; cmax = rem + ml; ceb = e0 + P.ne; cpi = P.np; cplen = 0;
      if constexpr (BUILD) {
        const u64 rb = rem ? wd.ld(off, rem) : 0ull;
        for (u32 a = 0; a < Ru; a++) {
          u32 cl = 0;
          const u64 cv = unit_choice(wd, U, T, a, cl);
          const u64 v = rb | (cv << (8 * rem));
          if (ceb + a < FW_WE) F->ent[ceb + a] = (v & FW_M56) | fw_meta(rem + cl, Ru);
          cplen |= (rem + cl) << (4 * a);
        }
      }
      P.ne += Ru; P.np++;
    }
    prev = U.e;
  }
  if (!P.ok) return P;
  // tail bytes + '\n'
  const u32 run = L - prev, tl = run + 1;
  if (open && cmax + tl <= FW_PLEN) {
    if constexpr (BUILD) {
      const u64 tb = (run ? wd.ld(prev, run) : 0ull) | (10ull << (8 * run));
      u32 nplen = 0;
      for (u32 a = 0; a < cR; a++) {
        const u32 ia = ceb + a;
        const u64 old = (ia < FW_WE) ? F->ent[ia] : 0ull;
        const u32 ol = fw_len(old);
        if (ia < FW_WE) F->ent[ia] = ((old | (tb << (8 * ol))) & FW_M56) | fw_meta(ol + tl, cR);
        nplen |= (ol + tl) << (4 * a);
      }
      cplen = nplen;
    }
    cmax += tl;
  } else {
    if (open) {
      if constexpr (BUILD) {
        if (g0 + P.ng < FW_WG) {
          FGroup G;
          u32 mg, sh;
          divmagic(cR, mg, sh);
          G.magic = mg; G.shift = (uint8_t)sh; G.R = (uint8_t)cR; G.dsh = (uint8_t)(6 * (cpi % 10));
          G.dhi = (uint8_t)(cpi >= 10); G.plen = cplen; G.pad1 = 0;
          F->groups[g0 + P.ng] = G;
        }
      }
      P.ng++; P.maxl += cmax;
      open = false;
    }
    u32 off = prev, rem = tl;
    while (rem) {
      const u32 n = umin32(FW_PLEN, rem);
      if constexpr (BUILD) {
        const bool last = n == rem;
        const u32 nb = last ? n - 1 : n;
        u64 v = nb ? wd.ld(off, nb) : 0ull;
        if (last) v |= 10ull << (8 * nb);
        if (e0 + P.ne < FW_WE) F->ent[e0 + P.ne] = v | fw_meta(n, 1);
      }
      P.ne++; P.np++; P.lconst += n; P.maxl += n;
      off += n; rem -= n;
    }
  }
  if (open) {
    if constexpr (BUILD) {
      if (g0 + P.ng < FW_WG) {
        FGroup G;
        u32 mg, sh;
        divmagic(cR, mg, sh);
        G.magic = mg; G.shift = (uint8_t)sh; G.R = (uint8_t)cR; G.dsh = (uint8_t)(6 * (cpi % 10));
        G.dhi = (uint8_t)(cpi >= 10); G.plen = cplen; G.pad1 = 0;
        F->groups[g0 + P.ng] = G;
      }
    }
    P.ng++; P.maxl += cmax;
  }
  return P;
}

// ---------------------------------------------------------------------------
// keyspace of one word by the unit closed form (k_keyspace_thread)
// ---------------------------------------------------------------------------
struct WordClass {
  u64 count, bytes;
  u32 flags;       // A5X_WF_* (+ FAST fields) or A5X_WF_DEFER
  bool ovf;        // count/bytes overflow u64
};

// ringmax: the slow kernel's per-wave ring (a radix word's longest candidate must fit)
template <class W>
A5X_HD WordClass classify_word(const W& wd, u32 L, const Tab& T, int mn, int mx, u32 ringmax) {
  WordClass C;
  C.count = 0; C.bytes = 0; C.flags = 0; C.ovf = false;
  if (mx < 1 || L == 0) {  // processWord emits nothing
    C.flags = A5X_WF_RADIX | A5X_WF_FAST;
    return C;
  }
  u32 p = 0, nmatch = 0, maxl = L + 1, nunits = 0;
  bool bin = true, clusters = false, ok = true, ovf = false;
  u64 P = 1, Dp = 0, Dn = 0;
  Unit U;
  while (next_unit(wd, L, p, T, U)) {
    nunits++;
    nmatch += U.nm;
    if (U.k) {
      clusters = true;
      if (!U.ok) { ok = false; break; }
    }
    const u64 R = U.R;
    // sum over the unit's choices of (|choice| - span), split by sign
    Dp = add_ovf(mul_ovf(Dp, R, ovf), mul_ovf(P, U.spos, ovf), ovf);
    Dn = add_ovf(mul_ovf(Dn, R, ovf), mul_ovf(P, U.sneg, ovf), ovf);
    P = mul_ovf(P, R, ovf);
    if (U.k || U.R != 2) bin = false;
    if (U.maxd > 0) maxl += (u32)U.maxd;
  }
  if (ok && nunits == 0) {
    C.flags = A5X_WF_RADIX | A5X_WF_FAST;
    return C;
  }
  const bool freew = (mn <= 1) && ((i64)nmatch <= (i64)mx);
  if (!ok || !freew || ovf || P > (1ull << 32) || maxl > ringmax) {
    C.flags = A5X_WF_DEFER;
    return C;
  }
  bool o2 = false;
  const u64 cnt = P - 1;
  u64 byt = add_ovf(mul_ovf(cnt, (u64)L + 1, o2), Dp, o2);
  if (byt < Dn) o2 = true;
  byt -= Dn;
  if (o2) {
    C.flags = A5X_WF_ERR_OVF;
    C.ovf = true;
    return C;
  }
  C.count = cnt; C.bytes = byt;
  const Plan PL = plan_word<false>(wd, L, T, (FWin*)nullptr, 0, 0);
  const bool fast = PL.ok && PL.np <= FW_PMAX && PL.ne <= 255 && PL.ng <= FW_WG && PL.maxl <= FW_RING / 2 - 16;
  if (fast) {
    C.flags = (clusters ? 0u : (A5X_WF_RADIX | (bin ? A5X_WF_BIN : 0u))) | A5X_WF_FAST | (PL.ng << 10) |
              (PL.ne << 16) | (PL.np << 24);
  } else {
    // the slow kernel re-derives the word (radix or DP walk); clusters need its DP
    C.flags = clusters ? 0u : (A5X_WF_RADIX | (bin ? A5X_WF_BIN : 0u));
  }
  return C;
}

// ---------------------------------------------------------------------------
// pass 1 of k_expand_fast for one candidate: group digits -> per-piece fields
// (digit | (R-1) << 3) << 6 (i mod 10) in dlo (pieces 0-9) / dhi (10-19); literal
// pieces keep field 0 (R = 1, entry 0).  n = candidate index in the word + 1.
// Returns the candidate's length including '\n'.
// ---------------------------------------------------------------------------
A5X_HD u32 fw_pass1(const FGroup* gp, u32 ng, u32 lconst, u32 n, u64& dlo, u64& dhi) {
  u32 len = lconst;
  dlo = 0; dhi = 0;
  for (u32 i = 0; i < ng; i++) {
    const FGroup G = gp[i];
    const u32 q = fastdiv_hd(n, G.magic, G.shift);
    const u32 d = n - q * G.R;
    n = q;
    const u64 f = (u64)(d | ((u32)(G.R - 1) << 3)) << G.dsh;
    dlo |= G.dhi ? 0ull : f;
    dhi |= G.dhi ? f : 0ull;
    len += (G.plen >> (4 * d)) & 15u;
  }
  return len;
}
