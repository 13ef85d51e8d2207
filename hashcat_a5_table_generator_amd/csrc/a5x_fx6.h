// a5x_fx6.h -- round machinery of k_expand_fast (device only; included by
// a5x_kernels.hip).
//
// A window holds the big-piece entries of up to FX_WW consecutive FAST words in LDS
// (a5x_plan.h: a word's candidate n <-> the mixed-radix digits of n + 1 over its big
// pieces, piece 0 least significant).  A round covers 64 * K consecutive candidates of
// the window: lane L takes the RUN of candidates [K L, K L + K) (consecutive ranks of
// one word), so after one division per run the digits advance as an odometer.  Per round:
//   pass 1  digits -> entry indices -> candidate lengths;
//   scan    DPP wave prefix sum of the run lengths -> byte offset of every run;
//   pass 2  every piece ORed into the per-wave LDS ring at its byte offset (a5x_ring.h
//           fx7_put: the ring is zero between flushes and entries are zero past their
//           length, so no ordering or cross-lane merge is needed);
//   flush   complete 16-B ring blocks -> global_store_dwordx4 (1 KiB per instruction),
//           the ring zeroed behind them.
#pragma once

#ifndef FX_HOLDNB
#define FX_HOLDNB 2      // rounds of <= this many big pieces keep their entries in registers
#endif
#ifndef FX6_SWZ
#define FX6_SWZ 0        // XOR-swizzled ring (FX_SWZ of the includer)
#endif
#ifndef FX6_ABL
#define FX6_ABL 0        // timing ablations (FX_ABL of the includer)
#endif
#ifndef FX6_ZBE
#define FX6_ZBE 255      // the window entry that holds the empty piece (set by the includer)
#endif

// (FxRun, the wave's staging state, and the ring flush are defined by the includer.)

#include "a5x_ring.h"

// Per window word j: q0 = {magic of big pieces 0..3}, q1 = {R-1 of pieces 0..3 (6 bits
// each), entry base of pieces 0/1 (16 bits each), pieces 2/3, first run of the word
// (window-relative; a run = FX6 K consecutive ranks of one word)}.  Pieces past the
// word's count have R = 1 and base FX6_ZBE (they read the empty entry).
__device__ __forceinline__ u32 fx6_r(u32 rm, int b) { return ((rm >> (6 * b)) & 63u) + 1u; }

template <int NB>
__device__ __forceinline__ void fx6_digits(u32 n, const uint4 q0, u32 rm, u32 (&d)[4]) {
#pragma unroll
  for (int b = 0; b < NB; b++) {
    const u32 mg = b == 0 ? q0.x : b == 1 ? q0.y : b == 2 ? q0.z : q0.w;
    const u32 q = __umulhi(n, mg) + (mg ? 0u : n);
    d[b] = n - __umul24(q, fx6_r(rm, b));
    n = q;
  }
}

// odometer step (ranks of one word): d0 + 1 with carries
template <int NB>
__device__ __forceinline__ void fx6_step(u32 rm, u32 (&d)[4]) {
  u32 cy = 1;
#pragma unroll
  for (int b = 0; b < NB; b++) {
    const u32 nd = d[b] + cy;
    cy = nd >= fx6_r(rm, b) ? 1u : 0u;
    d[b] = cy ? 0u : nd;
  }
}

__device__ __forceinline__ u32 fx6_eb(const uint4 q1, int b) {
  return b == 0 ? (q1.y & 0xFFFFu) : b == 1 ? (q1.y >> 16) : b == 2 ? (q1.z & 0xFFFFu) : (q1.z >> 16);
}

// Window word of each lane's run: j = last word whose first run <= rr + lane.
// rw = the per-lane register holding word lane's first run (lanes >= k: ~0);
// jcur (uniform, in/out) = word of run rr; nl = runs in the round.
__device__ __forceinline__ u32 fx6_word(u32 rw, u32 k, u32 rr, u32 nl, u32& jcur) {
  while (jcur + 1 < k && readlane_u32(rw, jcur + 1) <= rr) jcur++;
  const u32 r = rr + lane_id();
  u32 j = jcur;
  for (u32 jn = jcur + 1; jn < k; jn++) {
    const u32 sj = readlane_u32(rw, jn);
    if (sj >= rr + nl) break;
    j += r >= sj ? 1u : 0u;
  }
  return j;
}

// One round: window runs [rr, rr + nl): lane L < nl takes run rr + L of window word j
// (ranks rb[j] + K (run - first run of j) .. + K, clipped to the word's rank end re[j];
// words start on run boundaries, so a run never crosses words).  be / wq / rb / re: the
// window's entries and per-word info in LDS; ring = LDS byte address of ring byte 0.
// Runs are taken while they fit cap ring bytes (a prefix: the scan is monotonic; the
// rest wait for the next round); returns the runs taken (uniform).
// A lane's run of the last round, for the fused digest (FLUSH::DIGEST): ring byte
// offset of its first candidate, candidate lengths ('\n' included), window word, rank.
#ifndef FX6_KMAX
#define FX6_KMAX 4       // candidates per lane run (FX_K of the includer)
#endif
struct FxLaneRun {
  u32 off, nc, j, st;
  u32 clen[FX6_KMAX];
};

template <int NB, int K, class FLUSH>
__device__ __forceinline__ u32 fx7_round(const uint4* be, const uint4 (*wq)[2], const u32* rb, const u32* re, u32 ring,
                                         u32 cap, FxRun& R, u32 rr, u32 j, bool act, FLUSH& flush, FxLaneRun& lr) {
  static_assert(K <= FX6_KMAX, "FxLaneRun holds FX6_KMAX candidates");
  constexpr bool SWZ = FX6_SWZ && !FLUSH::DIGEST;  // (the digest reads its candidates linearly)
  const u32 lane = lane_id();
  const uint4 q0 = wq[j][0], q1 = wq[j][1];
  const u32 st = act ? (rr + lane - q1.w) * K + rb[j] : 0u;  // first rank of the run
  const u32 cw = act ? re[j] : 0u;
  const u32 nc = cw > st ? min((u32)K, cw - st) : 0u;
  u32 d[4];
  fx6_digits<NB>(st + 1u, q0, q1.x, d);
  constexpr bool HOLD = NB <= FX_HOLDNB;
  uint4 ent[HOLD ? K : 1][HOLD ? NB : 1];
  u32 idx[HOLD ? 1 : K][HOLD ? 1 : NB];
  u32 len = 0, clen[K];
  const uint8_t* lenb = (const uint8_t*)be + 15;
#pragma unroll
  for (int c = 0; c < K; c++) {
    if (c > 0) fx6_step<NB>(q1.x, d);
    clen[c] = 0;
#pragma unroll
    for (int b = 0; b < NB; b++) {
      const u32 ix = c < (int)nc ? fx6_eb(q1, b) + d[b] : (u32)FX6_ZBE;  // past the run: empty
      if constexpr (HOLD) {
        ent[c][b] = be[ix];
        clen[c] += ent[c][b].w >> 24;
      } else {
        idx[c][b] = ix;
        clen[c] += lenb[16u * ix];
      }
    }
    len += clen[c];
  }
  const u32 incl = wave_incl_scan_u32(len);
  const u32 used = (u32)(R.pos - R.B);
  const bool fit = nc > 0 && used + incl <= cap;
  const u32 nact = uniform((u32)__popcll(__ballot(fit)));
  const u32 tot = nact ? readlane_u32(incl, nact - 1u) : 0u;
  u32 P = ring + used + incl - len;
  if (fit && !(FX6_ABL & 64)) {  // (FX_ABL 64: no placement, timing ablation)
    if constexpr (HOLD) {
#pragma unroll
      for (int c = 0; c < K; c++)
#pragma unroll
        for (int b = 0; b < NB; b++) fx7_put<SWZ>(ent[c][b], P);
    } else {
      // Entries read again here, one candidate ahead: candidate c + 1's NB reads are
      // issued before candidate c's ORs (in the same basic block, ahead of the puts'
      // uniform branches), so each candidate waits only for its own reads
      // (lgkmcnt(#ORs since)).  Read right before its put, every piece cost a full LDS
      // round trip behind the previous piece's ORs (s_waitcnt lgkmcnt(0)).
      uint4 cur[NB], nxt[NB];
#pragma unroll
      for (int b = 0; b < NB; b++) cur[b] = be[idx[0][b]];
#pragma unroll
      for (int c = 0; c < K; c++) {
        if (c + 1 < K) {
#pragma unroll
          for (int b = 0; b < NB; b++) nxt[b] = be[idx[c + 1][b]];
        }
#pragma unroll
        for (int b = 0; b < NB; b++) fx7_put<SWZ>(cur[b], P);
        if (c + 1 < K) {
#pragma unroll
          for (int b = 0; b < NB; b++) cur[b] = nxt[b];
        }
      }
    }
  }
  R.pos = uniform64(R.pos + tot);
  WAVE_SYNC();
  if constexpr (FLUSH::DIGEST) {  // the caller hashes the runs where they were placed
    lr.off = used + incl - len;
    lr.nc = fit ? nc : 0u;
    lr.j = j;
    lr.st = st;
#pragma unroll
    for (int c = 0; c < FX6_KMAX; c++) lr.clen[c] = c < K ? clen[c] : 0u;
  } else {
    flush(R);
  }
  return nact;
}
