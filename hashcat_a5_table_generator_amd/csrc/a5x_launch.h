// a5x_launch.h -- host-side launch interface of a5x_kernels.hip (internal to liba5x).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

struct A5xKsLaunch {
  const uint8_t* table;
  uint32_t table_bytes;
  const uint8_t* words;
  const uint64_t* woff;
  uint64_t nw;
  int mn, mx;
  uint64_t* count;
  uint64_t* bytes;
  uint32_t* flags;
  uint32_t* defer_list;
  uint32_t* defer_n;
  uint32_t* nbig;
  uint32_t* nslow;
  uint32_t* big_list;   // nw entries each
  uint32_t* slow_list;
  uint32_t* err;
  uint32_t defer_blocks;
  uint64_t* rec;   // FAST plan records (tile regions of FW_TILE_REC u64, then complex slots)
  uint32_t* roff;  // per-word record offsets
  uint32_t* cplx_list;  // words for the general (per-lane walk) keyspace pass
  uint32_t* cplx_n;
  uint32_t cplx_cap;    // record slots of FW_RMAX u64 from rec + cplx_base
  uint64_t cplx_base;
  uint32_t* glob_list;  // words beyond the pass-B LDS budget (k_keyspace_wave appends)
  uint32_t* glob_n;
  uint8_t* gscr;        // pass G scratch: gslots x a5x_gslot_bytes() (ring zeroed)
  uint32_t gslots;
  int rmode;            // 1 / 2 / 3: -r / -s / -s -r FAST probe (k_keyspace_thread, mode_unit, then
                        // k_keyspace_rprobe over the words a tile could not decide: cplx_list,
                        // records in cplx slots); the other words are listed in defer_list / defer_n
  uint32_t rcmin;       // -r: max(min, 0)
  uint64_t* rnseg;      // -r: per FAST word, ceil(count / rseg) mode-engine items
  uint64_t rseg;
  // -s / -s -r virtual words (k_keyspace_vsub over defer_list): the words it leaves to the
  // mode engine, per word sub-words - 1 and record u64, the sub-word records (bump area)
  uint32_t* vout_list;
  uint32_t* vout_n;
  uint64_t* vn;
  uint64_t* vrsz;
  uint64_t* vrec;
  uint64_t* vrec_n;
  uint64_t vrec_cap;
  uint16_t* vocc;  // per word 16 u16: k_keyspace_thread's occurrence rows for k_keyspace_vsub (null: none)
  uint32_t* vlong_list;  // k_keyspace_vsub: words the small-slot pass hands to the large one (null: large only)
  uint32_t* vlong_n;
  uint32_t* hiflag;      // zeroed u32: k_keyspace_thread walks UTF-8 words by lead bytes (null: by bytes)
};

// the virtual word list of a batch with virtual words (k_vwords_fill)
struct A5xVwLaunch {
  const uint32_t* flags;
  const uint64_t* cand_off;
  const uint64_t* byte_off;  // null: no layout (fused digest)
  const uint32_t* roff;
  const uint64_t* rec;
  const uint64_t* vrec;
  const uint64_t* vpre;
  const uint64_t* vrpre;
  uint64_t nw;
  uint64_t* vcand_off;
  uint64_t* vbyte_off;
  uint32_t* vflags;
  uint32_t* vroff;
  uint32_t* vmap;
  uint32_t* vobase;
  uint64_t* vrec2;
  // fixed-width virtual words (A5X_WF_VFIX): their sub-words' records are written here from the
  // descriptors k_keyspace_vsub left
  const uint8_t* table;
  uint32_t table_bytes;
  int rmode;
  uint32_t rcmin;
  const uint8_t* words;
  const uint64_t* woff;
};
size_t a5x_keyspace_vsub_lds(uint32_t table_bytes);
hipError_t a5x_launch_vsub(const A5xKsLaunch& L, hipStream_t st);
hipError_t a5x_launch_vwords_sizes(const uint32_t* flags, const uint64_t* cand_off, uint64_t nw, uint64_t* vn,
                                   uint64_t* vrsz, hipStream_t st);
hipError_t a5x_launch_vwords_fill(const A5xVwLaunch& L, hipStream_t st);

struct A5xHitRaw;
struct A5xExpLaunch {
  const uint8_t* table;
  uint32_t table_bytes;
  const uint8_t* words;
  const uint64_t* woff;
  uint64_t nw;
  const uint64_t* cand_off;
  const uint64_t* byte_off;
  const uint32_t* flags;
  const uint32_t* chunk_w0;
  const uint64_t* segs;    // k_expand_slow / k_expand_b items (a5x_launch_segments)
  const uint32_t* nsegs;   // device count of segs
  uint64_t nsegs_bound;    // host bound on *nsegs
  uint64_t cand_begin, cand_end;
  uint64_t CH;
  uint64_t SEG;  // candidates per slow / BIG segment
  uint8_t* out;
  uint64_t out_base;
  uint64_t out_cap;
  int mn, mx;
  uint32_t* err;
  uint64_t* dbg;
  uint32_t waves_per_block;       // k_expand_slow
  uint32_t waves_per_block_fast;  // k_expand_fast (one wave per chunk; 1 measured fastest)
  const uint64_t* rec;
  const uint32_t* roff;
  uint64_t rec_n;   // u64 in rec
  // fused digest (kinds 3, 5): target set + hit buffer (see A5xDigLaunch)
  const uint32_t* dg_bitmap;
  uint32_t dg_bm_mask, dg_has_zero, dg_hit_cap;
  const uint4* dg_table;
  uint64_t dg_tmask;
  A5xHitRaw* dg_hits;
  uint32_t* dg_nhits;
  // pass G (words beyond the pass-B LDS budget): HBM scratch slots, one per wave
  uint8_t* gscr;
  uint32_t gslots;
  // the virtual word list (-s / -s -r batches with virtual words): entry -> word and its
  // first candidate in the word, for the fused digest's hit records (null: words)
  const uint32_t* vmap;
  const uint32_t* vobase;
};

hipError_t a5x_set_kernel_attrs();
// pass G: bytes per scratch slot (ring of A5X_RING_G bytes, then the word's WaveLds)
uint64_t a5x_gslot_bytes();
// k_keyspace_g over the words k_keyspace_wave listed (grid = gslots)
hipError_t a5x_launch_keyspace_g(const A5xKsLaunch& L, hipStream_t st);
int a5x_read_stamps(unsigned long long* out16, int reset);
hipError_t a5x_launch_keyspace(const A5xKsLaunch& L, hipStream_t st);
size_t a5x_keyspace_wave_lds(uint32_t table_bytes);
size_t a5x_keyspace_thread_lds(uint32_t table_bytes);
size_t a5x_keyspace_rprobe_lds(uint32_t table_bytes);
uint64_t a5x_scan_tmp_elems(uint64_t n);
hipError_t a5x_launch_scan(const uint64_t* ca, const uint64_t* cb, uint64_t n, uint64_t* outa, uint64_t* outb,
                           uint64_t* tmp, uint32_t* err, hipStream_t st);
hipError_t a5x_launch_plan(const uint64_t* cand_off, uint64_t nw, uint64_t CH, uint32_t* chunk_w0, hipStream_t st);
// (word, segment) items of the listed words' candidates in [cb, ce), CH per segment
hipError_t a5x_launch_segments(const uint32_t* list, const uint32_t* list_n, uint32_t n_bound,
                               const uint64_t* cand_off, uint64_t cb, uint64_t ce, uint64_t CH, uint64_t* segs,
                               uint32_t* nsegs, hipStream_t st);
size_t a5x_expand_lds(uint32_t table_bytes, int kind, uint32_t waves);
// kind 0: k_expand_fast, 1: k_expand_slow, 2: k_expand_b (pass B), 3: k_expand_fast_md5,
// 4: k_expand_g (pass G: the GLOB words of the BIG segment list), 5: k_expand_fast_ntlm
hipError_t a5x_launch_expand(const A5xExpLaunch& L, int kind, hipStream_t st);
hipError_t a5x_launch_locate(const A5xExpLaunch& L, const uint64_t* cands, uint32_t n, uint64_t* out_bytes,
                             hipStream_t st);
hipError_t a5x_launch_word_of(const uint64_t* cand_off, uint64_t nw, const uint64_t* g, uint32_t nt, uint64_t* word,
                              uint64_t* ciw, hipStream_t st);
hipError_t a5x_launch_digest(const uint8_t* out, const uint64_t* byte_off, uint64_t out_base, uint64_t nw,
                             uint64_t* dig, hipStream_t st);

// ---- -r / -s / -s -r engines (a5x_modes.hip) --------------------------------
struct A5xModeLaunch {
  const uint8_t* mtab;  // A5xMHdr blob (a5x_format.h)
  uint32_t mtab_bytes;
  const uint8_t* words;
  const uint64_t* woff;
  uint64_t nw;
  int mode, mn, mx;
  uint64_t SEG;          // candidates per item
  uint64_t* count;       // k_mode_count outputs: per-word count, items, flags
  uint64_t* nseg;
  uint32_t* flags;
  const uint64_t* cand_off;  // exclusive scans (n+1)
  const uint64_t* seg_off;
  const uint32_t* item_w;    // item -> word
  uint64_t nitems;
  uint64_t item_begin, item_end;
  uint64_t* seg_bytes;       // length pass output (per item)
  uint8_t* item_fl;          // per item: which layout expands it (set by the length pass)
  uint64_t* wbytes;          // per word: closed-form output bytes of single-item positional words (~0: none)
  const uint64_t* seg_boff;  // exclusive scan of seg_bytes (nitems+1)
  uint64_t cand_begin, cand_end;
  uint8_t* out;
  uint64_t out_base, out_cap;
  uint32_t* err;
  // mode pass G: words longer than A5X_M_LMAX (flag A5X_WF_GLOB), listed by k_mode_count,
  // run by one wave per HBM scratch slot (gslots x a5x_mode_gslot_bytes(); gscr null: none)
  uint32_t* glob_list;
  uint32_t* glob_n;
  uint8_t* gscr;
  uint32_t gslots;
  // -r FAST words (flags & A5X_WF_FAST, set by the k_keyspace_thread -r probe): counted
  // there, their items sized L + 1 per candidate and expanded by k_expand_fast
  int rfast;
  // -s / -s -r lane-per-word keyspace (k_mode_count_thread): the words it leaves to the
  // wave kernel k_mode_count (cl_list null: k_mode_count takes every word)
  uint32_t* cl_list;
  uint32_t* cl_n;
  const uint32_t* in_list;  // k_mode_count_thread's words (null: all; else the probe's list)
  const uint32_t* in_n;
  const uint64_t* rec;      // FAST plan records / offsets (k_mode_locate inside -s FAST words)
  const uint32_t* roff;
  // virtual words (flags & A5X_WF_VIRT; k_mode_locate): the virtual word list
  const uint64_t* vpre;
  const uint64_t* vcand_off;
  const uint64_t* vbyte_off;
  const uint32_t* vroff;
  const uint64_t* vrec;
  // fused digest (op 2): every candidate hashed where it is built and probed against the
  // target set; hits as (word, candidate in word) -- see A5xDigLaunch
  int dg_algo;
  const uint32_t* dg_bitmap;
  uint32_t dg_bm_mask, dg_has_zero, dg_hit_cap;
  const uint4* dg_table;
  uint64_t dg_tmask;
  struct A5xHitRaw* dg_hits;
  uint32_t* dg_nhits;
  uint32_t grid_cap;  // item kernels: workgroups at most (0: M_GRID_MAX); a few mode words among many
                      // FAST ones are filtered by a small grid beside k_expand_fast
};
size_t a5x_mode_lds(uint32_t mtab_bytes);
uint64_t a5x_mode_gslot_bytes();
hipError_t a5x_launch_mode_count(const A5xModeLaunch& L, hipStream_t st);
// -s / -s -r: radix positional words counted lane per word; the others listed for
// a5x_launch_mode_count (which then runs over L.cl_list)
hipError_t a5x_launch_mode_count_thread(const A5xModeLaunch& L, hipStream_t st);
hipError_t a5x_launch_mode_count_g(const A5xModeLaunch& L, hipStream_t st);
// op 0: per-item output bytes (seg_bytes); op 1: expand items [item_begin, item_end);
// op 2: fused digest of items [item_begin, item_end) (no length pass needed before it)
hipError_t a5x_launch_mode_items(const A5xModeLaunch& L, int op, hipStream_t st);
// out[3q..3q+2] = {item, index in item, byte offset} of global candidate cands[q]
hipError_t a5x_launch_mode_locate(const A5xModeLaunch& L, const uint64_t* cands, uint32_t n, uint64_t* out,
                                  hipStream_t st);
hipError_t a5x_launch_mode_wordbytes(const uint64_t* seg_off, const uint64_t* seg_boff, uint64_t nw,
                                     uint64_t* byte_off, uint64_t* bytes, hipStream_t st);

// ---- fused digest + lookup (a5x_digest.hip) ----------------------------------
struct A5xHitRaw {  // (block, ordinal) until k_hits_resolve, then (word, candidate in word)
  uint64_t blk;
  uint64_t idx;
  uint32_t d[4];
};
struct A5xDigLaunch {
  const uint8_t* out;  // "cand\n" stream, 16-B aligned, starts at a candidate
  uint64_t nbytes;
  int algo;            // A5X_ALGO_MD5 / A5X_ALGO_NTLM
  const uint32_t* bitmap;
  uint32_t bm_mask;    // prefilter index mask: 2^k - 1 for a 2^k-bit bitmap (k <= 32)
  const uint4* table;  // open addressing, all-zero = empty
  uint64_t tmask;
  uint32_t has_zero_target;
  A5xHitRaw* hits;
  uint32_t* nhits;
  uint32_t hit_cap;
  uint64_t* blk_cnt;        // op 1 output (per 2 KiB block line starts)
  const uint64_t* blk_pre;  // op 2 / resolve input (exclusive scan of blk_cnt)
  uint8_t* dig_out;         // op 2 output: 16 B per candidate
  uint32_t* err;
};
size_t a5x_digest_lds(int algo);
uint64_t a5x_digest_blocks(uint64_t nbytes, int algo);  // 4 KiB (MD5) / 2 KiB (NTLM) blocks
hipError_t a5x_launch_digest_stream(const A5xDigLaunch& L, int op, uint32_t grid, hipStream_t st);
// hybrid fused digest: list the candidate-bearing non-FAST words (n: device counter),
// then gather them into a sub-batch (lens != null: their lengths; else the bytes at sub_off)
hipError_t a5x_launch_nonfast_list(const uint32_t* flags, const uint64_t* cand_off, uint64_t nw, uint64_t cb,
                                   uint64_t ce, uint32_t* list, uint32_t* n, hipStream_t st);
hipError_t a5x_launch_gather_words(const uint8_t* words, const uint64_t* woff, const uint32_t* idx, uint32_t m,
                                   uint64_t* lens, const uint64_t* sub_off, uint8_t* out, hipStream_t st);
hipError_t a5x_launch_hits_resolve(A5xHitRaw* hits, uint32_t n, const uint64_t* blk_pre, uint64_t cand_base,
                                   const uint64_t* cand_off, uint64_t nw, hipStream_t st);
