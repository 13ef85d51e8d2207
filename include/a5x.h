/*
 * a5x.h -- C ABI of liba5x.so, the MI355X (gfx950) backend for hashcat -a 5
 * table-attack candidate expansion.
 *
 * Drop-in boundary: the reference calls one of four
 * engines per word from a goroutine,
 *     func processWord(word string, subMap map[string][]string,
 *                      minSubstitute, maxSubstitute int, out chan<- string)
 *     /root/reference/main.go:168   (also :208 -r, :308 -s, :369 -s -r;
 *                                     dispatcher main.go:77-93)
 * and sends every candidate on a channel that one writer drains as s+"\n"
 * (main.go:58-68).  liba5x replaces that per-word call with a batch call:
 * contiguous word bytes + offsets in, "cand\n" bytes out, grouped per word.
 *
 * Conventions: every function returns 0 (A5X_OK) or a negative A5X_E_* code and
 * records a message readable with a5x_last_error().  Inputs are caller-owned and
 * copied/staged; output spans handed to a sink are library-owned and valid only
 * during the callback.  One in-flight call per context (thread-compatible).
 * Go pointers must not be retained across calls (cgo rules): the library never
 * keeps a caller pointer after returning.
 *
 * mode: A5X_MODE_DEFAULT (processWord, main.go:168), A5X_MODE_REVERSE (-r,
 * main.go:208), A5X_MODE_SUBALL (-s, main.go:308), A5X_MODE_SUBALL_REVERSE
 * (-s -r, main.go:369) -- the switch of main.go:80-92.  min/max are passed raw
 * (--table-min/--table-max, main.go:21-22); the library applies processWord's
 * min==0 -> 1 bump itself (main.go:169-171).
 */
#ifndef A5X_H
#define A5X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define A5X_API __attribute__((visibility("default")))

#define A5X_ABI_VERSION 1

enum {
  A5X_OK = 0,
  A5X_E_ARG = -1,         /* bad argument */
  A5X_E_HIP = -2,         /* HIP runtime error (no device, launch failure, ...) */
  A5X_E_NOMEM = -3,       /* host or device allocation failed */
  A5X_E_IO = -4,          /* table / dictionary file could not be read (main.go:43-45, 53-55) */
  A5X_E_TOOLONG = -5,     /* bufio.ErrTooLong on a table line (main.go:143 -> log.Fatal) */
  A5X_E_BOUNDS = -6,      /* -r slice-bounds panic of the reference (main.go:255) */
  A5X_E_OVERFLOW = -7,    /* a keyspace does not fit 64 bits */
  A5X_E_CAPACITY = -8,    /* caller's output buffer too small (device API) */
  A5X_E_UNSUPPORTED = -9, /* mode/word beyond this build's device limits */
  A5X_E_NOTABLE = -10,    /* no substitution table loaded */
  A5X_E_SINK = -11        /* the sink callback returned non-zero */
};

enum {
  A5X_MODE_DEFAULT = 0,
  A5X_MODE_REVERSE = 1,
  A5X_MODE_SUBALL = 2,
  A5X_MODE_SUBALL_REVERSE = 3
};

/* digest algorithms of the fused digest + lookup stage */
enum {
  A5X_ALGO_MD5 = 0,  /* RFC 1321 over the candidate bytes (== Go crypto/md5) */
  A5X_ALGO_NTLM = 1  /* MD4 (RFC 1320) over UTF-16LE of the candidate ([]rune + utf16.Encode) */
};

/* One target hit: word index in the batch, candidate index inside that word (in the
 * library's per-word candidate order, the one a5x_expand emits), digest bytes. */
typedef struct a5x_hit {
  uint64_t word;
  uint64_t cand;
  uint8_t digest[16];
} a5x_hit;

typedef struct a5x_ctx a5x_ctx;

/* Sink for expanded bytes: a run of complete "cand\n" lines.  Return 0 to go on. */
typedef int (*a5x_sink_fn)(void* user, const uint8_t* data, size_t len);

typedef struct a5x_stats {
  uint64_t candidates;  /* candidates produced by the call */
  uint64_t bytes;       /* bytes produced (sum of len(cand)+1) */
  uint64_t words;       /* words in the batch */
  uint64_t words_pass_b;/* words expanded by the large-LDS pass */
  double ms_keyspace;   /* device time: keyspace + scans + plan (HIP events) */
  double ms_expand;     /* device time: expansion kernels only (HIP events) */
  double ms_total;      /* device time of the whole call */
  uint32_t expand_launches;
  uint32_t words_slow;   /* words expanded by the per-word (non-FAST) pass */
} a5x_stats;

/* ---- context ------------------------------------------------------------ */
A5X_API int a5x_abi_version(void);
/* device = -1: host-only context (table parsing/export, no GPU; device calls fail). */
A5X_API int a5x_create(int device, a5x_ctx** out);
A5X_API void a5x_destroy(a5x_ctx* ctx);
A5X_API const char* a5x_last_error(const a5x_ctx* ctx);
/* Why the calling thread's last a5x_create failed ("" after a success): the failing HIP
   call with hipGetErrorString, or the argument problem (no context exists to carry it). */
A5X_API const char* a5x_create_error(void);
/* device name / gfx arch of the context's GPU */
A5X_API int a5x_device_info(a5x_ctx* ctx, char* name, size_t name_cap, int* cu_count);

/* ---- substitution tables (main.go:40-50, 102-162) ------------------------ */
/* readSubstitutionTable(path) + merge into the context's map in call order. */
A5X_API int a5x_load_table_file(a5x_ctx* ctx, const char* path);
/* Same for in-memory file contents. */
A5X_API int a5x_parse_table(a5x_ctx* ctx, const uint8_t* data, size_t len);
/* Replace the map with an already-merged one:
 * key i = keys_bytes[key_off[i] .. key_off[i+1]); value j = vals_bytes[val_off[j]
 * .. val_off[j+1]) belongs to key val_key[j]; values keep their array order per key. */
A5X_API int a5x_set_table(a5x_ctx* ctx, const uint8_t* keys_bytes, const uint64_t* key_off, uint32_t n_keys,
                          const uint8_t* vals_bytes, const uint64_t* val_off, const uint32_t* val_key,
                          uint32_t n_vals);
A5X_API int a5x_clear_table(a5x_ctx* ctx);
/* Export the merged map: sizes first (any out pointer may be NULL). */
A5X_API int a5x_table_export(const a5x_ctx* ctx, uint32_t* n_keys, uint32_t* n_vals, uint64_t* key_bytes,
                             uint64_t* val_bytes, uint8_t* keys_out, uint64_t* key_off_out, uint8_t* vals_out,
                             uint64_t* val_off_out, uint32_t* val_key_out);

/* ---- dictionary splitting (bufio.Scanner + ScanLines, main.go:72-74) ------- */
/* Splits data into words exactly as the reference's dict scanner: "\n" split,
 * one trailing "\r" dropped, a line >= 64 KiB silently ends the input.  words_out
 * receives the concatenated word bytes (<= len bytes), off_out n+1 offsets.
 * With words_out == NULL only *n_words is computed. */
A5X_API int a5x_split_words(const uint8_t* data, size_t len, uint8_t* words_out, uint64_t* off_out,
                            uint64_t off_cap, uint64_t* n_words);

/* ---- host-buffer API -------------------------------------------------------- */
/* Per-word candidate count and output bytes (len+1 per candidate). */
A5X_API int a5x_keyspace(a5x_ctx* ctx, const uint8_t* words, const uint64_t* word_off, uint64_t n_words, int mode,
                         int min, int max, uint64_t* out_count, uint64_t* out_bytes);
/* Expand and stream "cand\n" lines to sink, words in order; a word's candidates are
 * contiguous.  Replaces the goroutine-per-word dispatch + channel of main.go:70-98. */
A5X_API int a5x_expand(a5x_ctx* ctx, const uint8_t* words, const uint64_t* word_off, uint64_t n_words, int mode,
                       int min, int max, a5x_sink_fn sink, void* user, a5x_stats* stats);
/* a5x_expand of the batch's global candidates [cand_begin, cand_end) only (cand_end =
 * UINT64_MAX: to the end): a resume cursor over the stream (CLI --skip / --limit, the
 * role of hashcat's own -s / -l on the pipe the reference feeds, README.MD:69).  A
 * word's candidate order does not depend on the batch it is in, so (batch offset +
 * index) names one candidate of the dictionary's stream.  stats->candidates / bytes
 * count the window. */
A5X_API int a5x_expand_range(a5x_ctx* ctx, const uint8_t* words, const uint64_t* word_off, uint64_t n_words,
                             int mode, int min, int max, uint64_t cand_begin, uint64_t cand_end, a5x_sink_fn sink,
                             void* user, a5x_stats* stats);

/* Make a5x_expand's buffers ahead of the first call (pinned double buffer, HBM range
 * buffers, copy stream, the keyspace state of a batch of `words` words / `word_bytes`
 * bytes, the table upload), so a pipeline's first batch does not pay for them; a host may
 * call it on a second thread while it reads its first batch.  Optional. */
A5X_API int a5x_stream_reserve(a5x_ctx* ctx, uint64_t words, uint64_t word_bytes);

/* ---- device-resident API (words already in HBM; used by bench and multi-GPU) -- */
/* Expands global candidates [cand_begin, cand_end) of the batch (cand_end =
 * UINT64_MAX: to the end) into d_out (d_out[0] = first byte of cand_begin).
 * d_word_byte_off (n_words+1, optional) receives each word's byte offset in the
 * batch's full output; d_word_cand_off likewise for candidate offsets.
 * stream: a hipStream_t (NULL = the context's stream).  Synchronises once to
 * read the totals; returns A5X_E_CAPACITY (with stats->bytes = need) if the
 * range does not fit out_cap. */
A5X_API int a5x_expand_device(a5x_ctx* ctx, const uint8_t* d_words, const uint64_t* d_word_off, uint64_t n_words,
                              int mode, int min, int max, uint64_t cand_begin, uint64_t cand_end, uint8_t* d_out,
                              uint64_t out_cap, uint64_t* d_word_cand_off, uint64_t* d_word_byte_off,
                              a5x_stats* stats, void* stream);
/* Keyspace of device-resident words: totals only (and per-word offsets if given). */
A5X_API int a5x_keyspace_device(a5x_ctx* ctx, const uint8_t* d_words, const uint64_t* d_word_off, uint64_t n_words,
                                int mode, int min, int max, uint64_t* d_word_cand_off, uint64_t* d_word_byte_off,
                                uint64_t* total_cands, uint64_t* total_bytes, void* stream);
/* Order-independent per-word digest of an expanded batch (verification):
 * d_digest[4*w..] = {count, bytes, sum h, sum h^2}, h = fmix64(fnv1a64(cand)). */
A5X_API int a5x_digest_device(a5x_ctx* ctx, const uint8_t* d_out, const uint64_t* d_word_byte_off, uint64_t out_base,
                              uint64_t n_words, uint64_t* d_digest, void* stream);

/* ---- fused digest + lookup (no reference counterpart: hashcat
 * hashes the candidates main.go:66 prints, README.MD:69) ----------------------- */
/* Replace the device-resident target set: n 16-byte digests of algorithm algo
 * (duplicates allowed).  Built on the host (prefilter bitmap + open-addressing table)
 * and uploaded once. */
A5X_API int a5x_set_targets(a5x_ctx* ctx, int algo, const uint8_t* digests, uint64_t n);
/* Expand the batch (device-resident words) in ranges that fit a device scratch of
 * scratch_bytes (0 = library default), hash every candidate on the device and probe the
 * target set.  Hits go to hits (host memory, hit_cap entries, any order); *n_hits gets
 * the total (which may exceed hit_cap: A5X_E_CAPACITY after filling hit_cap).
 * stats->candidates/bytes cover the whole batch; ms_expand is expansion time,
 * ms_total - ms_keyspace - ms_expand the digest time. */
A5X_API int a5x_expand_digest_device(a5x_ctx* ctx, const uint8_t* d_words, const uint64_t* d_word_off,
                                     uint64_t n_words, int mode, int min, int max, uint64_t scratch_bytes,
                                     a5x_hit* hits, uint64_t hit_cap, uint64_t* n_hits, a5x_stats* stats,
                                     void* stream);
/* The same for the batch's global candidates [cand_begin, cand_end) only (clipped to the
 * batch): a shard whose ends cut words (a5x_split_device gives the cut
 * points), as a5x_expand_device's range.  Hits name (word, candidate in word) of the
 * batch; stats->candidates counts the range. */
A5X_API int a5x_expand_digest_range_device(a5x_ctx* ctx, const uint8_t* d_words, const uint64_t* d_word_off,
                                           uint64_t n_words, int mode, int min, int max, uint64_t cand_begin,
                                           uint64_t cand_end, uint64_t scratch_bytes, a5x_hit* hits,
                                           uint64_t hit_cap, uint64_t* n_hits, a5x_stats* stats, void* stream);
/* Host-buffer version (stages the words into HBM first). */
A5X_API int a5x_expand_digest(a5x_ctx* ctx, const uint8_t* words, const uint64_t* word_off, uint64_t n_words,
                              int mode, int min, int max, a5x_hit* hits, uint64_t hit_cap, uint64_t* n_hits,
                              a5x_stats* stats);
/* Digest of every line of a device "cand\n" stream (d_lines 16-B aligned, nbytes
 * ending in '\n') into d_digests (16 B per line, in line order); *n_lines = lines.
 * Verification hook for the digest kernels (tests compare with hashlib / RFC MD4). */
A5X_API int a5x_digest_lines_device(a5x_ctx* ctx, int algo, const uint8_t* d_lines, uint64_t nbytes,
                                    uint8_t* d_digests, uint64_t digests_cap, uint64_t* n_lines, void* stream);

/* ---- hashcat-style hit output: "hash:plain" lines --------------- */
/* The plain as hashcat's outfile writes it: unchanged, or $HEX[lowercase hex] when it
 * is not valid UTF-8, contains a control byte (< 0x20, 0x7f) or has the $HEX[...] form
 * itself (README.MD:171-176 uses the same notation for input).  *out_len = the size;
 * out == NULL: size only; A5X_E_CAPACITY when cap is too small.  Pure host function. */
A5X_API int a5x_format_plain(const uint8_t* plain, size_t len, uint8_t* out, size_t cap, size_t* out_len);
/* One "hexdigest:plain\n" line per hit, in hit order, through sink (hashcat -m 0 /
 * -m 1000 potfile form, README.MD:74-106): the plains are regenerated on the device
 * from the hit's (word, cand) with the same batch (host buffers), mode and limits the
 * hits were found with. */
A5X_API int a5x_format_hits(a5x_ctx* ctx, const uint8_t* words, const uint64_t* word_off, uint64_t n_words,
                            int mode, int min, int max, const a5x_hit* hits, uint64_t n_hits, a5x_sink_fn sink,
                            void* user);

/* Output byte offset, in the batch's full "cand\n" stream, of each global candidate index
 * cands[i] (cands[i] = the batch's total candidates gives its total bytes; larger: clamped).
 * Device-resident words; the keyspace runs once per call.  Candidate numbering is the one
 * a5x_expand_device's [cand_begin, cand_end) uses. */
A5X_API int a5x_locate_device(a5x_ctx* ctx, const uint8_t* d_words, const uint64_t* d_word_off, uint64_t n_words,
                              int mode, int min, int max, const uint64_t* cands, uint64_t n, uint64_t* byte_off_out,
                              void* stream);
/* Candidate-granular split points for byte targets (a word larger than
 * a rank's share is cut inside, where the reference serialises it on one goroutine,
 * main.go:77-93): for each byte_targets[i] (<= the batch's total bytes), cand_out[i] =
 * the first global candidate whose first output byte is >= the target (the total
 * candidates when none), word_out[i] = the word holding it (n_words when none) and
 * cand_in_word_out[i] = its index inside that word.  Exact (binary search over
 * a5x_locate_device's offsets); the keyspace runs once per call. */
A5X_API int a5x_split_device(a5x_ctx* ctx, const uint8_t* d_words, const uint64_t* d_word_off, uint64_t n_words,
                             int mode, int min, int max, const uint64_t* byte_targets, uint32_t n_targets,
                             uint64_t* cand_out, uint64_t* word_out, uint64_t* cand_in_word_out, void* stream);

/* ---- multi-GPU partition --------------------------------------- */
/* Balanced split of [0, total) for `parts` ranks from an inclusive/exclusive
 * prefix (n+1 entries, e.g. per-word byte offsets): split[r] = first word of
 * rank r, split[parts] = n.  Pure host function. */
A5X_API int a5x_partition(const uint64_t* prefix, uint64_t n, uint32_t parts, uint64_t* split);

/* Diagnostic builds only (compiled with -DA5X_STAMPS): per-phase cycle sums of
 * the fast expansion kernel.  A5X_E_UNSUPPORTED in shipped builds. */
A5X_API int a5x_debug_stamps(unsigned long long* out16, int reset);

/* Test hook (CPU test suite): run the device keyspace classification and the FAST
 * piece plan of ONE word on the host (the same a5x_plan.h code the kernels run)
 * and, for FAST words, replay passes 1-2 of k_expand_fast into out.  info[0..3] =
 * {count, bytes, flags | big pieces << 32 | big entries << 40, bytes written};
 * out = NULL: classification and plan only.  Never called by a5x_expand*: it checks the
 * plan, it is not a compute path. */
A5X_API int a5x_debug_plan_word(a5x_ctx* ctx, const uint8_t* word, size_t len, int min_sub, int max_sub,
                                uint8_t* out, size_t cap, uint64_t* info);

/* ---- device memory helpers (so hosts without torch can drive the API) ---------- */
A5X_API int a5x_dev_alloc(a5x_ctx* ctx, void** p, size_t bytes);
A5X_API int a5x_dev_free(a5x_ctx* ctx, void* p);
A5X_API int a5x_memcpy_h2d(a5x_ctx* ctx, void* dst, const void* src, size_t bytes);
A5X_API int a5x_memcpy_d2h(a5x_ctx* ctx, void* dst, const void* src, size_t bytes);
A5X_API int a5x_synchronize(a5x_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif /* A5X_H */
