// a5x_format.h -- layouts shared by the host compiler of substitution tables
// (a5x_host.cpp) and the HIP kernels (a5x_kernels.hip).
//
// The merged Go map[string][]string of main.go:40-50 is compiled into one flat
// "device table" blob that every workgroup copies into LDS once:
//
//   A5xTableHdr                                   (80 B: static_assert below; the
//                                                 lead_only flag + reserved[3] grew it
//                                                 from 64 B, so A5X_TABLE_LDS_MAX holds
//                                                 16 B less of keys / choices / blob)
//   u16 bucket[257]  keys whose first byte is b are [bucket[b], bucket[b+1])
//   A5xKey  keys[nkeys]                           (32 B each, 16-B aligned)
//   A5xChoice choices[nchoices]                   (8 B each)
//   u8 blob[blob_bytes]                           (key + value bytes, 8-B padded)
//
// Choice 0 of key k (choices[k.choice_base]) is the key itself (the "keep"
// branch); choice 1+v is value v in (-t file, line) order (main.go:141, 48).
#pragma once
#include <stdint.h>

#define A5X_TABLE_MAGIC 0x58354131u  // "1A5X"

struct A5xTableHdr {
  uint32_t magic;
  uint32_t total_bytes;   // whole blob, multiple of 16
  uint32_t nkeys;         // keys with length >= 1 (an empty key never matches in
                          // processWord / processWordReverse: keyLength >= 1)
  uint32_t nchoices;
  uint32_t off_bucket;    // byte offsets inside the blob
  uint32_t off_keys;
  uint32_t off_choices;
  uint32_t off_blob;
  uint32_t blob_bytes;
  uint32_t max_klen;
  uint32_t max_vlen;
  uint32_t has_empty_key; // the map has "" (matters for -s only, main.go:315)
  uint32_t max_bucket;    // most keys sharing a first byte
  uint32_t off_kmatch;    // u64 kmatch[max(nkeys, 1)]: key k's first min(klen, 4) bytes | klen << 32
  uint32_t off_bucket2;   // u32 bucket2[256]: bucket[b] | bucket[b + 1] << 16 (one read per byte)
  uint32_t off_cval;      // u64 cval[nchoices]: choice's first min(len, 7) bytes | min(len, 255) << 56
  uint32_t lead_only;     // no key starts with a UTF-8 continuation byte (0x80-0xBF): the keyspace
                          // walk steps over them (k_keyspace_thread psk_walk)
  uint32_t reserved[3];
};

struct A5xKey {
  uint16_t klen;
  uint16_t nvals;
  uint32_t choice_base;   // choices[choice_base] = key, [choice_base+1+v] = value v
  uint32_t sumlen;        // sum of value lengths (byte DP)
  int16_t maxdelta;       // max(|v|) - klen
  uint16_t maxclen;       // max(klen, max |v|): longest choice
  uint16_t minclen;       // min(klen, min |v|): shortest choice
  uint16_t pad0;
  uint32_t pad1;
  uint32_t sum_dpos;      // sum over values of max(|v| - klen, 0)
  uint32_t sum_dneg;      // sum over values of max(klen - |v|, 0)
};

struct A5xChoice {
  uint32_t first4;        // first min(len,4) bytes, little-endian, zero padded
  uint16_t len;
  uint16_t blob_off;      // offset in blob (valid for any len)
};

static_assert(sizeof(A5xTableHdr) == 80, "hdr");
static_assert(sizeof(A5xKey) == 32, "key");
static_assert(sizeof(A5xChoice) == 8, "choice");

// Per-word class flags written by the keyspace pass (u32 per word).
enum : uint32_t {
  A5X_WF_RADIX = 1u << 0,   // disjoint single matches, free count window: mixed radix
  A5X_WF_BIN = 1u << 1,     // ... and every slot has exactly one value (radix 2)
  A5X_WF_GENERAL = 1u << 2, // overlapping / multi matches or capped: DP walk
  A5X_WF_BIG = 1u << 3,     // does not fit the pass-A wave budget: pass B
  A5X_WF_DEFER = 1u << 4,   // keyspace needs the wave-level DP kernel
  A5X_WF_FAST = 1u << 5,    // radix, <= 64 B, piece plan fits (plan_word): k_expand_fast
  A5X_WF_GLOB = 1u << 6,    // (with BIG) beyond the pass-B LDS budget: pass G, global scratch
  A5X_WF_VIRT = 1u << 7,    // (with FAST) -s / -s -r word split into FAST sub-words (k_keyspace_vsub)
  A5X_WF_ERR_OVF = 1u << 8, // count/bytes overflow u64
  A5X_WF_ERR_BIG = 1u << 9, // exceeds pass-B limits
};

// FAST words: bits 10..14 = group pieces, 16..23 = piece entries, 24..28 = pieces
// (plan_word in a5x_kernels.hip).  Virtual words: bit 29 = A5X_WF_VFIX (below).
enum : uint32_t {
  A5X_WF_VFIX = 1u << 29,  // (with VIRT) fixed-width word: k_keyspace_vsub left a descriptor, k_vwords_fill writes
                           // its sub-words' records
};

// Limits of the expansion passes (documented in DESIGN.md).
#define A5X_WAVE 64
#define A5X_LMAX_A 64          // pass A: word bytes (one lane per position)
#define A5X_DPENT_A 256        // pass A: DP table entries (G and H each), (events+1) x W
#define A5X_MLMAX_A 128        // pass A: total key matches in a word
#define A5X_RING_A 4096        // pass A: staging ring bytes per wave
#define A5X_LMAX_B 2048        // pass B (one wave per workgroup)
#define A5X_DPENT_B 4096
#define A5X_MLMAX_B 4096
#define A5X_RING_B 16384
// pass G: one wave per scratch slot in HBM (WaveLds + ring), for words beyond pass B --
// any line the reference reads (bufio.Scanner stops at 64 KiB lines, main.go:72-74)
#define A5X_LMAX_G 65535
#define A5X_MLMAX_G 65536
#define A5X_DPENT_G (1u << 20)
#define A5X_RING_G (1u << 20)
#define A5X_G_SLOTS 16
#define A5X_CMAX 63            // max DP columns-1 (count window)
#define A5X_TABLE_LDS_MAX 32768

// ---------------------------------------------------------------------------
// "Mode table" for the -r / -s / -s -r engines (main.go:208-440), staged into LDS
// by a5x_modes.hip.  Keys are sorted bytewise (Go sort.Strings, main.go:327), so
//   * the sorted pattern list of a word = the set bits of a key bitmap in index
//     order (processWordSubstituteAll, main.go:310-327);
//   * keys sharing a first byte are contiguous, and the keys matching at one
//     word position come out in increasing length (they are all prefixes of the
//     same suffix), i.e. in the j-loop order of validSubstitutionPositions
//     (main.go:288-293);
//   * an empty key (matched by -s at every position, main.go:315) is key 0.
//
//   A5xMHdr (64 B) | u16 bucket[257] (non-empty keys with first byte b:
//   [bucket[b], bucket[b+1])) | A5xMKey keys[nkeys] | A5xMVal vals[nvals] | blob
// ---------------------------------------------------------------------------
#define A5X_MTAB_MAGIC 0x4D354131u  // "1A5M"
#define A5X_MTAB_LDS_MAX 32768     // staging limit (bytes; + the 26 KB work area < 64 KB)
#define A5X_MTAB_KEYS_MAX 4096     // key bitmap of 128 dwords

struct A5xMHdr {
  uint32_t magic;
  uint32_t total_bytes;  // multiple of 16
  uint32_t nkeys;
  uint32_t nvals;
  uint32_t off_bucket;
  uint32_t off_keys;
  uint32_t off_vals;
  uint32_t off_blob;
  uint32_t has_empty;    // key 0 is ""
  uint32_t pad[7];
};

struct A5xMKey {
  uint32_t key_off;   // blob offset of the key bytes
  uint16_t klen;
  uint16_t nvals;     // values in (-t file, line) order (main.go:141, 48)
  uint32_t val_base;  // vals[val_base + v] = value v
  uint32_t pad;
};

struct A5xMVal {
  uint32_t off;  // blob offset
  uint32_t len;
};

static_assert(sizeof(A5xMHdr) == 64, "mhdr");
static_assert(sizeof(A5xMKey) == 16, "mkey");
static_assert(sizeof(A5xMVal) == 8, "mval");

// Limits of the -r / -s / -s -r device engines (a5x_modes.hip).
#define A5X_M_LMAX 128    // word bytes
#define A5X_M_CBUF 128    // candidate buffer per lane: candidates <= 127 bytes
#define A5X_M_NMAX 63     // sorted patterns (-s) or match positions (-r) per word
#define A5X_M_DPMAX 1024  // DP entries (patterns/positions + 1) x (count window + 1)
// mode pass G (HBM scratch slots, a5x_modes.hip): words longer than A5X_M_LMAX, up to a
// ScanLines line (main.go:72-74), with candidates of up to A5X_MG_CBUF - 1 bytes
#define A5X_MG_LMAX 65535
#define A5X_MG_CBUF (1u << 17)
