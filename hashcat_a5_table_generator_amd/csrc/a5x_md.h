// a5x_md.h -- MD5 (RFC 1321) / MD4 (RFC 1320) compression, LDS message loads and the
// target-set probe (device only; shared by the two-pass digest stream, a5x_digest.hip,
// and the fused digest of k_expand_fast, a5x_kernels.hip).
#pragma once
#include <stdint.h>

__device__ __forceinline__ uint32_t rotl(uint32_t x, uint32_t s) { return __builtin_amdgcn_alignbit(x, x, 32u - s); }

// ---------------------------------------------------------------------------
// MD5 (RFC 1321) and MD4 (RFC 1320) compression functions
// ---------------------------------------------------------------------------
#define MD5_STEP(f, a, b, c, d, x, t, s) \
  a += f(b, c, d) + (x) + (t);           \
  a = rotl(a, s) + b;
#define MD5_F(x, y, z) (((x) & (y)) | (~(x) & (z)))
#define MD5_G(x, y, z) (((x) & (z)) | ((y) & ~(z)))
#define MD5_H(x, y, z) ((x) ^ (y) ^ (z))
#define MD5_I(x, y, z) ((y) ^ ((x) | ~(z)))

// steps 1-62: after them a and d hold their final values (digest words 0 and 3 = IV + a, d),
// so the target prefilter (md_prefilter) can reject before steps 63-64 (md_block_probe)
__device__ __forceinline__ void md5_steps62(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d, const uint32_t* M) {
  MD5_STEP(MD5_F, a, b, c, d, M[0], 0xd76aa478u, 7) MD5_STEP(MD5_F, d, a, b, c, M[1], 0xe8c7b756u, 12)
  MD5_STEP(MD5_F, c, d, a, b, M[2], 0x242070dbu, 17) MD5_STEP(MD5_F, b, c, d, a, M[3], 0xc1bdceeeu, 22)
  MD5_STEP(MD5_F, a, b, c, d, M[4], 0xf57c0fafu, 7) MD5_STEP(MD5_F, d, a, b, c, M[5], 0x4787c62au, 12)
  MD5_STEP(MD5_F, c, d, a, b, M[6], 0xa8304613u, 17) MD5_STEP(MD5_F, b, c, d, a, M[7], 0xfd469501u, 22)
  MD5_STEP(MD5_F, a, b, c, d, M[8], 0x698098d8u, 7) MD5_STEP(MD5_F, d, a, b, c, M[9], 0x8b44f7afu, 12)
  MD5_STEP(MD5_F, c, d, a, b, M[10], 0xffff5bb1u, 17) MD5_STEP(MD5_F, b, c, d, a, M[11], 0x895cd7beu, 22)
  MD5_STEP(MD5_F, a, b, c, d, M[12], 0x6b901122u, 7) MD5_STEP(MD5_F, d, a, b, c, M[13], 0xfd987193u, 12)
  MD5_STEP(MD5_F, c, d, a, b, M[14], 0xa679438eu, 17) MD5_STEP(MD5_F, b, c, d, a, M[15], 0x49b40821u, 22)
  MD5_STEP(MD5_G, a, b, c, d, M[1], 0xf61e2562u, 5) MD5_STEP(MD5_G, d, a, b, c, M[6], 0xc040b340u, 9)
  MD5_STEP(MD5_G, c, d, a, b, M[11], 0x265e5a51u, 14) MD5_STEP(MD5_G, b, c, d, a, M[0], 0xe9b6c7aau, 20)
  MD5_STEP(MD5_G, a, b, c, d, M[5], 0xd62f105du, 5) MD5_STEP(MD5_G, d, a, b, c, M[10], 0x02441453u, 9)
  MD5_STEP(MD5_G, c, d, a, b, M[15], 0xd8a1e681u, 14) MD5_STEP(MD5_G, b, c, d, a, M[4], 0xe7d3fbc8u, 20)
  MD5_STEP(MD5_G, a, b, c, d, M[9], 0x21e1cde6u, 5) MD5_STEP(MD5_G, d, a, b, c, M[14], 0xc33707d6u, 9)
  MD5_STEP(MD5_G, c, d, a, b, M[3], 0xf4d50d87u, 14) MD5_STEP(MD5_G, b, c, d, a, M[8], 0x455a14edu, 20)
  MD5_STEP(MD5_G, a, b, c, d, M[13], 0xa9e3e905u, 5) MD5_STEP(MD5_G, d, a, b, c, M[2], 0xfcefa3f8u, 9)
  MD5_STEP(MD5_G, c, d, a, b, M[7], 0x676f02d9u, 14) MD5_STEP(MD5_G, b, c, d, a, M[12], 0x8d2a4c8au, 20)
  MD5_STEP(MD5_H, a, b, c, d, M[5], 0xfffa3942u, 4) MD5_STEP(MD5_H, d, a, b, c, M[8], 0x8771f681u, 11)
  MD5_STEP(MD5_H, c, d, a, b, M[11], 0x6d9d6122u, 16) MD5_STEP(MD5_H, b, c, d, a, M[14], 0xfde5380cu, 23)
  MD5_STEP(MD5_H, a, b, c, d, M[1], 0xa4beea44u, 4) MD5_STEP(MD5_H, d, a, b, c, M[4], 0x4bdecfa9u, 11)
  MD5_STEP(MD5_H, c, d, a, b, M[7], 0xf6bb4b60u, 16) MD5_STEP(MD5_H, b, c, d, a, M[10], 0xbebfbc70u, 23)
  MD5_STEP(MD5_H, a, b, c, d, M[13], 0x289b7ec6u, 4) MD5_STEP(MD5_H, d, a, b, c, M[0], 0xeaa127fau, 11)
  MD5_STEP(MD5_H, c, d, a, b, M[3], 0xd4ef3085u, 16) MD5_STEP(MD5_H, b, c, d, a, M[6], 0x04881d05u, 23)
  MD5_STEP(MD5_H, a, b, c, d, M[9], 0xd9d4d039u, 4) MD5_STEP(MD5_H, d, a, b, c, M[12], 0xe6db99e5u, 11)
  MD5_STEP(MD5_H, c, d, a, b, M[15], 0x1fa27cf8u, 16) MD5_STEP(MD5_H, b, c, d, a, M[2], 0xc4ac5665u, 23)
  MD5_STEP(MD5_I, a, b, c, d, M[0], 0xf4292244u, 6) MD5_STEP(MD5_I, d, a, b, c, M[7], 0x432aff97u, 10)
  MD5_STEP(MD5_I, c, d, a, b, M[14], 0xab9423a7u, 15) MD5_STEP(MD5_I, b, c, d, a, M[5], 0xfc93a039u, 21)
  MD5_STEP(MD5_I, a, b, c, d, M[12], 0x655b59c3u, 6) MD5_STEP(MD5_I, d, a, b, c, M[3], 0x8f0ccc92u, 10)
  MD5_STEP(MD5_I, c, d, a, b, M[10], 0xffeff47du, 15) MD5_STEP(MD5_I, b, c, d, a, M[1], 0x85845dd1u, 21)
  MD5_STEP(MD5_I, a, b, c, d, M[8], 0x6fa87e4fu, 6) MD5_STEP(MD5_I, d, a, b, c, M[15], 0xfe2ce6e0u, 10)
  MD5_STEP(MD5_I, c, d, a, b, M[6], 0xa3014314u, 15) MD5_STEP(MD5_I, b, c, d, a, M[13], 0x4e0811a1u, 21)
  MD5_STEP(MD5_I, a, b, c, d, M[4], 0xf7537e82u, 6) MD5_STEP(MD5_I, d, a, b, c, M[11], 0xbd3af235u, 10)
}
__device__ __forceinline__ void md5_steps63_64(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d, const uint32_t* M) {
  MD5_STEP(MD5_I, c, d, a, b, M[2], 0x2ad7d2bbu, 15) MD5_STEP(MD5_I, b, c, d, a, M[9], 0xeb86d391u, 21)
}
__device__ __forceinline__ void md5_block(uint32_t* st, const uint32_t* M) {
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3];
  md5_steps62(a, b, c, d, M);
  md5_steps63_64(a, b, c, d, M);
  st[0] += a; st[1] += b; st[2] += c; st[3] += d;
}

#define MD4_F(x, y, z) (((x) & (y)) | (~(x) & (z)))
#define MD4_G(x, y, z) (((x) & (y)) | ((x) & (z)) | ((y) & (z)))
#define MD4_H(x, y, z) ((x) ^ (y) ^ (z))
#define MD4_R1(a, b, c, d, k, s) a = rotl(a + MD4_F(b, c, d) + M[k], s);
#define MD4_R2(a, b, c, d, k, s) a = rotl(a + MD4_G(b, c, d) + M[k] + 0x5a827999u, s);
#define MD4_R3(a, b, c, d, k, s) a = rotl(a + MD4_H(b, c, d) + M[k] + 0x6ed9eba1u, s);

// steps 1-46: a and d final (digest words 0 and 3), as md5_steps62
__device__ __forceinline__ void md4_steps46(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d, const uint32_t* M) {
  MD4_R1(a, b, c, d, 0, 3) MD4_R1(d, a, b, c, 1, 7) MD4_R1(c, d, a, b, 2, 11) MD4_R1(b, c, d, a, 3, 19)
  MD4_R1(a, b, c, d, 4, 3) MD4_R1(d, a, b, c, 5, 7) MD4_R1(c, d, a, b, 6, 11) MD4_R1(b, c, d, a, 7, 19)
  MD4_R1(a, b, c, d, 8, 3) MD4_R1(d, a, b, c, 9, 7) MD4_R1(c, d, a, b, 10, 11) MD4_R1(b, c, d, a, 11, 19)
  MD4_R1(a, b, c, d, 12, 3) MD4_R1(d, a, b, c, 13, 7) MD4_R1(c, d, a, b, 14, 11) MD4_R1(b, c, d, a, 15, 19)
  MD4_R2(a, b, c, d, 0, 3) MD4_R2(d, a, b, c, 4, 5) MD4_R2(c, d, a, b, 8, 9) MD4_R2(b, c, d, a, 12, 13)
  MD4_R2(a, b, c, d, 1, 3) MD4_R2(d, a, b, c, 5, 5) MD4_R2(c, d, a, b, 9, 9) MD4_R2(b, c, d, a, 13, 13)
  MD4_R2(a, b, c, d, 2, 3) MD4_R2(d, a, b, c, 6, 5) MD4_R2(c, d, a, b, 10, 9) MD4_R2(b, c, d, a, 14, 13)
  MD4_R2(a, b, c, d, 3, 3) MD4_R2(d, a, b, c, 7, 5) MD4_R2(c, d, a, b, 11, 9) MD4_R2(b, c, d, a, 15, 13)
  MD4_R3(a, b, c, d, 0, 3) MD4_R3(d, a, b, c, 8, 9) MD4_R3(c, d, a, b, 4, 11) MD4_R3(b, c, d, a, 12, 15)
  MD4_R3(a, b, c, d, 2, 3) MD4_R3(d, a, b, c, 10, 9) MD4_R3(c, d, a, b, 6, 11) MD4_R3(b, c, d, a, 14, 15)
  MD4_R3(a, b, c, d, 1, 3) MD4_R3(d, a, b, c, 9, 9) MD4_R3(c, d, a, b, 5, 11) MD4_R3(b, c, d, a, 13, 15)
  MD4_R3(a, b, c, d, 3, 3) MD4_R3(d, a, b, c, 11, 9)
}
__device__ __forceinline__ void md4_steps47_48(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d, const uint32_t* M) {
  MD4_R3(c, d, a, b, 7, 11) MD4_R3(b, c, d, a, 15, 15)
}
__device__ __forceinline__ void md4_block(uint32_t* st, const uint32_t* M) {
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3];
  md4_steps46(a, b, c, d, M);
  md4_steps47_48(a, b, c, d, M);
  st[0] += a; st[1] += b; st[2] += c; st[3] += d;
}

// 4 message bytes at byte offset off of an LDS buffer (two aligned reads + funnel shift)
__device__ __forceinline__ uint32_t lds4(const uint8_t* base, uint32_t off) {
  const uint32_t* p = (const uint32_t*)(base + (off & ~3u));
  return __builtin_amdgcn_alignbyte(p[1], p[0], off & 3u);
}

// Target set: a 2^k-bit prefilter, then an open-addressing table of 16-B digests
// (all-zero slot = empty; the all-zero digest is a flag).  The prefilter is a blocked
// Bloom filter: digest word 0 picks a 64-bit word, word 3 two bits in it (one load, both
// bits tested): at 64 bits per target a false positive is ~1/1000 instead of 1/64, so a
// wave of 64 candidates reaches the table probe in ~6 % of its rounds instead of ~63 %
// (MD_BLOOM2=0: one bit, the round-4 filter; the host builds the same layout).  Words 0
// and 3 are final two MD5 steps (MD4: two steps) before the end of the last block, so a
// wave whose candidates all miss the filter skips those steps (md_block_probe).
#ifndef MD_BLOOM2
#define MD_BLOOM2 1
#endif
__host__ __device__ __forceinline__ uint64_t md_bloom_bits(uint32_t d3) {
  return MD_BLOOM2 ? (1ull << (d3 & 63u)) | (1ull << ((d3 >> 6) & 63u)) : 0ull;
}
// the prefilter alone, on digest words 0 and 3 (a possible all-zero target passes)
__device__ __forceinline__ bool md_prefilter(const uint32_t* bitmap, uint32_t bm_mask, bool has_zero, uint32_t d0,
                                             uint32_t d3) {
  if (has_zero && (d0 | d3) == 0u) return true;
  const uint32_t bi = d0 & bm_mask;
  if (MD_BLOOM2) {
    const uint64_t m = md_bloom_bits(d3);
    return (((const uint64_t*)bitmap)[bi >> 6] & m) == m;
  }
  return (bitmap[bi >> 5] >> (bi & 31u)) & 1u;
}
__device__ __forceinline__ bool md_probe(const uint32_t* bitmap, uint32_t bm_mask, const uint4* table, uint64_t tmask,
                                         bool has_zero, const uint32_t* d) {
  if ((d[0] | d[1] | d[2] | d[3]) == 0u) return has_zero;
  if (!md_prefilter(bitmap, bm_mask, false, d[0], d[3])) return false;
  const uint64_t h = ((uint64_t)d[1] | ((uint64_t)d[2] << 32)) * 0x9E3779B97F4A7C15ull;
  uint64_t slot = (h >> 20) & tmask;
  for (uint64_t n = 0; n <= tmask; n++) {
    const uint4 e = table[slot];
    if (e.x == d[0] && e.y == d[1] && e.z == d[2] && e.w == d[3]) return true;
    if ((e.x | e.y | e.z | e.w) == 0u) return false;
    slot = (slot + 1) & tmask;
  }
  return false;
}

// One-block digest + probe with early rejection: steps 1-62 (MD4: 1-46) give digest words 0
// and 3; when no lane of the wave passes the prefilter on them the last two steps and the
// table probe are skipped (no hit is possible).  h = the digest (words 1, 2 only when the
// wave went on).  Wave-collective (the ballot): call with every lane of the wave.
template <bool MD5>
__device__ __forceinline__ bool md_block_probe(const uint32_t* M, bool on, const uint32_t* bitmap, uint32_t bm_mask,
                                               const uint4* table, uint64_t tmask, bool has_zero, uint32_t* h) {
  uint32_t a = 0x67452301u, b = 0xefcdab89u, c = 0x98badcfeu, d = 0x10325476u;
  if (MD5) md5_steps62(a, b, c, d, M); else md4_steps46(a, b, c, d, M);
  h[0] = 0x67452301u + a; h[3] = 0x10325476u + d;
  h[1] = h[2] = 0u;
  const bool pass = on && md_prefilter(bitmap, bm_mask, has_zero, h[0], h[3]);
  if (!__builtin_amdgcn_ballot_w64(pass)) return false;
  if (MD5) md5_steps63_64(a, b, c, d, M); else md4_steps47_48(a, b, c, d, M);
  h[1] = 0xefcdab89u + b; h[2] = 0x98badcfeu + c;
  return pass && md_probe(bitmap, bm_mask, table, tmask, has_zero, h);
}

// Merkle-Damgard over message bytes [off, off + len) of an LDS buffer (readable 8 bytes
// past the message): RFC 1321 / 1320 padding (0x80, zeros, 64-bit little-endian bit
// length); d = the 16-byte digest as 4 little-endian words.
template <bool MD5>
__device__ __forceinline__ void md_lds(const uint8_t* base, uint32_t off, uint32_t len, uint32_t* d) {
  d[0] = 0x67452301u; d[1] = 0xefcdab89u; d[2] = 0x98badcfeu; d[3] = 0x10325476u;
  const uint32_t nb = (len + 8u) / 64u + 1u;
  for (uint32_t blk = 0; blk < nb; blk++) {
    uint32_t M[16];
#pragma unroll
    for (uint32_t j = 0; j < 16; j++) {
      const uint32_t b = blk * 64u + 4u * j;
      const int k = (int)len - (int)b;
      const uint32_t raw = k > 0 ? lds4(base, off + b) : 0u;
      const uint32_t keep = k >= 4 ? 0xffffffffu : (k <= 0 ? 0u : ((1u << (8 * k)) - 1u));
      const uint32_t pad = (k >= 0 && k < 4) ? (0x80u << (8 * k)) : 0u;
      M[j] = (raw & keep) | pad;
    }
    if (blk == nb - 1) {
      M[14] = len << 3;
      M[15] = len >> 29;
    }
    if (MD5) md5_block(d, M); else md4_block(d, M);
  }
}

// Message byte sources for the UTF-16 walk: 4 bytes at message offset i (readable
// past the message end).
struct MdLds {  // LDS buffer, readable 4 bytes past the message
  const uint8_t* base;
  uint32_t off;
  __device__ __forceinline__ uint32_t at4(uint32_t i) const { return lds4(base, off + i); }
};

// Next UTF-16 unit of Go's utf16.Encode([]rune(s)) over message bytes [0, len) of src:
// i = byte position, pend = the pending low surrogate (0: none).  Invalid UTF-8 ->
// U+FFFD consuming one byte, as utf8.DecodeRune.  Returns false at the end of the message.
template <class S>
__device__ __forceinline__ bool utf16_next(const S& src, uint32_t len, uint32_t& i, uint32_t& pend, uint32_t& u) {
  if (pend) { u = pend; pend = 0; return true; }
  if (i >= len) return false;
  const uint32_t x = src.at4(i);
  const uint32_t b0 = x & 255u, b1 = (x >> 8) & 255u, b2 = (x >> 16) & 255u, b3 = x >> 24;
  uint32_t r = b0, sz = 1;
  if (b0 >= 0x80u) {
    r = 0xFFFDu;
    uint32_t size = 0, lo = 0x80u, hi = 0xBFu;
    if (b0 >= 0xC2u && b0 <= 0xDFu) size = 2;
    else if (b0 >= 0xE0u && b0 <= 0xEFu) { size = 3; lo = b0 == 0xE0u ? 0xA0u : 0x80u; hi = b0 == 0xEDu ? 0x9Fu : 0xBFu; }
    else if (b0 >= 0xF0u && b0 <= 0xF4u) { size = 4; lo = b0 == 0xF0u ? 0x90u : 0x80u; hi = b0 == 0xF4u ? 0x8Fu : 0xBFu; }
    const bool c2 = b2 >= 0x80u && b2 <= 0xBFu, c3 = b3 >= 0x80u && b3 <= 0xBFu;
    const bool ok = size && i + size <= len && b1 >= lo && b1 <= hi && (size < 3 || c2) && (size < 4 || c3);
    if (ok) {
      sz = size;
      r = size == 2 ? ((b0 & 0x1Fu) << 6) | (b1 & 0x3Fu)
        : size == 3 ? ((b0 & 0x0Fu) << 12) | ((b1 & 0x3Fu) << 6) | (b2 & 0x3Fu)
                    : ((b0 & 0x07u) << 18) | ((b1 & 0x3Fu) << 12) | ((b2 & 0x3Fu) << 6) | (b3 & 0x3Fu);
    }
  }
  i += sz;
  if (r >= 0x10000u) {
    const uint32_t v = r - 0x10000u;
    u = 0xD800u + (v >> 10);
    pend = 0xDC00u + (v & 0x3FFu);
  } else {
    u = r;
  }
  return true;
}

// NTLM = MD4 over the UTF-16LE of the candidate's runes (Go []rune + utf16.Encode), the
// units produced while each 64-byte message block is filled (no UTF-16 buffer, any
// length).  Wave-collective loop over the active lanes: lanes whose digest is done keep
// their state.
template <class S>
__device__ __forceinline__ void ntlm_stream(const S& src, uint32_t len, uint32_t* d) {
  uint32_t st[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
  uint32_t i = 0, pend = 0, nu = 0;
  bool padded = false, fin = false;
  while (__builtin_amdgcn_ballot_w64(!fin)) {
    uint32_t M[16];
    const bool padprev = padded;
    uint32_t padw = 16;  // message word of this block holding the 0x80 pad
#pragma unroll
    for (int j = 0; j < 16; j++) {
      uint32_t w = 0;
#pragma unroll
      for (int h = 0; h < 2; h++) {
        uint32_t u = 0;
        if (utf16_next(src, len, i, pend, u)) {
          w |= u << (16 * h);
          nu++;
        } else if (!padded) {
          w |= 0x80u << (16 * h);
          padded = true;
          padw = (uint32_t)j;
        }
      }
      M[j] = w;
    }
    const bool last = padprev || (padded && padw <= 13u);
    if (last) {  // 64-bit little-endian bit length: 16 bits per unit
      M[14] = nu << 4;
      M[15] = nu >> 28;
    }
    if (!fin) {
      uint32_t s2[4] = {st[0], st[1], st[2], st[3]};
      md4_block(s2, M);
      st[0] = s2[0]; st[1] = s2[1]; st[2] = s2[2]; st[3] = s2[3];
    }
    fin = fin || last;
  }
  d[0] = st[0]; d[1] = st[1]; d[2] = st[2]; d[3] = st[3];
}

// the fused kernel's form: the candidate in the LDS ring
__device__ __forceinline__ void ntlm_lds(const uint8_t* base, uint32_t off, uint32_t len, uint32_t* d) {
  MdLds src;
  src.base = base;
  src.off = off;
  ntlm_stream(src, len, d);
}
