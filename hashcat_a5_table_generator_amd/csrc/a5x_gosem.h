// a5x_gosem.h -- the Go 1.23 standard-library behaviours the reference's table
// loader and dictionary reader depend on, restated for
// the C++ host side of liba5x:
//   bufio.Scanner + ScanLines        main.go:72-74 (dict), main.go:116 (tables)
//   strings.TrimSpace                main.go:118
//   strings.SplitN(line, "=", 2)     main.go:123
//   decodeHexNotation/hex.DecodeString  main.go:147-162
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <string.h>

#include <string>

namespace a5x {
namespace gosem {

constexpr size_t kMaxScanToken = 64 * 1024;  // bufio.MaxScanTokenSize
constexpr int kRuneError = 0xFFFD;

// utf8.DecodeRuneInString
inline int decode_rune(const uint8_t* s, size_t n, int* size) {
  if (n == 0) { *size = 0; return kRuneError; }
  const uint8_t b0 = s[0];
  if (b0 < 0x80) { *size = 1; return b0; }
  int sz;
  uint8_t lo = 0x80, hi = 0xBF;
  if (b0 >= 0xC2 && b0 <= 0xDF) sz = 2;
  else if (b0 >= 0xE0 && b0 <= 0xEF) { sz = 3; if (b0 == 0xE0) lo = 0xA0; if (b0 == 0xED) hi = 0x9F; }
  else if (b0 >= 0xF0 && b0 <= 0xF4) { sz = 4; if (b0 == 0xF0) lo = 0x90; if (b0 == 0xF4) hi = 0x8F; }
  else { *size = 1; return kRuneError; }
  if (n < (size_t)sz || s[1] < lo || s[1] > hi) { *size = 1; return kRuneError; }
  for (int k = 2; k < sz; k++)
    if (s[k] < 0x80 || s[k] > 0xBF) { *size = 1; return kRuneError; }
  *size = sz;
  if (sz == 2) return ((b0 & 0x1F) << 6) | (s[1] & 0x3F);
  if (sz == 3) return ((b0 & 0x0F) << 12) | ((s[1] & 0x3F) << 6) | (s[2] & 0x3F);
  return ((b0 & 0x07) << 18) | ((s[1] & 0x3F) << 12) | ((s[2] & 0x3F) << 6) | (s[3] & 0x3F);
}

// utf8.DecodeLastRuneInString(s[:end])
inline int decode_last_rune(const uint8_t* s, size_t end, int* size) {
  if (end == 0) { *size = 0; return kRuneError; }
  long start = (long)end - 1;
  if (s[start] < 0x80) { *size = 1; return s[start]; }
  long lim = (long)end - 4;
  if (lim < 0) lim = 0;
  for (start--; start >= lim; start--)
    if ((s[start] & 0xC0) != 0x80) break;
  if (start < 0) start = 0;
  int sz;
  const int r = decode_rune(s + start, end - (size_t)start, &sz);
  if ((size_t)start + (size_t)sz != end) { *size = 1; return kRuneError; }
  *size = sz;
  return r;
}

// unicode.IsSpace
inline bool is_space_rune(int r) {
  switch (r) {
    case '\t': case '\n': case '\v': case '\f': case '\r': case ' ': case 0x85: case 0xA0:
    case 0x1680: case 0x2028: case 0x2029: case 0x202F: case 0x205F: case 0x3000:
      return true;
    default:
      return r >= 0x2000 && r <= 0x200A;
  }
}

inline bool is_ascii_space(uint8_t c) {
  return c == '\t' || c == '\n' || c == '\v' || c == '\f' || c == '\r' || c == ' ';
}

// strings.TrimSpace: ASCII fast path from both ends; at the first non-ASCII byte
// Go falls back to rune-wise unicode.IsSpace trimming (TrimFunc/TrimRightFunc).
inline void trim_space(const uint8_t** b, size_t* n) {
  const uint8_t* s = *b;
  const size_t len = *n;
  size_t start = 0;
  auto trim_right = [](const uint8_t* p, size_t m) {
    while (m > 0) {
      int sz;
      const int r = decode_last_rune(p, m, &sz);
      if (!is_space_rune(r)) break;
      m -= (size_t)sz;
    }
    return m;
  };
  for (; start < len; start++) {
    const uint8_t c = s[start];
    if (c >= 0x80) {
      const uint8_t* p = s + start;
      size_t m = len - start, i = 0;
      while (i < m) {
        int sz;
        const int r = decode_rune(p + i, m - i, &sz);
        if (!is_space_rune(r)) break;
        i += (size_t)sz;
      }
      *b = p + i;
      *n = trim_right(p + i, m - i);
      return;
    }
    if (!is_ascii_space(c)) break;
  }
  size_t stop = len;
  for (; stop > start; stop--) {
    const uint8_t c = s[stop - 1];
    if (c >= 0x80) {
      *b = s + start;
      *n = trim_right(s + start, stop - start);
      return;
    }
    if (!is_ascii_space(c)) break;
  }
  *b = s + start;
  *n = stop - start;
}

inline int hexval(uint8_t c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}

// decodeHexNotation: "$HEX[..]" (len >= 7) -> bytes with ' ' removed; otherwise
// the input unchanged.  false = hex.DecodeString error (the line is skipped).
inline bool decode_hex_notation(const uint8_t* v, size_t n, std::string* out) {
  if (n < 7 || v[0] != '$' || v[1] != 'H' || v[2] != 'E' || v[3] != 'X' || v[4] != '[' || v[n - 1] != ']') {
    out->assign((const char*)v, n);
    return true;
  }
  std::string hex;
  for (size_t i = 5; i + 1 < n; i++)
    if (v[i] != ' ') hex.push_back((char)v[i]);
  if (hex.size() % 2) return false;
  out->clear();
  for (size_t i = 0; i < hex.size(); i += 2) {
    const int a = hexval((uint8_t)hex[i]), b = hexval((uint8_t)hex[i + 1]);
    if (a < 0 || b < 0) return false;
    out->push_back((char)((a << 4) | b));
  }
  return true;
}

// bufio.Scanner.Scan with ScanLines: returns 1 (token), 0 (EOF), -1 (ErrTooLong)
inline int scan_line(const uint8_t* d, size_t n, size_t* pos, const uint8_t** line, size_t* len) {
  if (*pos >= n) return 0;
  size_t lim = n - *pos;
  if (lim > kMaxScanToken) lim = kMaxScanToken;
  const uint8_t* nl = (const uint8_t*)memchr(d + *pos, '\n', lim);
  size_t l;
  if (!nl) {
    if (n - *pos >= kMaxScanToken) return -1;
    l = n - *pos;
    *line = d + *pos;
    *pos = n;
  } else {
    l = (size_t)(nl - (d + *pos));
    *line = d + *pos;
    *pos += l + 1;
  }
  if (l && (*line)[l - 1] == '\r') l--;
  *len = l;
  return 1;
}

}  // namespace gosem
}  // namespace a5x
