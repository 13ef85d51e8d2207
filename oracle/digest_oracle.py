"""Digest oracle for the fused digest + lookup stage.

TEST INFRASTRUCTURE ONLY: tests/, __graft_entry__.smoke() and bench.py's checks may
use it as the checker; the product path never calls it.

* MD5  = ``hashlib.md5`` (RFC 1321, the same function as Go ``crypto/md5``).
* NTLM = MD4(UTF-16LE(candidate)).  OpenSSL 3 in this image refuses ``md4``
  ("unsupported hash type md4"), so MD4 is restated here from RFC 1320 and pinned by
  the RFC's own test suite (tests/test_digest_oracle.py) and the well-known vector
  NTLM("password") = 8846f7eaee8fb117ad06bdd830b7586c.  The UTF-16 conversion follows
  Go's ``utf16.Encode([]rune(s))``: each invalid UTF-8 byte becomes U+FFFD
  (``decode_rune`` of oracle/a5_oracle.py, Go 1.23 ``unicode/utf8``), runes above
  U+FFFF become surrogate pairs.
"""
from __future__ import annotations

import hashlib
import struct

from oracle.a5_oracle import decode_rune

MASK = 0xFFFFFFFF


def _rotl(x: int, s: int) -> int:
    x &= MASK
    return ((x << s) | (x >> (32 - s))) & MASK


def md4(msg: bytes) -> bytes:
    """RFC 1320 MD4."""
    n = len(msg)
    m = msg + b"\x80" + b"\x00" * ((55 - n) % 64) + struct.pack("<Q", (8 * n) & 0xFFFFFFFFFFFFFFFF)
    a, b, c, d = 0x67452301, 0xEFCDAB89, 0x98BADCFE, 0x10325476
    F = lambda x, y, z: (x & y) | (~x & z)
    G = lambda x, y, z: (x & y) | (x & z) | (y & z)
    H = lambda x, y, z: x ^ y ^ z
    for off in range(0, len(m), 64):
        X = struct.unpack("<16I", m[off:off + 64])
        aa, bb, cc, dd = a, b, c, d
        for i, s in zip(range(16), [3, 7, 11, 19] * 4):
            k = i
            if i % 4 == 0: a = _rotl(a + F(b, c, d) + X[k], s)
            elif i % 4 == 1: d = _rotl(d + F(a, b, c) + X[k], s)
            elif i % 4 == 2: c = _rotl(c + F(d, a, b) + X[k], s)
            else: b = _rotl(b + F(c, d, a) + X[k], s)
        for i, (k, s) in enumerate(zip([0, 4, 8, 12, 1, 5, 9, 13, 2, 6, 10, 14, 3, 7, 11, 15], [3, 5, 9, 13] * 4)):
            if i % 4 == 0: a = _rotl(a + G(b, c, d) + X[k] + 0x5A827999, s)
            elif i % 4 == 1: d = _rotl(d + G(a, b, c) + X[k] + 0x5A827999, s)
            elif i % 4 == 2: c = _rotl(c + G(d, a, b) + X[k] + 0x5A827999, s)
            else: b = _rotl(b + G(c, d, a) + X[k] + 0x5A827999, s)
        for i, (k, s) in enumerate(zip([0, 8, 4, 12, 2, 10, 6, 14, 1, 9, 5, 13, 3, 11, 7, 15], [3, 9, 11, 15] * 4)):
            if i % 4 == 0: a = _rotl(a + H(b, c, d) + X[k] + 0x6ED9EBA1, s)
            elif i % 4 == 1: d = _rotl(d + H(a, b, c) + X[k] + 0x6ED9EBA1, s)
            elif i % 4 == 2: c = _rotl(c + H(d, a, b) + X[k] + 0x6ED9EBA1, s)
            else: b = _rotl(b + H(c, d, a) + X[k] + 0x6ED9EBA1, s)
        a, b, c, d = (a + aa) & MASK, (b + bb) & MASK, (c + cc) & MASK, (d + dd) & MASK
    return struct.pack("<4I", a, b, c, d)


def utf16le_go(s: bytes) -> bytes:
    """``utf16.Encode([]rune(string(s)))`` as little-endian bytes."""
    out = bytearray()
    i = 0
    while i < len(s):
        r, size = decode_rune(s, i)
        i += size
        if r >= 0x10000:
            v = r - 0x10000
            out += struct.pack("<HH", 0xD800 + (v >> 10), 0xDC00 + (v & 0x3FF))
        else:
            out += struct.pack("<H", r)
    return bytes(out)


def ntlm(cand: bytes) -> bytes:
    return md4(utf16le_go(cand))


def md5(cand: bytes) -> bytes:
    return hashlib.md5(cand).digest()


ALGOS = {0: md5, 1: ntlm}
