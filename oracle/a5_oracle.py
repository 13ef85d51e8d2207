"""CPU restatement of the reference ``main.go`` -- TEST INFRASTRUCTURE ONLY.

This module is the parity *checker*.  Only ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg may import it; the product path
(``hashcat_a5_table_generator_amd``) never does and fails loudly when its HIP
library is missing.

It restates, byte for byte, the Go reference (``/root/reference/main.go``,
go 1.23.5 per ``go.mod:3``) including the Go standard-library behaviours the
reference relies on:

* ``bufio.Scanner`` + ``ScanLines`` (``main.go:72-74``, ``116``)
* ``strings.TrimSpace`` with Go's ASCII fast path and ``unicode.IsSpace`` fallback
  (``main.go:118``)
* ``strings.SplitN(line, "=", 2)`` (``main.go:123``)
* ``decodeHexNotation`` / ``hex.DecodeString`` (``main.go:147-162``)
* the table merge across ``-t`` files (``main.go:40-50``)
* the four engines ``processWord`` (``main.go:168-205``), ``processWordReverse``
  (``main.go:208-305``, including the running-offset bug and its panic),
  ``processWordSubstituteAll`` (``main.go:308-365``) and
  ``processWordSubstituteAllReverse`` (``main.go:369-440``)
* the output format ``candidate + "\\n"`` (``main.go:66``).

Parity is pinned by SURVEY.md Appendix B's known-answer vectors (the reference
ships no tests; see DESIGN.md "Oracle") -- ``tests/test_oracle_golden.py``.

Go map iteration order is randomised, which makes ``-s``/``-s -r`` results
order-dependent for non-confluent tables (``main.go:339-341``, ``411-413``).  This
module applies replacements in *sorted pattern order* (the canonical order the
GPU engine uses) and offers :func:`substitute_all_possible` to enumerate every
application order for membership checks.
"""
from __future__ import annotations

import itertools
from typing import Dict, Iterable, Iterator, List, Optional, Sequence, Tuple

MAX_SCAN_TOKEN = 64 * 1024  # bufio.MaxScanTokenSize

MODE_DEFAULT = 0
MODE_REVERSE = 1
MODE_SUBALL = 2
MODE_SUBALL_REVERSE = 3


class ScanTooLong(Exception):
    """bufio.ErrTooLong -- token longer than the 64 KiB scanner buffer."""


class GoPanic(Exception):
    """A Go runtime panic in the reference (e.g. slice bounds out of range)."""


# ---------------------------------------------------------------------------
# Go stdlib restatements
# ---------------------------------------------------------------------------

def scan_lines(data: bytes, strict: bool) -> List[bytes]:
    """``bufio.Scanner`` with ``ScanLines`` (split on ``\\n``, drop one ``\\r``).

    A final unterminated line is returned; no empty token follows a trailing
    newline.  A line whose raw content is >= 64 KiB stops the scanner with
    ``ErrTooLong``: raised when ``strict`` (table path, ``main.go:143`` -> fatal),
    silently ending the token stream otherwise (dict path, ``main.go:73`` never
    checks ``scanner.Err()``).
    """
    out: List[bytes] = []
    pos = 0
    n = len(data)
    while pos < n:
        nl = data.find(b"\n", pos, pos + MAX_SCAN_TOKEN)
        if nl < 0:
            rest = n - pos
            if rest >= MAX_SCAN_TOKEN:
                if strict:
                    raise ScanTooLong()
                return out
            line = data[pos:]
            pos = n
        else:
            line = data[pos:nl]
            pos = nl + 1
        if line.endswith(b"\r"):
            line = line[:-1]
        out.append(line)
    return out


_ASCII_SPACE = frozenset(b"\t\n\v\f\r ")
_UNICODE_SPACE = frozenset(
    [0x09, 0x0A, 0x0B, 0x0C, 0x0D, 0x20, 0x85, 0xA0, 0x1680]
    + list(range(0x2000, 0x200B))
    + [0x2028, 0x2029, 0x202F, 0x205F, 0x3000]
)
RUNE_ERROR = 0xFFFD


def decode_rune(s: bytes, i: int) -> Tuple[int, int]:
    """``utf8.DecodeRuneInString(s[i:])`` -> (rune, size); invalid -> (U+FFFD, 1)."""
    n = len(s) - i
    if n <= 0:
        return RUNE_ERROR, 0
    b0 = s[i]
    if b0 < 0x80:
        return b0, 1
    if 0xC2 <= b0 <= 0xDF:
        size, lo, hi = 2, 0x80, 0xBF
    elif 0xE0 <= b0 <= 0xEF:
        size = 3
        lo, hi = (0xA0, 0xBF) if b0 == 0xE0 else ((0x80, 0x9F) if b0 == 0xED else (0x80, 0xBF))
    elif 0xF0 <= b0 <= 0xF4:
        size = 4
        lo, hi = (0x90, 0xBF) if b0 == 0xF0 else ((0x80, 0x8F) if b0 == 0xF4 else (0x80, 0xBF))
    else:
        return RUNE_ERROR, 1
    if n < size:
        # Go checks the accept range of the 2nd byte and continuation of the
        # rest before declaring a short sequence invalid; either way: (RuneError, 1).
        return RUNE_ERROR, 1
    b1 = s[i + 1]
    if not (lo <= b1 <= hi):
        return RUNE_ERROR, 1
    for k in range(2, size):
        if not (0x80 <= s[i + k] <= 0xBF):
            return RUNE_ERROR, 1
    if size == 2:
        return ((b0 & 0x1F) << 6) | (b1 & 0x3F), 2
    if size == 3:
        return ((b0 & 0x0F) << 12) | ((b1 & 0x3F) << 6) | (s[i + 2] & 0x3F), 3
    return (((b0 & 0x07) << 18) | ((b1 & 0x3F) << 12) | ((s[i + 2] & 0x3F) << 6)
            | (s[i + 3] & 0x3F)), 4


def decode_last_rune(s: bytes, end: int) -> Tuple[int, int]:
    """``utf8.DecodeLastRuneInString(s[:end])``."""
    if end <= 0:
        return RUNE_ERROR, 0
    start = end - 1
    if s[start] < 0x80:
        return s[start], 1
    lim = max(end - 4, 0)
    start -= 1
    while start >= lim:
        if (s[start] & 0xC0) != 0x80:
            break
        start -= 1
    if start < 0:
        start = 0
    r, size = decode_rune(s[:end], start)
    if start + size != end:
        return RUNE_ERROR, 1
    return r, size


def trim_space(s: bytes) -> bytes:
    """``strings.TrimSpace`` (go1.23): ASCII fast path, else ``unicode.IsSpace`` on runes."""
    start = 0
    while start < len(s):
        c = s[start]
        if c >= 0x80:
            return _trim_func(s[start:])
        if c not in _ASCII_SPACE:
            break
        start += 1
    stop = len(s)
    while stop > start:
        c = s[stop - 1]
        if c >= 0x80:
            return _trim_right_func(s[start:stop])
        if c not in _ASCII_SPACE:
            break
        stop -= 1
    return s[start:stop]


def _trim_left_func(s: bytes) -> bytes:
    i = 0
    while i < len(s):
        r, size = decode_rune(s, i)
        if r not in _UNICODE_SPACE or (r == RUNE_ERROR and size == 1):
            break
        i += size
    return s[i:]


def _trim_right_func(s: bytes) -> bytes:
    end = len(s)
    while end > 0:
        r, size = decode_last_rune(s, end)
        if r not in _UNICODE_SPACE:
            break
        end -= size
    return s[:end]


def _trim_func(s: bytes) -> bytes:
    return _trim_right_func(_trim_left_func(s))


_HEXVAL = {c: int(chr(c), 16) for c in b"0123456789abcdefABCDEF"}


def hex_decode_string(h: bytes) -> Optional[bytes]:
    """``hex.DecodeString``; ``None`` on any error (odd length or bad digit)."""
    if len(h) % 2:
        return None
    out = bytearray()
    for j in range(0, len(h), 2):
        a = _HEXVAL.get(h[j])
        b = _HEXVAL.get(h[j + 1])
        if a is None or b is None:
            return None
        out.append((a << 4) | b)
    return bytes(out)


def decode_hex_notation(value: bytes) -> Optional[bytes]:
    """``decodeHexNotation`` (``main.go:147-162``); ``None`` = decode error."""
    if len(value) < 7 or not value.startswith(b"$HEX[") or not value.endswith(b"]"):
        return value
    return hex_decode_string(value[5:-1].replace(b" ", b""))


def replace_all(s: bytes, old: bytes, new: bytes) -> bytes:
    """``strings.ReplaceAll``; an empty ``old`` inserts ``new`` around every UTF-8 rune."""
    if old:
        return s.replace(old, new)
    out = bytearray(new)
    i = 0
    while i < len(s):
        _, size = decode_rune(s, i)
        out += s[i:i + size]
        out += new
        i += size
    return bytes(out)


# ---------------------------------------------------------------------------
# Table loading (main.go:40-50, 102-162)
# ---------------------------------------------------------------------------

SubMap = Dict[bytes, List[bytes]]


def parse_table_bytes(data: bytes, log: Optional[list] = None) -> SubMap:
    """``readSubstitutionTable`` on file contents (``main.go:108-144``)."""
    subs: SubMap = {}
    for raw in scan_lines(data, strict=True):
        line = trim_space(raw)
        if not line or line.startswith(b"#"):
            continue
        eq = line.find(b"=")
        if eq < 0:
            continue
        key = decode_hex_notation(line[:eq])
        if key is None:
            if log is not None:
                log.append(("key", line))
            continue
        val = decode_hex_notation(line[eq + 1:])
        if val is None:
            if log is not None:
                log.append(("value", line))
            continue
        subs.setdefault(key, []).append(val)
    return subs


def merge_tables(tables: Iterable[SubMap]) -> SubMap:
    """``-t`` merge: per key, values appended in (-t order, line order) (``main.go:40-50``)."""
    merged: SubMap = {}
    for t in tables:
        for k, vs in t.items():
            merged.setdefault(k, []).extend(vs)
    return merged


def load_tables(paths: Sequence[str]) -> SubMap:
    tabs = []
    for p in paths:
        with open(p, "rb") as f:
            tabs.append(parse_table_bytes(f.read()))
    return merge_tables(tabs)


def read_words(data: bytes) -> List[bytes]:
    """Dictionary words as ``bufio.Scanner`` yields them (``main.go:72-74``)."""
    return scan_lines(data, strict=False)


# ---------------------------------------------------------------------------
# Engines
# ---------------------------------------------------------------------------

def process_word(word: bytes, sub: SubMap, mn: int, mx: int) -> List[bytes]:
    """``processWord`` (``main.go:168-205``): DFS over non-overlapping matches."""
    if mn == 0:
        mn = 1
    out: List[bytes] = []

    def gen(cur: bytes, cnt: int, start: int) -> None:
        i = start
        while i < len(cur):
            for kl in range(len(cur) - i, 0, -1):
                subs = sub.get(cur[i:i + kl])
                if subs is None:
                    continue
                for s in subs:
                    nw = cur[:i] + s + cur[i + kl:]
                    nc = cnt + 1
                    if nc > mx:
                        continue
                    if nc >= mn:
                        out.append(nw)
                    gen(nw, nc, i + len(s))
            i += 1

    gen(word, 0, 0)
    return out


def _go_combinations(n: int, k: int) -> List[List[int]]:
    """``generateCombinations`` (``main.go:263-281``); indices descending."""
    if k == 0:
        return [[]]
    if n < k:
        return []
    if k < 0:
        # main.go:273 recursion never reaches k==0 or n<k: unbounded recursion,
        # i.e. a fatal Go stack overflow.
        raise GoPanic("stack overflow in generateCombinations (negative k)")
    res = []
    for i in range(n - 1, k - 2, -1):
        for c in _go_combinations(i, k - 1):
            res.append([i] + c)
    return res


def process_word_reverse(word: bytes, sub: SubMap, mn: int, mx: int) -> List[bytes]:
    """``processWordReverse`` (``main.go:208-261``), bug-compatible.

    Combos are applied in descending index order with a running offset
    (``main.go:249-257``); a negative/oversized slice bound raises
    :class:`GoPanic` exactly where the Go runtime would panic.
    """
    positions: List[Tuple[int, int, List[bytes]]] = []
    for i in range(len(word)):
        for kl in range(1, len(word) - i + 1):
            s = sub.get(word[i:i + kl])
            if s is not None:
                positions.append((i, kl, s))
    total = len(positions)
    if total < mn:
        return []
    amax = min(mx, total)
    out: List[bytes] = []
    for k in range(amax, mn - 1, -1):
        for combo in _go_combinations(total, k):
            iv = sorted((positions[j][0], positions[j][0] + positions[j][1] - 1) for j in combo)
            if any(iv[t][0] <= iv[t - 1][1] for t in range(1, len(iv))):
                continue
            res = word
            off = 0
            for j in combo:
                st, kl, subs = positions[j]
                s0 = subs[0]
                a = st + off
                b = a + kl
                if a < 0 or a > len(res) or b > len(res):
                    raise GoPanic("slice bounds out of range")
                res = res[:a] + s0 + res[b:]
                off += len(s0) - kl
            out.append(res)
    return out


def unique_patterns(word: bytes, sub: SubMap) -> List[bytes]:
    """Sorted unique patterns present in ``word`` (``main.go:310-326``)."""
    pats = set()
    for i in range(len(word)):
        for p in sub:
            if i + len(p) <= len(word) and word[i:i + len(p)] == p:
                pats.add(p)
    return sorted(pats)


def _apply_in_order(word: bytes, assignment: Sequence[Tuple[bytes, bytes]]) -> bytes:
    r = word
    for p, v in assignment:
        r = replace_all(r, p, v)
    return r


def process_word_substitute_all(word: bytes, sub: SubMap, mn: int, mx: int) -> List[bytes]:
    """``processWordSubstituteAll`` (``main.go:308-365``), sorted-order application."""
    pats = unique_patterns(word, sub)
    out: List[bytes] = []

    def gen(cur: List[Tuple[bytes, bytes]], pos: int) -> None:
        if pos >= len(pats):
            if mn <= len(cur) <= mx:
                out.append(_apply_in_order(word, cur))
            return
        p = pats[pos]
        for v in sub[p]:
            gen(cur + [(p, v)], pos + 1)
        gen(cur, pos + 1)

    gen([], 0)
    return out


def process_word_substitute_all_reverse(word: bytes, sub: SubMap, mn: int, mx: int) -> List[bytes]:
    """``processWordSubstituteAllReverse`` (``main.go:369-440``), sorted-order application."""
    pats = unique_patterns(word, sub)
    if len(pats) < mn:
        return []
    allsubs = [(p, sub[p][0]) for p in pats if sub.get(p)]
    out: List[bytes] = []

    def gen(cur: List[Tuple[bytes, bytes]], pos: int) -> None:
        c = len(cur)
        if c < mn:
            return
        if c <= mx:
            out.append(_apply_in_order(word, cur))
        if c <= mn:
            return
        present = {p for p, _ in cur}
        for i in range(pos, len(pats)):
            if pats[i] not in present:
                continue
            gen([(p, v) for p, v in cur if p != pats[i]], i + 1)

    gen(allsubs, 0)
    return out


def substitute_all_possible(word: bytes, assignment: Sequence[Tuple[bytes, bytes]]) -> set:
    """Every result ``main.go:339-341`` can produce for one leaf (any map order)."""
    return {_apply_in_order(word, perm) for perm in itertools.permutations(assignment)}


def leaves_substitute_all(word: bytes, sub: SubMap, mn: int, mx: int, reverse: bool):
    """The (pattern, value) assignments of every emitted ``-s`` / ``-s -r`` leaf."""
    pats = unique_patterns(word, sub)
    leaves: List[List[Tuple[bytes, bytes]]] = []
    if not reverse:
        def gen(cur, pos):
            if pos >= len(pats):
                if mn <= len(cur) <= mx:
                    leaves.append(cur)
                return
            for v in sub[pats[pos]]:
                gen(cur + [(pats[pos], v)], pos + 1)
            gen(cur, pos + 1)
        gen([], 0)
    else:
        if len(pats) < mn:
            return leaves
        base = [(p, sub[p][0]) for p in pats]
        for k in range(len(base), -1, -1):
            if k < mn or k > mx:
                continue
            for comb in itertools.combinations(base, k):
                leaves.append(list(comb))
    return leaves


ENGINES = {
    MODE_DEFAULT: process_word,
    MODE_REVERSE: process_word_reverse,
    MODE_SUBALL: process_word_substitute_all,
    MODE_SUBALL_REVERSE: process_word_substitute_all_reverse,
}


def mode_of(substitute_all: bool, reverse: bool) -> int:
    """The engine switch of ``main.go:80-92``."""
    return (MODE_SUBALL if substitute_all else MODE_DEFAULT) + (1 if reverse else 0)


def expand(word: bytes, sub: SubMap, mode: int, mn: int, mx: int) -> List[bytes]:
    return ENGINES[mode](word, sub, mn, mx)


def expand_stream(words: Iterable[bytes], sub: SubMap, mode: int, mn: int, mx: int) -> Iterator[bytes]:
    """Whole-run output bytes in word order (one valid order of ``main.go:58-98``)."""
    for w in words:
        for c in expand(w, sub, mode, mn, mx):
            yield c + b"\n"


# ---------------------------------------------------------------------------
# Default-mode keyspace DP -- count and output bytes
# ---------------------------------------------------------------------------

def keyspace_default(word: bytes, sub: SubMap, mn: int, mx: int) -> Tuple[int, int]:
    """Exact (count, bytes incl. newline) of ``processWord`` without enumerating."""
    if mn == 0:
        mn = 1
    L = len(word)
    if mx < 1:
        return 0, 0
    C = min(mx, L)
    keys = {}
    for k, vs in sub.items():
        if k:
            keys.setdefault(len(k), {})[k] = vs
    N = [[0] * (C + 2) for _ in range(L + 1)]
    B = [[0] * (C + 2) for _ in range(L + 1)]
    # N[p][c]: number of ways to finish from p with exactly c more substitutions;
    # B[p][c]: total suffix bytes of those ways (without the newline).
    N[L][0] = 1
    for p in range(L - 1, -1, -1):
        for c in range(C + 1):
            n = N[p + 1][c]
            b = B[p + 1][c] + N[p + 1][c]
            if c >= 1:
                for kl, tab in keys.items():
                    if p + kl > L:
                        continue
                    vs = tab.get(word[p:p + kl])
                    if vs is None:
                        continue
                    for v in vs:
                        n += N[p + kl][c - 1]
                        b += B[p + kl][c - 1] + N[p + kl][c - 1] * len(v)
            N[p][c] = n
            B[p][c] = b
    lo = max(mn, 1)
    cnt = sum(N[0][c] for c in range(lo, C + 1))
    byt = sum(B[0][c] for c in range(lo, C + 1)) + cnt
    return cnt, byt
