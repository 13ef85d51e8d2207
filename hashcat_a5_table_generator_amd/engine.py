"""Host-side mirror of the reference's operator interface, running on liba5x.

Reference functions (``/root/reference/main.go``) and their counterparts here:

=====================================  ==========================================
``readSubstitutionTable`` (108-144)    :func:`read_substitution_table`
``decodeHexNotation`` (147-162)        :func:`decode_hex_notation`
``-t`` merge loop (40-50)              :meth:`Context.load_tables`
``processWord`` (168-205)              :func:`process_word` / :meth:`Context.expand`
``processWordReverse`` (208-261)       :func:`process_word_reverse` (mode 1)
``processWordSubstituteAll`` (308)     :func:`process_word_substitute_all` (mode 2)
``...SubstituteAllReverse`` (369)      :func:`process_word_substitute_all_reverse`
word scanner (72-74)                   :func:`split_words`
channel + writer (58-68)               :meth:`Context.expand` sink / :func:`generate`
=====================================  ==========================================

Everything computes on the GPU through the C ABI (``include/a5x.h``); there is
no host fallback.
"""
from __future__ import annotations

import ctypes
import io
import os
import sys
from typing import BinaryIO, Dict, Iterable, Iterator, List, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from ._lib import A5xError, Stats, check

MODE_DEFAULT = 0
MODE_REVERSE = 1
MODE_SUBALL = 2
MODE_SUBALL_REVERSE = 3
ALGO_MD5 = 0   # RFC 1321 (Go crypto/md5)
ALGO_NTLM = 1  # MD4 over UTF-16LE ([]rune + utf16.Encode)

SubMap = Dict[bytes, List[bytes]]


def mode_of(substitute_all: bool, reverse_sub: bool) -> int:
    """The engine switch of ``main.go:80-92``."""
    return (MODE_SUBALL if substitute_all else MODE_DEFAULT) + (1 if reverse_sub else 0)


def pack_words(words: Sequence[bytes]) -> Tuple[np.ndarray, np.ndarray]:
    """Contiguous word bytes + ``n+1`` u64 offsets (the batch layout of the ABI)."""
    offs = np.zeros(len(words) + 1, dtype=np.uint64)
    if len(words):
        offs[1:] = np.cumsum(np.fromiter((len(w) for w in words), dtype=np.uint64, count=len(words)))
    data = np.frombuffer(b"".join(words) + b"\0" * 16, dtype=np.uint8).copy()
    return data, offs


def split_words(data: bytes) -> Tuple[np.ndarray, np.ndarray]:
    """Dictionary bytes -> words exactly as ``bufio.Scanner`` yields them (``main.go:72-74``)."""
    L = _lib.load()
    n = ctypes.c_uint64()
    check(L.a5x_split_words(data, len(data), None, None, 0, ctypes.byref(n)))
    words = np.zeros(len(data) + 16, dtype=np.uint8)
    offs = np.zeros(n.value + 2, dtype=np.uint64)
    check(L.a5x_split_words(data, len(data), words.ctypes.data, offs.ctypes.data, offs.size, ctypes.byref(n)))
    return words, offs[: n.value + 1]


class Context:
    """One device context (``a5x_ctx``) with its merged substitution map."""

    def __init__(self, device: int = 0):
        self._L = _lib.load()
        h = ctypes.c_void_p()
        rc = self._L.a5x_create(device, ctypes.byref(h))
        if rc != 0:
            why = (self._L.a5x_create_error() or b"").decode(errors="replace")
            raise A5xError(rc, why or f"a5x_create(device={device}) failed")
        self.h = h
        self.device = device

    def close(self) -> None:
        if getattr(self, "h", None):
            self._L.a5x_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _chk(self, rc: int) -> None:
        check(rc, self.h)

    @property
    def device_name(self) -> str:
        buf = ctypes.create_string_buffer(256)
        cu = ctypes.c_int()
        self._chk(self._L.a5x_device_info(self.h, buf, 256, ctypes.byref(cu)))
        return buf.value.decode()

    # ---- tables ------------------------------------------------------------
    def load_tables(self, paths: Iterable[str]) -> "Context":
        """``-t`` files merged in order (``main.go:40-50``)."""
        for p in paths:
            self._chk(self._L.a5x_load_table_file(self.h, os.fsencode(p)))
        return self

    def parse_table(self, data: bytes) -> "Context":
        self._chk(self._L.a5x_parse_table(self.h, data, len(data)))
        return self

    def set_table(self, sub: SubMap) -> "Context":
        keys = list(sub.keys())
        kb = b"".join(keys)
        koff = np.zeros(len(keys) + 1, dtype=np.uint64)
        koff[1:] = np.cumsum([len(k) for k in keys]) if keys else []
        vals, vkey = [], []
        for i, k in enumerate(keys):
            for v in sub[k]:
                vals.append(v)
                vkey.append(i)
        vb = b"".join(vals)
        voff = np.zeros(len(vals) + 1, dtype=np.uint64)
        if vals:
            voff[1:] = np.cumsum([len(v) for v in vals])
        vk = np.array(vkey, dtype=np.uint32)
        kbuf = np.frombuffer(kb + b"\0", dtype=np.uint8)
        vbuf = np.frombuffer(vb + b"\0", dtype=np.uint8)
        self._chk(self._L.a5x_set_table(self.h, kbuf.ctypes.data, koff.ctypes.data, len(keys), vbuf.ctypes.data,
                                        voff.ctypes.data, vk.ctypes.data if len(vk) else None, len(vals)))
        return self

    def clear_table(self) -> None:
        self._chk(self._L.a5x_clear_table(self.h))

    def table(self) -> SubMap:
        nk, nv, kb, vb = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint64(), ctypes.c_uint64()
        self._chk(self._L.a5x_table_export(self.h, ctypes.byref(nk), ctypes.byref(nv), ctypes.byref(kb),
                                           ctypes.byref(vb), None, None, None, None, None))
        ko = np.zeros(kb.value + 1, dtype=np.uint8)
        vo = np.zeros(vb.value + 1, dtype=np.uint8)
        koff = np.zeros(nk.value + 1, dtype=np.uint64)
        voff = np.zeros(nv.value + 1, dtype=np.uint64)
        vkey = np.zeros(max(nv.value, 1), dtype=np.uint32)
        self._chk(self._L.a5x_table_export(self.h, None, None, None, None, ko.ctypes.data, koff.ctypes.data,
                                           vo.ctypes.data, voff.ctypes.data, vkey.ctypes.data))
        kbytes, vbytes = ko.tobytes(), vo.tobytes()
        keys = [kbytes[koff[i]:koff[i + 1]] for i in range(nk.value)]
        out: SubMap = {k: [] for k in keys}
        for j in range(nv.value):
            out[keys[vkey[j]]].append(vbytes[voff[j]:voff[j + 1]])
        return out

    # ---- expansion (host buffers) -----------------------------------------
    def keyspace(self, words: np.ndarray, offs: np.ndarray, mode: int = MODE_DEFAULT, mn: int = 0,
                 mx: int = 15) -> Tuple[np.ndarray, np.ndarray]:
        n = len(offs) - 1
        cnt = np.zeros(max(n, 1), dtype=np.uint64)
        byt = np.zeros(max(n, 1), dtype=np.uint64)
        self._chk(self._L.a5x_keyspace(self.h, words.ctypes.data, offs.ctypes.data, n, mode, mn, mx,
                                       cnt.ctypes.data, byt.ctypes.data))
        return cnt[:n], byt[:n]

    def expand(self, words: np.ndarray, offs: np.ndarray, mode: int = MODE_DEFAULT, mn: int = 0, mx: int = 15,
               sink=None, cand_begin: int = 0, cand_end: Optional[int] = None) -> Tuple[bytes, dict]:
        """Expand a packed batch; returns the output bytes (words in order) unless a sink is given.
        cand_begin / cand_end: only the batch's candidates [cand_begin, cand_end) (a5x_expand_range)."""
        chunks: List[bytes] = []

        def _cb(_u, p, n):
            data = ctypes.string_at(p, n)
            if sink is not None:
                return 1 if sink(data) else 0
            chunks.append(data)
            return 0

        st = Stats()
        cb = _lib.SINK(_cb)
        ce = (1 << 64) - 1 if cand_end is None else cand_end
        self._chk(self._L.a5x_expand_range(self.h, words.ctypes.data, offs.ctypes.data, len(offs) - 1, mode, mn, mx,
                                           cand_begin, ce, cb, None, ctypes.byref(st)))
        return b"".join(chunks), st.as_dict()

    def expand_words(self, words: Sequence[bytes], mode: int = MODE_DEFAULT, mn: int = 0, mx: int = 15) -> List[List[bytes]]:
        """Per-word candidate lists (newline framing removed)."""
        data, offs = pack_words(words)
        cnt, byt = self.keyspace(data, offs, mode, mn, mx)
        out, _ = self.expand(data, offs, mode, mn, mx)
        res, pos = [], 0
        for i in range(len(words)):
            seg = out[pos:pos + int(byt[i])]
            pos += int(byt[i])
            res.append(_split_lines(seg, int(cnt[i])))
        return res

    # ---- device-resident ----------------------------------------------------
    def expand_device(self, d_words: int, d_offs: int, n_words: int, d_out: int, out_cap: int,
                      mode: int = MODE_DEFAULT, mn: int = 0, mx: int = 15, cand_begin: int = 0,
                      cand_end: int = (1 << 64) - 1, d_cand_off: int = 0, d_byte_off: int = 0,
                      stream: int = 0) -> dict:
        st = Stats()
        self._chk(self._L.a5x_expand_device(self.h, d_words, d_offs, n_words, mode, mn, mx, cand_begin, cand_end,
                                            d_out or None, out_cap, d_cand_off or None, d_byte_off or None,
                                            ctypes.byref(st), stream or None))
        return st.as_dict()

    # ---- fused digest + lookup ----------------------------------
    def set_targets(self, algo: int, digests) -> None:
        """Device target set from 16-byte digests (bytes of length 16*n or an (n,16) uint8 array)."""
        buf = np.ascontiguousarray(np.frombuffer(bytes(digests), dtype=np.uint8) if isinstance(digests, (bytes, bytearray))
                                   else np.asarray(digests, dtype=np.uint8)).reshape(-1)
        if buf.size % 16:
            raise ValueError("digests must be 16 bytes each")
        self._chk(self._L.a5x_set_targets(self.h, algo, buf.ctypes.data if buf.size else None, buf.size // 16))

    @staticmethod
    def _hits(arr, n) -> List[Tuple[int, int, bytes]]:
        return [(int(h.word), int(h.cand), bytes(h.digest)) for h in arr[:n]]

    def expand_digest(self, words: np.ndarray, offs: np.ndarray, mode: int = MODE_DEFAULT, mn: int = 0,
                      mx: int = 15, hit_cap: int = 1 << 16) -> Tuple[List[Tuple[int, int, bytes]], dict]:
        """Expand + hash + probe on the device; returns ([(word, cand_in_word, digest)], stats)."""
        arr = (_lib.Hit * max(1, hit_cap))()
        nh = ctypes.c_uint64()
        st = Stats()
        self._chk(self._L.a5x_expand_digest(self.h, words.ctypes.data, offs.ctypes.data, len(offs) - 1, mode, mn, mx,
                                            arr, hit_cap, ctypes.byref(nh), ctypes.byref(st)))
        return self._hits(arr, min(nh.value, hit_cap)), st.as_dict()

    def expand_digest_device(self, d_words: int, d_offs: int, n_words: int, mode: int = MODE_DEFAULT, mn: int = 0,
                             mx: int = 15, scratch_bytes: int = 0, hit_cap: int = 1 << 16,
                             stream: int = 0, cand_begin: int = 0,
                             cand_end: Optional[int] = None) -> Tuple[List[Tuple[int, int, bytes]], dict]:
        """Fused expansion + digest + target lookup of the batch's candidates (all of them,
        or the global candidates [cand_begin, cand_end): a5x_expand_digest_range_device)."""
        # (one hit buffer per context, grown on demand: a fresh 1M-entry ctypes array costs
        # milliseconds of host zeroing per call)
        buf = getattr(self, "_hit_buf", None)
        if buf is None or len(buf) < max(1, hit_cap):
            buf = self._hit_buf = (_lib.Hit * max(1, hit_cap))()
        arr = buf
        nh = ctypes.c_uint64()
        st = Stats()
        if cand_begin == 0 and cand_end is None:
            self._chk(self._L.a5x_expand_digest_device(self.h, d_words, d_offs, n_words, mode, mn, mx, scratch_bytes,
                                                       arr, hit_cap, ctypes.byref(nh), ctypes.byref(st),
                                                       stream or None))
        else:
            self._chk(self._L.a5x_expand_digest_range_device(
                self.h, d_words, d_offs, n_words, mode, mn, mx, cand_begin, (1 << 64) - 1 if cand_end is None else cand_end,
                scratch_bytes, arr, hit_cap, ctypes.byref(nh), ctypes.byref(st), stream or None))
        return self._hits(arr, min(nh.value, hit_cap)), st.as_dict()

    def format_hits(self, words: np.ndarray, offs: np.ndarray, hits, mode: int = MODE_DEFAULT, mn: int = 0,
                    mx: int = 15) -> bytes:
        """hashcat "hexdigest:plain\\n" lines for hits [(word, cand, digest)] of this batch
        (a5x_format_hits; plains in $HEX[] form when hashcat's outfile would hexify them)."""
        arr = (_lib.Hit * max(1, len(hits)))()
        for k, (w, c, d) in enumerate(hits):
            arr[k].word, arr[k].cand = int(w), int(c)
            ctypes.memmove(arr[k].digest, bytes(d), 16)
        chunks: List[bytes] = []

        def _cb(_u, p, n):
            chunks.append(ctypes.string_at(p, n))
            return 0

        cb = _lib.SINK(_cb)
        self._chk(self._L.a5x_format_hits(self.h, words.ctypes.data, offs.ctypes.data, len(offs) - 1, mode, mn, mx,
                                          arr, len(hits), cb, None))
        return b"".join(chunks)

    def digest_lines_device(self, algo: int, d_lines: int, nbytes: int, d_digests: int, cap: int,
                            stream: int = 0) -> int:
        """16-byte digest of every line of a device "cand\n" stream; returns the line count."""
        n = ctypes.c_uint64()
        self._chk(self._L.a5x_digest_lines_device(self.h, algo, d_lines, nbytes, d_digests or None, cap,
                                                  ctypes.byref(n), stream or None))
        return n.value

    def keyspace_device(self, d_words: int, d_offs: int, n_words: int, mode: int = MODE_DEFAULT, mn: int = 0,
                        mx: int = 15, d_cand_off: int = 0, d_byte_off: int = 0, stream: int = 0) -> Tuple[int, int]:
        tc, tb = ctypes.c_uint64(), ctypes.c_uint64()
        self._chk(self._L.a5x_keyspace_device(self.h, d_words, d_offs, n_words, mode, mn, mx, d_cand_off or None,
                                              d_byte_off or None, ctypes.byref(tc), ctypes.byref(tb),
                                              stream or None))
        return tc.value, tb.value

    def locate_device(self, d_words: int, d_offs: int, n_words: int, cands, mode: int = MODE_DEFAULT, mn: int = 0,
                      mx: int = 15, stream: int = 0) -> np.ndarray:
        """Output byte offsets of global candidate indices (``a5x_locate_device``)."""
        q = np.ascontiguousarray(cands, dtype=np.uint64)
        out = np.zeros(max(1, q.size), dtype=np.uint64)
        self._chk(self._L.a5x_locate_device(self.h, d_words, d_offs, n_words, mode, mn, mx,
                                            q.ctypes.data if q.size else None, q.size, out.ctypes.data,
                                            stream or None))
        return out[: q.size]

    def split_device(self, d_words: int, d_offs: int, n_words: int, byte_targets, mode: int = MODE_DEFAULT,
                     mn: int = 0, mx: int = 15, stream: int = 0) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        """(global candidate, word, candidate in word) of the first candidate starting at or
        after each byte target (``a5x_split_device``: intra-word split points)."""
        t = np.ascontiguousarray(byte_targets, dtype=np.uint64)
        g, w, c = (np.zeros(max(1, t.size), dtype=np.uint64) for _ in range(3))
        self._chk(self._L.a5x_split_device(self.h, d_words, d_offs, n_words, mode, mn, mx,
                                           t.ctypes.data if t.size else None, t.size, g.ctypes.data, w.ctypes.data,
                                           c.ctypes.data, stream or None))
        return g[: t.size], w[: t.size], c[: t.size]

    def digest_device(self, d_out: int, d_byte_off: int, out_base: int, n_words: int, d_digest: int,
                      stream: int = 0) -> None:
        self._chk(self._L.a5x_digest_device(self.h, d_out, d_byte_off, out_base, n_words, d_digest,
                                            stream or None))


def _split_lines(seg: bytes, count: int) -> List[bytes]:
    if not seg:
        return []
    parts = seg.split(b"\n")
    assert parts[-1] == b""
    parts = parts[:-1]
    return parts


def format_plain(plain: bytes) -> bytes:
    """The plain as a hashcat outfile line writes it (``a5x_format_plain``)."""
    L = _lib.load()
    n = ctypes.c_size_t()
    check(L.a5x_format_plain(plain, len(plain), None, 0, ctypes.byref(n)))
    out = ctypes.create_string_buffer(max(1, n.value))
    check(L.a5x_format_plain(plain, len(plain), out, n.value, ctypes.byref(n)))
    return out.raw[:n.value]


def partition(prefix: np.ndarray, parts: int) -> np.ndarray:
    """Balanced split points over a prefix array (``a5x_partition``)."""
    L = _lib.load()
    prefix = np.ascontiguousarray(prefix, dtype=np.uint64)
    split = np.zeros(parts + 1, dtype=np.uint64)
    check(L.a5x_partition(prefix.ctypes.data, len(prefix) - 1, parts, split.ctypes.data))
    return split


# ---------------------------------------------------------------------------
# function-level mirror of main.go
# ---------------------------------------------------------------------------
_default_ctx: Optional[Context] = None


def _ctx() -> Context:
    global _default_ctx
    if _default_ctx is None:
        _default_ctx = Context(int(os.environ.get("A5X_DEVICE", "0")))
    return _default_ctx


def read_substitution_table(path: str) -> SubMap:
    """``readSubstitutionTable`` (``main.go:108-144``) via the library's Go-exact parser
    (a private host-only context: the shared default context's table is left alone)."""
    with Context(-1) as c:
        c.load_tables([path])
        return c.table()


def decode_hex_notation(value: bytes) -> bytes:
    """``decodeHexNotation`` (``main.go:147-162``); raises ``ValueError`` like the Go error.
    Parsed in a private host-only context (no GPU, the default context untouched)."""
    if len(value) < 7 or not value.startswith(b"$HEX[") or not value.endswith(b"]"):
        return value
    with Context(-1) as c:
        c.parse_table(b"k=" + value + b"\n")
        t = c.table()
    if b"k" not in t:
        raise ValueError(f"invalid hex string {value[5:-1]!r}")
    return t[b"k"][0]


def _engine(word: bytes, sub_map: SubMap, mn: int, mx: int, mode: int) -> List[bytes]:
    c = _ctx()
    c.set_table(sub_map)
    return c.expand_words([word], mode, mn, mx)[0]


def process_word(word: bytes, sub_map: SubMap, min_substitute: int, max_substitute: int) -> List[bytes]:
    """``processWord`` (``main.go:168``): the candidates the reference sends on ``out``."""
    return _engine(word, sub_map, min_substitute, max_substitute, MODE_DEFAULT)


def process_word_reverse(word: bytes, sub_map: SubMap, min_substitute: int, max_substitute: int) -> List[bytes]:
    """``processWordReverse`` (``main.go:208``)."""
    return _engine(word, sub_map, min_substitute, max_substitute, MODE_REVERSE)


def process_word_substitute_all(word: bytes, sub_map: SubMap, min_substitute: int, max_substitute: int) -> List[bytes]:
    """``processWordSubstituteAll`` (``main.go:308``)."""
    return _engine(word, sub_map, min_substitute, max_substitute, MODE_SUBALL)


def process_word_substitute_all_reverse(word: bytes, sub_map: SubMap, min_substitute: int,
                                        max_substitute: int) -> List[bytes]:
    """``processWordSubstituteAllReverse`` (``main.go:369``)."""
    return _engine(word, sub_map, min_substitute, max_substitute, MODE_SUBALL_REVERSE)


MAX_SCAN_TOKEN = 64 * 1024  # bufio.MaxScanTokenSize


def iter_word_batches(f: BinaryIO, batch_words: int = 1 << 22,
                      chunk: int = 64 << 20) -> Iterator[Tuple[np.ndarray, np.ndarray]]:
    """The dictionary stream of ``main.go:52-56,72-74`` in bounded memory: ScanLines over
    ``chunk``-byte reads (LF split, one trailing CR dropped, a final unterminated line
    kept, and the first line with no newline in 64 KiB silently ends the input: the
    reference never checks ``scanner.Err()``).  Yields packed batches of at most
    ``batch_words`` words (``split_words`` layout)."""
    pend_w: List[np.ndarray] = []
    pend_o: List[np.ndarray] = []
    npend = 0

    def flush_pending():
        nonlocal pend_w, pend_o, npend
        lens = np.concatenate([np.diff(o.astype(np.int64)) for o in pend_o])
        body = np.concatenate([w[: int(o[-1])] for w, o in zip(pend_w, pend_o)])
        offs = np.zeros(len(lens) + 1, dtype=np.uint64)
        np.cumsum(lens, out=offs[1:])
        data = np.zeros(len(body) + 16, dtype=np.uint8)
        data[: len(body)] = body
        pend_w, pend_o, npend = [], [], 0
        return data, offs

    def take(words, offs):
        # split (words, offs) into the pending batch, yielding every full batch
        nonlocal npend
        n = len(offs) - 1
        i = 0
        while i < n:
            k = min(n - i, batch_words - npend)
            sub_o = (offs[i:i + k + 1] - offs[i]).astype(np.uint64)
            pend_w.append(words[int(offs[i]):int(offs[i + k])])
            pend_o.append(sub_o)
            npend += k
            i += k
            if npend == batch_words:
                yield flush_pending()

    rest = b""
    while True:
        block = f.read(chunk)
        eof = not block
        buf = rest + block
        if eof:
            part, rest = buf, b""
        else:
            cut = buf.rfind(b"\n") + 1
            part, rest = buf[:cut], buf[cut:]
        if part:
            words, offs = split_words(part)
            yield from take(words, offs)
            complete = part.count(b"\n") + (0 if part.endswith(b"\n") else 1)
            if len(offs) - 1 < complete:  # ErrTooLong inside this part: the input ends here
                break
        if eof:
            break
        if len(rest) >= MAX_SCAN_TOKEN:  # no newline in 64 KiB: ErrTooLong
            break
    if npend:
        yield flush_pending()


def generate(dict_file: str, table_files: Sequence[str], table_min: int = 0, table_max: int = 15,
             substitute_all: bool = False, reverse_sub: bool = False, out: Optional[BinaryIO] = None,
             device: int = 0, batch_words: int = 1 << 22, chunk: int = 64 << 20) -> int:
    """The whole ``main()`` (``main.go:28-100``): dict -> candidates on ``out``; returns
    candidates.  The dictionary is streamed (``iter_word_batches``): memory is bounded by
    one chunk and one batch, whatever the file size."""
    out = out if out is not None else sys.stdout.buffer
    mode = mode_of(substitute_all, reverse_sub)
    with Context(device) as c:
        c.load_tables(table_files)
        total = 0
        with open(dict_file, "rb") as f:
            for sub_words, sub_off in iter_word_batches(f, batch_words, chunk):
                _, st = c.expand(sub_words, sub_off, mode, table_min, table_max, sink=lambda d: out.write(d) and 0)
                total += st["candidates"]
        out.flush()
        return total


class DeviceBuffer:
    """A raw HBM allocation owned by a :class:`Context` (``a5x_dev_alloc``)."""

    def __init__(self, ctx: Context, nbytes: int):
        self.ctx = ctx
        self.nbytes = int(nbytes)
        p = ctypes.c_void_p()
        ctx._chk(ctx._L.a5x_dev_alloc(ctx.h, ctypes.byref(p), max(self.nbytes, 16)))
        self.ptr = p.value

    @classmethod
    def from_array(cls, ctx: Context, arr: np.ndarray) -> "DeviceBuffer":
        arr = np.ascontiguousarray(arr)
        b = cls(ctx, arr.nbytes)
        if arr.nbytes:
            ctx._chk(ctx._L.a5x_memcpy_h2d(ctx.h, b.ptr, arr.ctypes.data, arr.nbytes))
        return b

    def to_array(self, dtype=np.uint8, count: Optional[int] = None, offset: int = 0) -> np.ndarray:
        itemsize = np.dtype(dtype).itemsize
        n = (self.nbytes - offset) // itemsize if count is None else int(count)
        out = np.empty(n, dtype=dtype)
        if n:
            self.ctx._chk(self.ctx._L.a5x_memcpy_d2h(self.ctx.h, out.ctypes.data, self.ptr + offset, n * itemsize))
        return out

    def free(self) -> None:
        if self.ptr:
            self.ctx._L.a5x_dev_free(self.ctx.h, self.ptr)
            self.ptr = 0

    def __del__(self):
        try:
            if getattr(self.ctx, "h", None):
                self.free()
        except Exception:
            pass
