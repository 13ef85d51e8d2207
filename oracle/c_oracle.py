"""ctypes wrapper for oracle/_build/liba5oracle.so -- TEST INFRASTRUCTURE ONLY.

The C restatement (``oracle/a5_oracle.c``) is the parity checker at sizes the
Python oracle cannot reach and the ``cpu_baseline`` leg of ``bench.py``.  Build it
with ``make -C oracle`` (``__graft_entry__.build()`` does).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import List, Optional, Sequence, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.environ.get("A5X_ORACLE_LIB") or os.path.join(_HERE, "_build", "liba5oracle.so")
_lib = None  # (A5X_ORACLE_LIB: tools/sanitize.sh points it at the ASan/UBSan build)

_u8p = ctypes.POINTER(ctypes.c_uint8)
_u64p = ctypes.POINTER(ctypes.c_uint64)
EMIT = ctypes.CFUNCTYPE(None, ctypes.c_void_p, _u8p, ctypes.c_size_t)


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _SO


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = ctypes.CDLL(_SO)
        L.a5o_table_new.restype = ctypes.c_void_p
        L.a5o_table_free.argtypes = [ctypes.c_void_p]
        L.a5o_table_add.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t]
        L.a5o_table_parse.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t]
        L.a5o_table_load_file.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
        L.a5o_table_nkeys.argtypes = [ctypes.c_void_p]
        L.a5o_table_nkeys.restype = ctypes.c_size_t
        L.a5o_table_get.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(_u8p),
                                    ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_size_t)]
        L.a5o_table_get_val.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.POINTER(_u8p),
                                        ctypes.POINTER(ctypes.c_size_t)]
        L.a5o_expand_word.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_int, EMIT, ctypes.c_void_p]
        L.a5o_digest_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                       ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
        L.a5o_expand_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                       ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                                       ctypes.c_void_p]
        L.a5o_expand_batch.restype = ctypes.c_int64
        L.a5o_run_pipeline.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                       ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       _u64p, _u64p]
        L.a5o_digest.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p]
        L.a5o_digest_run.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                                     ctypes.c_int, _u64p, _u64p]
        L.a5o_cand_hash.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
        L.a5o_cand_hash.restype = ctypes.c_uint64
        _lib = L
    return _lib


class CTable:
    """The merged ``map[string][]string`` held by the C oracle."""

    def __init__(self, paths: Sequence[str] = (), data: Sequence[bytes] = ()):
        self.h = lib().a5o_table_new()
        for p in paths:
            rc = lib().a5o_table_load_file(self.h, p.encode())
            if rc:
                raise OSError(f"oracle table load failed rc={rc}: {p}")
        for d in data:
            rc = lib().a5o_table_parse(self.h, d, len(d))
            if rc:
                raise ValueError(f"oracle table parse failed rc={rc}")

    @classmethod
    def from_map(cls, m: dict) -> "CTable":
        t = cls()
        for k, vs in m.items():
            for v in vs:
                lib().a5o_table_add(t.h, k, len(k), v, len(v))
        return t

    def to_map(self) -> dict:
        L = lib()
        out = {}
        for e in range(L.a5o_table_nkeys(self.h)):
            kp = _u8p(); kn = ctypes.c_size_t(); nv = ctypes.c_size_t()
            L.a5o_table_get(self.h, e, ctypes.byref(kp), ctypes.byref(kn), ctypes.byref(nv))
            key = ctypes.string_at(kp, kn.value)
            vals = []
            for v in range(nv.value):
                vp = _u8p(); vn = ctypes.c_size_t()
                L.a5o_table_get_val(self.h, e, v, ctypes.byref(vp), ctypes.byref(vn))
                vals.append(ctypes.string_at(vp, vn.value))
            out[key] = vals
        return out

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.a5o_table_free(self.h)
            self.h = None

    def expand_word(self, word: bytes, mode: int, mn: int, mx: int) -> List[bytes]:
        out: List[bytes] = []

        def cb(_u, p, n):
            out.append(ctypes.string_at(p, n))

        rc = lib().a5o_expand_word(self.h, word, len(word), mode, mn, mx, EMIT(cb), None)
        if rc:
            raise RuntimeError(f"oracle expand rc={rc}")
        return out

    def expand_batch(self, words: np.ndarray, offs: np.ndarray, mode: int, mn: int, mx: int) -> Tuple[bytes, np.ndarray]:
        nw = len(offs) - 1
        wb = np.zeros(nw, dtype=np.uint64)
        need = lib().a5o_expand_batch(self.h, words.ctypes.data, offs.ctypes.data, nw, mode, mn, mx, None, 0,
                                      wb.ctypes.data)
        if need < 0:
            raise RuntimeError(f"oracle expand rc={need}")
        out = np.zeros(max(int(need), 1), dtype=np.uint8)
        got = lib().a5o_expand_batch(self.h, words.ctypes.data, offs.ctypes.data, nw, mode, mn, mx, out.ctypes.data,
                                     out.size, wb.ctypes.data)
        assert got == need
        return out[:need].tobytes(), wb

    def digest_batch(self, words: np.ndarray, offs: np.ndarray, mode: int, mn: int, mx: int,
                     nthreads: Optional[int] = None) -> np.ndarray:
        nw = len(offs) - 1
        out = np.zeros((nw, 4), dtype=np.uint64)
        rc = lib().a5o_digest_batch(self.h, words.ctypes.data, offs.ctypes.data, nw, mode, mn, mx, out.ctypes.data,
                                    nthreads or os.cpu_count() or 1)
        if rc:
            raise RuntimeError(f"oracle digest rc={rc}")
        return out

    def run_pipeline(self, words: np.ndarray, offs: np.ndarray, mode: int, mn: int, mx: int, nthreads: int,
                     fd: int) -> Tuple[int, int]:
        c = ctypes.c_uint64(); b = ctypes.c_uint64()
        rc = lib().a5o_run_pipeline(self.h, words.ctypes.data, offs.ctypes.data, len(offs) - 1, mode, mn, mx,
                                    nthreads, fd, ctypes.byref(c), ctypes.byref(b))
        if rc:
            raise RuntimeError(f"oracle pipeline rc={rc}")
        return c.value, b.value


    def digest_run(self, words: np.ndarray, offs: np.ndarray, mode: int, mn: int, mx: int, algo: int,
                   targets: np.ndarray, nthreads: int) -> Tuple[int, int]:
        """The reference expansion with every candidate digested (algo 0 MD5, 1 NTLM) and probed
        in the set of 16-B targets (n, 16) u8 by nthreads workers; returns (candidates, hits)."""
        t = np.ascontiguousarray(targets, dtype=np.uint8).reshape(-1, 16)
        c = ctypes.c_uint64(); h = ctypes.c_uint64()
        rc = lib().a5o_digest_run(self.h, words.ctypes.data, offs.ctypes.data, len(offs) - 1, mode, mn, mx, algo,
                                  t.ctypes.data, len(t), nthreads, ctypes.byref(c), ctypes.byref(h))
        if rc:
            raise RuntimeError(f"oracle digest run rc={rc}")
        return c.value, h.value


def digest(algo: int, b: bytes) -> bytes:
    """MD5 (algo 0) or NTLM (algo 1, MD4 of Go's UTF-16LE) in C (oracle/a5_oracle.c)."""
    out = ctypes.create_string_buffer(16)
    if lib().a5o_digest(algo, b, len(b), out):
        raise ValueError(algo)
    return out.raw


def cand_hash(b: bytes) -> int:
    return lib().a5o_cand_hash(b, len(b))


def pack_words(words: Sequence[bytes]) -> Tuple[np.ndarray, np.ndarray]:
    offs = np.zeros(len(words) + 1, dtype=np.uint64)
    if words:
        offs[1:] = np.cumsum([len(w) for w in words], dtype=np.uint64)
    data = np.frombuffer(b"".join(words) + b"\0", dtype=np.uint8).copy()
    return data, offs
