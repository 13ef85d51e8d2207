"""ctypes binding of liba5x.so (include/a5x.h).

The product path has no CPU fallback: if the in-tree HIP library is missing or a
GPU is absent, calls raise :class:`A5xError` instead of computing anything on
the host.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("A5X_LIB_PATH") or os.path.join(_PKG, "_build", "liba5x.so")

A5X_OK = 0
ERRORS = {
    -1: "A5X_E_ARG", -2: "A5X_E_HIP", -3: "A5X_E_NOMEM", -4: "A5X_E_IO", -5: "A5X_E_TOOLONG",
    -6: "A5X_E_BOUNDS", -7: "A5X_E_OVERFLOW", -8: "A5X_E_CAPACITY", -9: "A5X_E_UNSUPPORTED",
    -10: "A5X_E_NOTABLE", -11: "A5X_E_SINK",
}
E_CAPACITY = -8

# the exported symbols of include/a5x.h (checked by tests/test_abi.py)
EXPORTS = (
    "a5x_abi_version", "a5x_create", "a5x_create_error", "a5x_destroy", "a5x_last_error", "a5x_device_info",
    "a5x_load_table_file", "a5x_parse_table", "a5x_set_table", "a5x_clear_table", "a5x_table_export",
    "a5x_split_words", "a5x_keyspace", "a5x_expand", "a5x_expand_range", "a5x_expand_device", "a5x_keyspace_device",
    "a5x_digest_device", "a5x_partition", "a5x_dev_alloc", "a5x_dev_free", "a5x_memcpy_h2d",
    "a5x_memcpy_d2h", "a5x_synchronize", "a5x_debug_stamps", "a5x_debug_plan_word",
    "a5x_set_targets", "a5x_expand_digest", "a5x_expand_digest_device", "a5x_expand_digest_range_device",
    "a5x_digest_lines_device",
    "a5x_format_plain", "a5x_format_hits", "a5x_locate_device", "a5x_split_device",
    "a5x_stream_reserve",
)


class A5xError(RuntimeError):
    def __init__(self, code: int, msg: str = ""):
        self.code = code
        super().__init__(f"{ERRORS.get(code, code)}: {msg}" if msg else str(ERRORS.get(code, code)))


class Stats(ctypes.Structure):
    _fields_ = [
        ("candidates", ctypes.c_uint64), ("bytes", ctypes.c_uint64), ("words", ctypes.c_uint64),
        ("words_pass_b", ctypes.c_uint64), ("ms_keyspace", ctypes.c_double), ("ms_expand", ctypes.c_double),
        ("ms_total", ctypes.c_double), ("expand_launches", ctypes.c_uint32), ("words_slow", ctypes.c_uint32),
    ]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_ if k != "pad"}


class Hit(ctypes.Structure):
    """a5x_hit: word index, candidate index inside the word, digest."""
    _fields_ = [("word", ctypes.c_uint64), ("cand", ctypes.c_uint64), ("digest", ctypes.c_uint8 * 16)]


SINK = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint8), ctypes.c_size_t)

_lib: Optional[ctypes.CDLL] = None


def load(path: Optional[str] = None) -> ctypes.CDLL:
    """Load liba5x.so (building it first if hipcc is available and it is missing)."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or LIB_PATH
    if not os.path.exists(path):
        try:
            from . import build as _b
            _b.build()
        except Exception as e:  # pragma: no cover - depends on toolchain
            raise A5xError(-2, f"liba5x.so missing at {path} and build failed: {e}") from e
    L = ctypes.CDLL(path)
    vp, u64, u32, sz = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_size_t
    i = ctypes.c_int
    L.a5x_abi_version.restype = i
    L.a5x_create.argtypes = [i, ctypes.POINTER(vp)]
    L.a5x_create_error.argtypes = []
    L.a5x_create_error.restype = ctypes.c_char_p
    L.a5x_destroy.argtypes = [vp]
    L.a5x_destroy.restype = None
    L.a5x_last_error.argtypes = [vp]
    L.a5x_last_error.restype = ctypes.c_char_p
    L.a5x_device_info.argtypes = [vp, ctypes.c_char_p, sz, ctypes.POINTER(i)]
    L.a5x_load_table_file.argtypes = [vp, ctypes.c_char_p]
    L.a5x_parse_table.argtypes = [vp, ctypes.c_char_p, sz]
    L.a5x_set_table.argtypes = [vp, vp, vp, u32, vp, vp, vp, u32]
    L.a5x_clear_table.argtypes = [vp]
    L.a5x_table_export.argtypes = [vp, ctypes.POINTER(u32), ctypes.POINTER(u32), ctypes.POINTER(u64),
                                   ctypes.POINTER(u64), vp, vp, vp, vp, vp]
    L.a5x_split_words.argtypes = [vp, sz, vp, vp, u64, ctypes.POINTER(u64)]
    L.a5x_keyspace.argtypes = [vp, vp, vp, u64, i, i, i, vp, vp]
    L.a5x_expand.argtypes = [vp, vp, vp, u64, i, i, i, SINK, vp, ctypes.POINTER(Stats)]
    L.a5x_expand_range.argtypes = [vp, vp, vp, u64, i, i, i, u64, u64, SINK, vp, ctypes.POINTER(Stats)]
    L.a5x_expand_device.argtypes = [vp, vp, vp, u64, i, i, i, u64, u64, vp, u64, vp, vp, ctypes.POINTER(Stats), vp]
    L.a5x_keyspace_device.argtypes = [vp, vp, vp, u64, i, i, i, vp, vp, ctypes.POINTER(u64),
                                      ctypes.POINTER(u64), vp]
    L.a5x_digest_device.argtypes = [vp, vp, vp, u64, u64, vp, vp]
    L.a5x_partition.argtypes = [vp, u64, u32, vp]
    L.a5x_dev_alloc.argtypes = [vp, ctypes.POINTER(vp), sz]
    L.a5x_dev_free.argtypes = [vp, vp]
    L.a5x_memcpy_h2d.argtypes = [vp, vp, vp, sz]
    L.a5x_memcpy_d2h.argtypes = [vp, vp, vp, sz]
    L.a5x_synchronize.argtypes = [vp]
    L.a5x_debug_stamps.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), i]
    L.a5x_debug_plan_word.argtypes = [vp, vp, sz, i, i, vp, sz, vp]
    L.a5x_set_targets.argtypes = [vp, i, vp, u64]
    L.a5x_expand_digest.argtypes = [vp, vp, vp, u64, i, i, i, vp, u64, ctypes.POINTER(u64), ctypes.POINTER(Stats)]
    L.a5x_expand_digest_device.argtypes = [vp, vp, vp, u64, i, i, i, u64, vp, u64, ctypes.POINTER(u64),
                                           ctypes.POINTER(Stats), vp]
    L.a5x_expand_digest_range_device.argtypes = [vp, vp, vp, u64, i, i, i, u64, u64, u64, vp, u64, ctypes.POINTER(u64),
                                                 ctypes.POINTER(Stats), vp]
    L.a5x_digest_lines_device.argtypes = [vp, i, vp, u64, vp, u64, ctypes.POINTER(u64), vp]
    L.a5x_format_plain.argtypes = [ctypes.c_char_p, sz, vp, sz, ctypes.POINTER(sz)]
    L.a5x_format_hits.argtypes = [vp, vp, vp, u64, i, i, i, vp, u64, SINK, vp]
    L.a5x_locate_device.argtypes = [vp, vp, vp, u64, i, i, i, vp, u64, vp, vp]
    L.a5x_stream_reserve.argtypes = [vp, u64, u64]
    L.a5x_split_device.argtypes = [vp, vp, vp, u64, i, i, i, vp, u32, vp, vp, vp, vp]
    _lib = L
    return L


def check(rc: int, ctx=None) -> None:
    if rc != A5X_OK:
        msg = ""
        if ctx:
            m = load().a5x_last_error(ctx)
            msg = m.decode(errors="replace") if m else ""
        raise A5xError(rc, msg)
