"""The FAST piece plan (csrc/a5x_plan.h) against the oracle, on the CPU.

a5x_debug_plan_word runs the same host+device code the kernels run per word:
classify_word (unit scan + keyspace closed form + FAST fields) and plan_word
(pieces/groups/entries), then replays passes 1-2 of k_expand_fast.  Every FAST
word must give the oracle's candidate multiset (oracle/a5_oracle.py process_word,
main.go:168-205); every classified word must give the oracle's count and bytes.
"""
import collections
import ctypes
import random

import numpy as np
import pytest

from conftest import table_path
from oracle import a5_oracle as o

FAST = 1 << 5
DEFER = 1 << 4


class HostCtx:
    def __init__(self, tables=None, table_map=None):
        from hashcat_a5_table_generator_amd import _lib
        self.L = _lib.load()
        self.h = ctypes.c_void_p()
        assert self.L.a5x_create(-1, ctypes.byref(self.h)) == 0
        if tables:
            for t in tables:
                assert self.L.a5x_load_table_file(self.h, table_path(t).encode()) == 0
        else:
            txt = b"".join(k + b"=" + v + b"\n" for k, vs in table_map.items() for v in vs)
            assert self.L.a5x_parse_table(self.h, txt, len(txt)) == 0, self.L.a5x_last_error(self.h)

    def plan(self, word: bytes, mn=0, mx=15, cap=1 << 20):
        """(count, bytes, flags, candidates or None when they exceed cap bytes)"""
        info = np.zeros(4, dtype=np.uint64)
        out = np.zeros(max(cap, 1), dtype=np.uint8)
        wb = np.frombuffer(word + b"\0", dtype=np.uint8)
        rc = self.L.a5x_debug_plan_word(self.h, wb.ctypes.data, len(word), mn, mx, out.ctypes.data, cap,
                                        info.ctypes.data)
        if rc == -8 and int(info[1]) > cap:  # A5X_E_CAPACITY: too many candidates to replay here
            return int(info[0]), int(info[1]), int(info[2]), None
        assert rc == 0, self.L.a5x_last_error(self.h)
        n = int(info[3])
        cands = out[:n].tobytes().split(b"\n")[:-1] if n else []
        return int(info[0]), int(info[1]), int(info[2]), cands

    def close(self):
        self.L.a5x_destroy(self.h)


def check_word(ctx, sub, word, mn=0, mx=15):
    cnt, byt, fl, cands = ctx.plan(word, mn, mx)
    if fl & DEFER:
        return "defer"
    if cands is None:  # large keyspace: counts against the oracle's DP only
        assert (cnt, byt) == o.keyspace_default(word, sub, mn, mx), (word, fl)
        return "big"
    ref = o.process_word(word, sub, mn, mx)
    assert (cnt, byt) == (len(ref), sum(len(x) + 1 for x in ref)), (word, fl)
    if fl & FAST:
        assert collections.Counter(cands) == collections.Counter(ref), (word, fl)
        return "fast"
    return "slow"


@pytest.mark.parametrize("tables", [("czech", "german"), ("qwerty-cyrillic",), ("qwerty-azerty",),
                                    ("qwerty-greek",), ("greek-hebrew",), ("czech",)])
def test_plan_shipped_tables_random_words(tables):
    ctx = HostCtx(tables)
    sub = o.load_tables([table_path(t) for t in tables])
    rng = random.Random(hash(tables) & 0xffff)
    alpha = [k for k in sub if len(k) <= 2] + [b"a", b"b", b"q", b"x", b"1", b" "]
    kinds = collections.Counter()
    for _ in range(400):
        w = b"".join(rng.choice(alpha) for _ in range(rng.randint(0, 12)))
        kinds[check_word(ctx, sub, w)] += 1
    ctx.close()
    assert kinds["fast"] > 0


def test_plan_clusters_czech_german():
    """'ss' words: units s/s/ss overlap -> cluster units with 5+ choices (FAST now)."""
    ctx = HostCtx(("czech", "german"))
    sub = o.load_tables([table_path("czech"), table_path("german")])
    kinds = collections.Counter()
    for w in [b"strasse", b"ss", b"sss", b"ssss", b"masse", b"assa", b"sassafras", b"Strasse", b"kiss", b"ssx"]:
        kinds[check_word(ctx, sub, w)] += 1
    assert kinds["fast"] >= 6
    # 'sss' clusters: 12 choices (s, ss overlap) -> one unit of R = 12 > 8, FAST
    for w in [b"xsssy", b"asssbsssc", b"sssss", b"kissssa"]:
        kinds[check_word(ctx, sub, w)] += 1
    assert check_word(ctx, sub, b"zvasssgkpg") == "fast"
    ctx.close()


def test_plan_random_tables_with_overlaps():
    rng = random.Random(7)
    kinds = collections.Counter()
    for _ in range(150):
        m = {}
        for _ in range(rng.randint(1, 5)):
            k = bytes(rng.choice(b"abs") for _ in range(rng.randint(1, 3)))
            m.setdefault(k, []).append(bytes(rng.choice(b"absxyz") for _ in range(rng.randint(0, 3))))
        ctx = HostCtx(table_map=m)
        for _ in range(12):
            w = bytes(rng.choice(b"abs") for _ in range(rng.randint(0, 10)))
            kinds[check_word(ctx, m, w, rng.choice([0, 0, 1]), rng.choice([15, 15, 3, 8]))] += 1
        ctx.close()
    assert kinds["fast"] > 500 and kinds["defer"] > 0


def test_plan_edge_words():
    ctx = HostCtx(("qwerty-cyrillic",))
    sub = o.load_tables([table_path("qwerty-cyrillic")])
    for w in [b"", b"a", b"q" * 20, b"abcdefghijklmnop", b"xx" * 30, b"a" + b"1" * 50 + b"b", b"1" * 64,
              b"a1b2c3d4e5f6g7h8i9j0", b"z" + b" " * 40]:
        check_word(ctx, sub, w)
    # window caps: max 0 -> nothing; min 2 -> capped (DP)
    assert ctx.plan(b"hello", 0, 0)[0] == 0
    assert ctx.plan(b"hello", 2, 15)[2] & DEFER
    ctx.close()
