"""GPU parity: the HIP expansion path vs the oracle (bit-exact per-word multisets).

Reference engine: processWord, /root/reference/main.go:168-205.  The oracle is
oracle/a5_oracle.py (frozen into tests/golden/golden.json) and its C twin
oracle/a5_oracle.c (liba5oracle.so) for sizes Python cannot reach.
"""
import hashlib
import json
import os
import zlib
from collections import defaultdict

import numpy as np
import pytest

from conftest import ROOT, table_path

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(ROOT, "tests", "golden", "golden.json")


def _rw(rng, alpha, n):
    return np.asarray(rng.choice(alpha, size=int(n)), dtype=np.uint8).tobytes()


def _sha(cands):
    return hashlib.sha256(b"".join(sorted(c + b"\n" for c in cands))).hexdigest()


def _ctx(tables, chunk=None):
    from hashcat_a5_table_generator_amd import Context
    if chunk is not None:
        os.environ["A5X_CHUNK"] = str(chunk)
    try:
        c = Context(0)
    finally:
        os.environ.pop("A5X_CHUNK", None)
    c.load_tables([table_path(t) for t in tables])
    return c


def _golden_groups(mode):
    with open(GOLDEN) as f:
        cases = json.load(f)["cases"]
    groups = defaultdict(list)
    for c in cases:
        if c["mode"] == mode and c["error"] is None:
            groups[(tuple(c["tables"]), c["min"], c["max"])].append(c)
    return groups


@pytest.mark.parametrize("chunk", [None, 64, 100])
def test_golden_default_mode(chunk):
    """Every golden default-mode case: count, bytes and sorted-stream sha256."""
    groups = _golden_groups(0)
    n = 0
    ctxs = {}
    for (tabs, mn, mx), cases in sorted(groups.items()):
        if tabs not in ctxs:
            ctxs[tabs] = _ctx(tabs, chunk)
        c = ctxs[tabs]
        words = [bytes.fromhex(x["word"]) for x in cases]
        res = c.expand_words(words, 0, mn, mx)
        for x, cands in zip(cases, res):
            assert len(cands) == x["count"], (tabs, mn, mx, x["word"])
            assert sum(len(y) + 1 for y in cands) == x["bytes"]
            assert _sha(cands) == x["sha256"], (tabs, mn, mx, bytes.fromhex(x["word"]))
            n += 1
    for c in ctxs.values():
        c.close()
    assert n > 1000


def test_keyspace_matches_oracle_dp(gpu_ctx):
    from oracle import a5_oracle as o
    rng = np.random.default_rng(7)
    for tabs in (["czech", "german"], ["qwerty-cyrillic"], ["qwerty-azerty"], ["greek-hebrew"]):
        gpu_ctx.clear_table()
        gpu_ctx.load_tables([table_path(t) for t in tabs])
        sub = o.load_tables([table_path(t) for t in tabs])
        alpha = list(b"abcdefghijklmnopqrstuvwxyzAEOUZS0123456789;,.'")
        words = [_rw(rng, alpha, rng.integers(0, 40)) for _ in range(300)]
        words += [b"s" * k for k in range(0, 30)] + [b"ss" * k for k in range(1, 12)]
        from hashcat_a5_table_generator_amd import pack_words
        for mn, mx in [(0, 15), (2, 5), (0, 3), (4, 20)]:
            data, offs = pack_words(words)
            cnt, byt = gpu_ctx.keyspace(data, offs, 0, mn, mx)
            for w, c, b in zip(words, cnt, byt):
                assert (int(c), int(b)) == o.keyspace_default(w, sub, mn, mx), (tabs, w, mn, mx)


def _c_oracle_words(tabs, words, mn, mx):
    from oracle import c_oracle as co
    t = co.CTable([table_path(x) for x in tabs])
    data, offs = co.pack_words(words)
    out, wb = t.expand_batch(data, offs, 0, mn, mx)
    res, pos = [], 0
    for b in wb:
        seg = out[pos:pos + int(b)]
        pos += int(b)
        res.append(sorted(seg.split(b"\n")[:-1]) if seg else [])
    return res


@pytest.mark.parametrize("tabs", [["czech", "german"], ["qwerty-cyrillic"], ["qwerty-azerty"],
                                  ["greek-hebrew"], ["qwerty-greek"], ["czech", "czech"]])
def test_random_words_vs_c_oracle(tabs):
    rng = np.random.default_rng(zlib.crc32(",".join(tabs).encode()))
    alpha = list(b"abcdefghijklmnopqrstuvwxyzAEOUSZ0123456789;,.'\"`-=")
    alpha += list("αβγδεζηθικλμνξοπρστυφχψω".encode())
    words = [_rw(rng, alpha, rng.integers(0, 14)) for _ in range(2000)]
    c = _ctx(tabs, 256)
    for mn, mx in [(0, 15), (2, 4), (1, 3)]:
        got = [sorted(x) for x in c.expand_words(words, 0, mn, mx)]
        want = _c_oracle_words(tabs, words, mn, mx)
        for w, g, e in zip(words, got, want):
            assert g == e, (tabs, w, mn, mx, len(g), len(e))
    c.close()


def test_long_words_pass_b():
    """Words longer than pass A's 64-byte budget (k_expand_b) and capped DPs."""
    rng = np.random.default_rng(11)
    words = []
    for L in (65, 80, 127, 300, 1000, 2000):
        w = bytearray(_rw(rng, list(b"bfghjkmpqvwxyz0123456789"), L))
        for p in rng.choice(L, size=min(4, L), replace=False):
            w[p] = ord("a")
        words.append(bytes(w))
    words.append(b"strasse" * 12)  # overlaps, 84 bytes
    words.append(b"a" * 17)         # capped: 17 matches > max 15
    words.append(b"as" * 10)
    c = _ctx(["czech", "german"], 128)
    got = [sorted(x) for x in c.expand_words(words, 0, 0, 3)]
    want = _c_oracle_words(["czech", "german"], words, 0, 3)
    assert got == want
    c.close()


def test_candidate_ranges_concatenate(gpu_ctx):
    """a5x_expand_device over sub-ranges == the full expansion (byte-exact)."""
    from hashcat_a5_table_generator_amd import DeviceBuffer, pack_words
    gpu_ctx.clear_table()
    gpu_ctx.load_tables([table_path("czech"), table_path("german")])
    rng = np.random.default_rng(3)
    words = [_rw(rng, list(b"abcdefghijklmnopqrstuvwxyzs"), rng.integers(1, 13)) for _ in range(3000)]
    data, offs = pack_words(words)
    dw = DeviceBuffer.from_array(gpu_ctx, data)
    do = DeviceBuffer.from_array(gpu_ctx, offs)
    tc, tb = gpu_ctx.keyspace_device(dw.ptr, do.ptr, len(words))
    full = DeviceBuffer(gpu_ctx, tb)
    st = gpu_ctx.expand_device(dw.ptr, do.ptr, len(words), full.ptr, tb)
    assert st["candidates"] == tc and st["bytes"] == tb
    ref = full.to_array()
    cuts = sorted(set([0, tc] + [int(x) for x in rng.integers(0, tc, size=7)]))
    parts = []
    for a, b in zip(cuts[:-1], cuts[1:]):
        buf = DeviceBuffer(gpu_ctx, tb)
        st = gpu_ctx.expand_device(dw.ptr, do.ptr, len(words), buf.ptr, tb, cand_begin=a, cand_end=b)
        assert st["candidates"] == b - a
        parts.append(buf.to_array(count=st["bytes"]))
    assert np.array_equal(np.concatenate(parts), ref)


def test_digest_full_scale_c3_shape(gpu_ctx):
    """C3 shape (czech+german, [a-z] len U[6,12]) at 200k words: GPU digest == C oracle digest."""
    from hashcat_a5_table_generator_amd import DeviceBuffer
    from oracle import c_oracle as co
    from hashcat_a5_table_generator_amd import synth
    gpu_ctx.clear_table()
    gpu_ctx.load_tables([table_path("czech"), table_path("german")])
    data, offs = synth.words_az(200_000, 6, 12, seed=0x5A5)
    dw = DeviceBuffer.from_array(gpu_ctx, data)
    do = DeviceBuffer.from_array(gpu_ctx, offs)
    n = len(offs) - 1
    tc, tb = gpu_ctx.keyspace_device(dw.ptr, do.ptr, n)
    out = DeviceBuffer(gpu_ctx, tb)
    boff = DeviceBuffer(gpu_ctx, (n + 1) * 8)
    gpu_ctx.expand_device(dw.ptr, do.ptr, n, out.ptr, tb, d_byte_off=boff.ptr)
    dig = DeviceBuffer(gpu_ctx, n * 32)
    gpu_ctx.digest_device(out.ptr, boff.ptr, 0, n, dig.ptr)
    got = dig.to_array(np.uint64).reshape(n, 4)
    want = co.CTable([table_path("czech"), table_path("german")]).digest_batch(data, offs, 0, 0, 15)
    bad = np.nonzero((got != want).any(axis=1))[0]
    assert len(bad) == 0, [(bytes(data[int(offs[i]):int(offs[i + 1])]), got[i], want[i]) for i in bad[:5]]


def test_overflow_is_reported(gpu_ctx):
    from hashcat_a5_table_generator_amd import A5xError, pack_words
    gpu_ctx.set_table({b"a": [b"b", b"c", b"d", b"e", b"f", b"g", b"h", b"i"]})
    data, offs = pack_words([b"a" * 60])  # 9^60 candidates
    with pytest.raises(A5xError) as e:
        gpu_ctx.keyspace(data, offs, 0, 0, 60)
    assert "OVERFLOW" in str(e.value)


def test_bad_mode_fails_loudly(gpu_ctx):
    from hashcat_a5_table_generator_amd import A5xError, pack_words
    gpu_ctx.set_table({b"a": [b"b"]})
    data, offs = pack_words([b"abc"])
    with pytest.raises(A5xError):
        gpu_ctx.expand(data, offs, 7, 0, 15)
