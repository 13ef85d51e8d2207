"""GPU parity for pass G: dictionary lines beyond the pass-B LDS budget.

The reference reads any line shorter than 64 KiB (bufio.Scanner, /root/reference/
main.go:72-74) and runs processWord (main.go:168-205) on it.  Words longer than
A5X_LMAX_B (2048 B), with candidates longer than the 16 KiB pass-B ring, or with
DP tables beyond pass B are sized and expanded with their WaveLds / ring in HBM
scratch (k_keyspace_g / k_expand_g).  Checked per word against the C oracle
(oracle/a5_oracle.c) and the Python oracle's closed-form keyspace.
"""
import numpy as np
import pytest

from conftest import table_path

pytestmark = pytest.mark.gpu


def _word(rng, L, nmatch, alpha=b"bfghjkmpqvwx0123456789", keys=b"as"):  # no key bytes in alpha
    w = bytearray(np.asarray(rng.choice(list(alpha), size=L), dtype=np.uint8).tobytes())
    for p in rng.choice(L, size=min(nmatch, L), replace=False):
        w[p] = keys[int(rng.integers(0, len(keys)))]
    return bytes(w)


def _ctx(tables, chunk=None):
    import os
    from hashcat_a5_table_generator_amd import Context
    if chunk is not None:
        os.environ["A5X_CHUNK"] = str(chunk)
    try:
        c = Context(0)
    finally:
        os.environ.pop("A5X_CHUNK", None)
    c.load_tables([table_path(t) for t in tables])
    return c


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


def _long_words():
    rng = np.random.default_rng(2049)
    words = [_word(rng, L, k) for L, k in ((2049, 4), (5000, 3), (20000, 4), (65535, 3), (3000, 0))]
    words.append(b"x" * 40000 + b"strasse" + b"w" * 100)      # overlapping keys far into a long line
    words.append(_word(rng, 2100, 2000, keys=b"a"))           # 2000 matches, capped window below
    words.append(b"s" * 2500)                                  # s / ss clusters over 2500 bytes
    return words


@pytest.mark.parametrize("mn,mx", [(0, 15), (0, 1), (2, 2)])
def test_long_lines_vs_c_oracle(mn, mx):
    """Per-word candidate multisets of long lines (pass G) == the C oracle."""
    words = _long_words()
    if (mn, mx) != (0, 1):  # 2000-match / 2500-s words: billions of candidates beyond one substitution
        words = words[:6]
    c = _ctx(["czech", "german"], 4096)
    got = [sorted(x) for x in c.expand_words(words, 0, mn, mx)]
    want = _c_oracle_words(["czech", "german"], words, mn, mx)
    for w, g, e in zip(words, got, want):
        assert len(g) == len(e) and g == e, (len(w), mn, mx, len(g), len(e))
    c.close()


def test_long_lines_keyspace_vs_oracle(gpu_ctx):
    """Closed-form (count, bytes) of pass G words == the oracle's DP (main.go:168-205)."""
    from oracle import a5_oracle as o
    from hashcat_a5_table_generator_amd import pack_words
    gpu_ctx.clear_table()
    gpu_ctx.load_tables([table_path("czech"), table_path("german")])
    sub = o.load_tables([table_path("czech"), table_path("german")])
    words = _long_words()
    data, offs = pack_words(words)
    for mn, mx in [(0, 1), (2, 3), (0, 2)]:
        cnt, byt = gpu_ctx.keyspace(data, offs, 0, mn, mx)
        for w, cc, bb in zip(words, cnt, byt):
            assert (int(cc), int(bb)) == o.keyspace_default(w, sub, mn, mx), (len(w), mn, mx)


def test_pass_g_mixed_batch_ranges(gpu_ctx):
    """Short words around pass G words, expanded in candidate ranges that cut inside the long
    words (k_locate through a scratch slot): the pieces concatenate to the full stream."""
    from hashcat_a5_table_generator_amd import DeviceBuffer, pack_words
    gpu_ctx.clear_table()
    gpu_ctx.load_tables([table_path("czech"), table_path("german")])
    rng = np.random.default_rng(5)
    words = []
    for i in range(400):
        words.append(_word(rng, int(rng.integers(1, 12)), 3, alpha=b"bcdfgklmnprt", keys=b"aeiosu"))
        if i % 97 == 3:
            words.append(_word(rng, int(rng.integers(2100, 9000)), 6))
    data, offs = pack_words(words)
    dw = DeviceBuffer.from_array(gpu_ctx, data)
    do = DeviceBuffer.from_array(gpu_ctx, offs)
    tc, tb = gpu_ctx.keyspace_device(dw.ptr, do.ptr, len(words), 0, 0, 3)
    full = DeviceBuffer(gpu_ctx, tb)
    st = gpu_ctx.expand_device(dw.ptr, do.ptr, len(words), full.ptr, tb, 0, 0, 3)
    assert st["candidates"] == tc and st["bytes"] == tb and st["words_pass_b"] >= 5
    ref = full.to_array()
    want = _c_oracle_words(["czech", "german"], words, 0, 3)
    pos = 0
    lines = bytes(ref).split(b"\n")[:-1]
    assert sorted(lines) == sorted(x for ws in want for x in ws)
    cuts = sorted(set([0, tc] + [int(x) for x in rng.integers(0, tc, size=9)]))
    parts = []
    for a, b in zip(cuts[:-1], cuts[1:]):
        buf = DeviceBuffer(gpu_ctx, tb)
        s2 = gpu_ctx.expand_device(dw.ptr, do.ptr, len(words), buf.ptr, tb, 0, 0, 3, cand_begin=a, cand_end=b)
        parts.append(buf.to_array()[:s2["bytes"]])
        pos += s2["bytes"]
    assert pos == tb
    assert bytes(np.concatenate(parts)) == bytes(ref)


def _c_oracle_words_mode(tabs, words, mode, mn, mx):
    from oracle import c_oracle as co
    t = co.CTable([table_path(x) for x in tabs])
    data, offs = co.pack_words(words)
    out, wb = t.expand_batch(data, offs, mode, mn, mx)
    res, pos = [], 0
    for b in wb:
        seg = out[pos:pos + int(b)]
        pos += int(b)
        res.append(sorted(seg.split(b"\n")[:-1]) if seg else [])
    return res


def _mode_long_words():
    rng = np.random.default_rng(129)
    words = [_word(rng, L, k, keys=b"aesz") for L, k in ((129, 8), (200, 11), (1000, 6), (5000, 4), (65535, 3),
                                                          (3000, 0))]
    words.append(b"x" * 40000 + b"strasse" + b"w" * 100)  # "s" / "ss" patterns far into a long line
    words += [b"strasse", b"abc", b"", b"zebra"]           # short words in the same batch (LDS engines)
    return words


@pytest.mark.parametrize("mode,mn,mx", [(1, 0, 15), (2, 0, 15), (3, 0, 15), (1, 2, 2), (2, 1, 1), (3, 2, 3)])
def test_mode_long_lines_vs_c_oracle(mode, mn, mx):
    """-r / -s / -s -r on lines longer than the LDS engines' 128 B (mode pass G: word state
    and lane buffers in HBM scratch slots) == the C oracle per word, with small items
    (A5X_MSEG=64: a G word spans many items over all slots) and small host ranges (range
    starts located inside G words)."""
    import os
    from hashcat_a5_table_generator_amd import Context
    words = _mode_long_words()
    os.environ["A5X_MSEG"] = "64"
    os.environ["A5X_HOST_CHUNK_BYTES"] = "200000"
    try:
        c = Context(0)
    finally:
        os.environ.pop("A5X_MSEG")
        os.environ.pop("A5X_HOST_CHUNK_BYTES")
    c.load_tables([table_path("czech"), table_path("german")])
    got = [sorted(x) for x in c.expand_words(words, mode, mn, mx)]
    c.close()
    want = _c_oracle_words_mode(["czech", "german"], words, mode, mn, mx)
    assert sum(len(x) for x in want[:7]) > 0
    for w, g, e in zip(words, got, want):
        assert len(g) == len(e) and g == e, (len(w), mode, mn, mx, len(g), len(e))
