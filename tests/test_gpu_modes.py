"""GPU parity of the -r / -s / -s -r engines (a5x_modes.hip) through the C ABI.

Reference engines: processWordReverse (/root/reference/main.go:208-305),
processWordSubstituteAll (main.go:308-365), processWordSubstituteAllReverse
(main.go:369-440).  The oracle applies a leaf's patterns in sorted order (one of
the Go map orders; the only result for confluent words), and so does the device,
so per-word multisets must be identical.  Golden vectors: tests/golden/golden.json.
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
MODES = (1, 2, 3)


def _sha(cands):
    return hashlib.sha256(b"".join(sorted(c + b"\n" for c in cands))).hexdigest()


def _rw(rng, alpha, n):
    return np.asarray(rng.choice(alpha, size=int(n)), dtype=np.uint8).tobytes()


def _ctx(tables, mseg=None):
    from hashcat_a5_table_generator_amd import Context
    if mseg is not None:
        os.environ["A5X_MSEG"] = str(mseg)
    try:
        c = Context(0)
    finally:
        os.environ.pop("A5X_MSEG", None)
    c.load_tables([table_path(t) for t in tables])
    return c


def _c_oracle(tabs, words, mode, mn, mx):
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


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("mseg", [None, 7])
def test_golden_modes(mode, mseg):
    """Every golden -r / -s / -s -r case: count, bytes and sorted-stream sha256."""
    with open(GOLDEN) as f:
        cases = json.load(f)["cases"]
    groups = defaultdict(list)
    for x in cases:
        if x["mode"] == mode and x["error"] is None:
            groups[(tuple(x["tables"]), x["min"], x["max"])].append(x)
    from hashcat_a5_table_generator_amd import pack_words
    n = 0
    for (tabs, mn, mx), cs in sorted(groups.items()):
        c = _ctx(tabs, mseg)
        words = [bytes.fromhex(x["word"]) for x in cs]
        cnt, byt = c.keyspace(*pack_words(words), mode, mn, mx)
        res = c.expand_words(words, mode, mn, mx)
        for x, k, b, cands in zip(cs, cnt, byt, res):
            w = bytes.fromhex(x["word"])
            assert int(k) == x["count"] and int(b) == x["bytes"], (tabs, mode, mn, mx, w)
            assert len(cands) == x["count"], (tabs, mode, mn, mx, w)
            assert _sha(cands) == x["sha256"], (tabs, mode, mn, mx, w)
            n += 1
        c.close()
    assert n > 1000


@pytest.mark.parametrize("tabs", [["czech", "german"], ["qwerty-cyrillic"], ["qwerty-azerty"],
                                  ["greek-hebrew"], ["qwerty-greek"]])
@pytest.mark.parametrize("mode", MODES)
def test_random_words_modes_vs_c_oracle(tabs, mode):
    rng = np.random.default_rng(zlib.crc32((",".join(tabs) + str(mode)).encode()))
    alpha = list(b"abcdefghijklmnopqrstuvwxyzAEOUSZ;,.'`-=")
    alpha += list("αβγδεζηθικλμνξοπρστυφχψω".encode())
    words = [_rw(rng, alpha, rng.integers(0, 12)) for _ in range(600)]
    words += [b"", b"s", b"ss", b"sss", b"strasse", b"aqua", b"m,;1"]
    c = _ctx(tabs, 13)
    for mn, mx in [(0, 15), (2, 3), (1, 2), (0, 0)]:
        if mode == 1 and tabs == ["qwerty-azerty"]:
            # azerty has 2-byte keys with 1-byte values: -r panics on some words
            words_m = [w for w in words if _c_ok(tabs, w, mode, mn, mx)]
        else:
            words_m = words
        got = [sorted(x) for x in c.expand_words(words_m, mode, mn, mx)]
        want = _c_oracle(tabs, words_m, mode, mn, mx)
        for w, g, e in zip(words_m, got, want):
            assert g == e, (tabs, mode, w, mn, mx, len(g), len(e))
    c.close()


def _c_ok(tabs, w, mode, mn, mx):
    from oracle import c_oracle as co
    try:
        co.CTable([table_path(x) for x in tabs]).expand_word(w, mode, mn, mx)
        return True
    except Exception:
        return False


def test_reverse_panic_is_reported():
    """'1é' under qwerty-azerty: the -r running offset goes negative -> Go slice panic (main.go:255)."""
    from hashcat_a5_table_generator_amd import A5xError, pack_words
    c = _ctx(["qwerty-azerty"])
    data, offs = pack_words(["1é".encode()])
    with pytest.raises(A5xError) as e:
        c.expand(data, offs, 1, 0, 15)
    assert "BOUNDS" in str(e.value)
    # min < 0 with -r: generateCombinations(n, -1) never terminates (main.go:263-281)
    data, offs = pack_words([b"abc"])
    with pytest.raises(A5xError) as e:
        c.keyspace(data, offs, 1, -1, 15)
    assert "BOUNDS" in str(e.value)
    c.close()


def test_empty_key_and_multi_value_suball():
    """An empty key matches before every rune and at the end under -s (strings.ReplaceAll)."""
    from oracle import a5_oracle as o
    from hashcat_a5_table_generator_amd import A5xError, Context
    sub = {b"": [b"-", b"+"], b"a": [b"b", b"ab"], b"b": [b"a"], "é".encode(): [b"e"]}
    words = [b"abc", b"", b"a\xc3\xa9\xff", b"\xe2\x82", b"ba", b"bbbb", b"xyz"]
    with Context(0) as c:
        c.set_table(sub)
        for mode in MODES:
            for mn, mx in [(0, 15), (1, 2), (2, 2)]:
                for w in words:  # one word per call: a -r panic fails the whole batch
                    try:
                        want = sorted(o.expand(w, sub, mode, mn, mx))
                    except o.GoPanic:
                        with pytest.raises(A5xError) as e:
                            c.expand_words([w], mode, mn, mx)
                        assert "BOUNDS" in str(e.value), (mode, w, mn, mx)
                        continue
                    assert sorted(c.expand_words([w], mode, mn, mx)[0]) == want, (mode, w, mn, mx)


@pytest.mark.parametrize("mode", MODES)
def test_mode_ranges_concatenate(gpu_ctx, mode):
    """a5x_expand_device over candidate sub-ranges == the full expansion (byte-exact)."""
    from hashcat_a5_table_generator_amd import DeviceBuffer, pack_words
    gpu_ctx.clear_table()
    gpu_ctx.load_tables([table_path("czech"), table_path("german")])
    rng = np.random.default_rng(5 + mode)
    words = [_rw(rng, list(b"abcdefghijklmnopqrstuvwxyzs"), rng.integers(1, 13)) for _ in range(2000)]
    data, offs = pack_words(words)
    dw = DeviceBuffer.from_array(gpu_ctx, data)
    do = DeviceBuffer.from_array(gpu_ctx, offs)
    tc, tb = gpu_ctx.keyspace_device(dw.ptr, do.ptr, len(words), mode=mode)
    full = DeviceBuffer(gpu_ctx, tb)
    st = gpu_ctx.expand_device(dw.ptr, do.ptr, len(words), full.ptr, tb, mode=mode)
    assert st["candidates"] == tc and st["bytes"] == tb
    ref = full.to_array()
    cuts = sorted(set([0, tc] + [int(x) for x in rng.integers(0, tc, size=7)]))
    parts = []
    for a, b in zip(cuts[:-1], cuts[1:]):
        buf = DeviceBuffer(gpu_ctx, tb)
        st = gpu_ctx.expand_device(dw.ptr, do.ptr, len(words), buf.ptr, tb, mode=mode, cand_begin=a, cand_end=b)
        assert st["candidates"] == b - a
        parts.append(buf.to_array(count=st["bytes"]))
    assert np.array_equal(np.concatenate(parts), ref)
    # and the whole stream is the C oracle's, word by word
    want = _c_oracle(["czech", "german"], words, mode, 0, 15)
    lines = bytes(ref).split(b"\n")[:-1]
    assert sorted(lines) == sorted(x for ws in want for x in ws)


def test_reverse_negative_min_window():
    """-r with min < 0: generateCombinations(n, k < 0) recurses forever whenever the
    subCount loop runs (min(max, n) >= min, main.go:238, 263-281) -- the reference dies;
    with max < min the loop never runs and the output is empty."""
    from hashcat_a5_table_generator_amd import A5xError, pack_words
    c = _ctx(["qwerty-azerty"])
    data, offs = pack_words([b"abc", b"qwerty"])
    for mn, mx in [(-3, -2), (-1, 15), (-2, -2)]:
        with pytest.raises(A5xError) as e:
            c.keyspace(data, offs, 1, mn, mx)
        assert "BOUNDS" in str(e.value), (mn, mx)
    cnt, byt = c.keyspace(data, offs, 1, -3, -4)
    assert int(cnt.sum()) == 0 and int(byt.sum()) == 0
    c.close()


@pytest.mark.parametrize("wl,tabs", [("c5", ["greek-hebrew"]), ("c3", ["czech", "german"])])
@pytest.mark.parametrize("mode,mn", [(1, 0), (1, 1), (2, 0), (3, 1)])
def test_mode_hits_regenerate_their_plains(wl, tabs, mode, mn):
    """Every path numbers a word's candidates the same way: hits of the fused -r / -s /
    -s -r digest (FAST-probe words in k_expand_fast_md5, piece-engine and token-ring words
    in the mode kernels) come back through a5x_format_hits -- which regenerates each plain
    from (word, candidate) on the expansion path (locate inside FAST words included) -- as
    plains whose MD5 is the reported digest, every planted (word, candidate) found."""
    import binascii
    from hashcat_a5_table_generator_amd import Context, DeviceBuffer, pack_words, synth
    _, (data, offs) = synth.global_words(wl, 0, 3000, seed=0xE5 + mode)
    words = [bytes(data[int(offs[i]):int(offs[i + 1])]) for i in range(len(offs) - 1)]
    rng = np.random.default_rng(11 + mode)
    with Context(0) as ctx:
        ctx.load_tables([table_path(t) for t in tabs])
        cands = ctx.expand_words(words, mode, mn, 15)
        planted = {}
        for w in rng.choice(len(words), size=200, replace=False):
            if cands[w]:
                c = cands[w][int(rng.integers(0, len(cands[w])))]
                planted[hashlib.md5(c).digest()] = c
        ctx.set_targets(0, b"".join(planted))
        d, o = pack_words(words)
        dw, do = DeviceBuffer.from_array(ctx, d), DeviceBuffer.from_array(ctx, o)
        hits, _ = ctx.expand_digest_device(dw.ptr, do.ptr, len(words), mode, mn, 15, hit_cap=1 << 14)
        text = ctx.format_hits(d, o, hits, mode, mn, 15)
    seen = set()
    for line in text.split(b"\n")[:-1]:
        hx, plain = line.split(b":", 1)
        if plain.startswith(b"$HEX[") and plain.endswith(b"]"):
            plain = binascii.unhexlify(plain[5:-1])
        assert hashlib.md5(plain).hexdigest().encode() == hx, line
        seen.add(bytes.fromhex(hx.decode()))
    assert set(planted) <= seen


@pytest.mark.parametrize("mode,mn", [(1, 0), (2, 0), (3, 1), (2, 1)])
def test_mode_fused_md5_every_candidate(mode, mn):
    """-r / -s / -s -r fused MD5 with EVERY candidate of the batch a target: the mode
    engines' slot layout (one leaf per 48-B or 64-B slot, the 0x80 pad placed after it, the
    block read straight from the ring) and its fallbacks (leaves past a slot: the run
    layout / the contiguous positional ring) must each report every (word, candidate) once
    with the hashlib MD5 of the candidate that index names.  Greek words (C5 shape) with
    2-8 letters, and digit runs with a few letters (leaves of 30-70 bytes) so rounds of both
    kinds occur."""
    from hashcat_a5_table_generator_amd import Context, pack_words
    rng = np.random.default_rng(70 + mode)
    letters = "αβγδεζηθικλμνξοπρστυφχψω"

    def greek(n):
        return "".join(letters[int(x)] for x in rng.integers(0, 24, size=int(n)))

    words = [greek(rng.integers(2, 9)).encode() for _ in range(1200)]
    words += [("7" * int(n) + greek(3)).encode() for n in range(24, 64, 3)]
    with Context(0) as ctx:
        ctx.load_tables([table_path("greek-hebrew")])
        per_word = ctx.expand_words(words, mode, mn, 15)
        want = {}
        for w, cs in enumerate(per_word):
            for i, c in enumerate(cs):
                want.setdefault(hashlib.md5(c).digest(), set()).add((w, i))
        ctx.set_targets(0, b"".join(want))
        hits, _ = ctx.expand_digest(*pack_words(words), mode, mn, 15, hit_cap=1 << 20)
    got = {}
    for w, c, d in hits:
        assert hashlib.md5(per_word[w][c]).digest() == d, (mode, w, c)
        got.setdefault(d, set()).add((w, c))
    assert sum(len(v) for v in got.values()) == len(hits)
    assert got == want
