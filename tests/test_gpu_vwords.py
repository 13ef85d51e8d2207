"""-s / -s -r virtual words (k_keyspace_vsub, k_vwords_fill) against the oracle.

processWordSubstituteAll / ...Reverse (/root/reference/main.go:308-440) give every
occurrence of a pattern the same value (strings.ReplaceAll), so a word with a repeated
pattern has tied digits.  The engine splits such a word into FAST sub-words, one per
choice of its tied patterns, and k_expand_fast expands them from the virtual word list.
Checked here, through the C ABI: per-word multisets, counts and bytes vs the oracle
(tables with 1-3 values per key, size windows that keep or refuse the split), a word's
candidate order independent of its batch, byte-exact candidate sub-ranges (locate inside
sub-words), fused MD5 hits regenerating their plains, and that the split is taken.
"""
import binascii
import hashlib
import os

import numpy as np
import pytest

from conftest import table_path

pytestmark = pytest.mark.gpu

LETTERS = "αβγδεζηθικλμνξοπρστυφχψω"


def _table():
    # single-codepoint keys with 1-3 valid UTF-8 values that contain no key (positional)
    sub = {}
    for i, k in enumerate("αβγδεζηθ"):
        vals = [chr(0x5D0 + i), "x" * (1 + i % 3), chr(0x410 + i) + "7"][: 1 + i % 3]
        sub[k.encode()] = [v.encode() for v in vals]
    return sub


def _words(rng, n, alpha="αβγδεζηθικλμ"):
    out = []
    for _ in range(n):
        k = int(rng.integers(1, 10))
        out.append("".join(alpha[int(x)] for x in rng.integers(0, len(alpha), size=k)).encode())
    return out


@pytest.fixture(scope="module")
def vtab(tmp_path_factory):
    p = tmp_path_factory.mktemp("vw") / "multi.table"
    with open(p, "wb") as f:
        for k, vs in _table().items():
            for v in vs:
                f.write(k + b"=" + v + b"\n")
    return str(p)


def _oracle(tpath, words, mode, mn, mx):
    from oracle import c_oracle as co
    t = co.CTable([tpath])
    data, offs = co.pack_words(words)
    out, wb = t.expand_batch(data, offs, mode, mn, mx)
    res, pos = [], 0
    for b in wb:
        seg = out[pos:pos + int(b)]
        pos += int(b)
        res.append(sorted(seg.split(b"\n")[:-1]) if seg else [])
    return res


@pytest.mark.parametrize("mode", [2, 3])
@pytest.mark.parametrize("mn,mx", [(0, 15), (1, 15), (1, 2), (0, 3), (-1, 8)])
def test_virtual_words_vs_oracle(vtab, mode, mn, mx):
    """Random Greek words (repeated letters: tied patterns) x a 1-3-value table."""
    from hashcat_a5_table_generator_amd import Context, pack_words
    rng = np.random.default_rng(100 * mode + mn * 7 + mx)
    words = _words(rng, 1500) + ["ααα".encode(), "αβαβαβ".encode(), "γγδδεε".encode(), "ζηθζηθ".encode()]
    want = _oracle(vtab, words, mode, mn, mx)
    with Context(0) as c:
        c.load_tables([vtab])
        cnt, byt = c.keyspace(*pack_words(words), mode, mn, mx)
        got = c.expand_words(words, mode, mn, mx)
    for w, k, b, g, e in zip(words, cnt, byt, got, want):
        assert sorted(g) == e, (mode, mn, mx, w.decode(), len(g), len(e))
        assert int(k) == len(e) and int(b) == sum(len(x) + 1 for x in e), (mode, mn, mx, w.decode())


@pytest.mark.parametrize("mode,mn", [(2, 0), (3, 1), (2, 1)])
def test_virtual_order_independent_of_batch(mode, mn):
    """C5 words (greek-hebrew): every word's ordered candidates equal its list in a
    16-word batch; and the split is taken (the mode engine alone, A5X_NO_VSUB, numbers
    some repeated-pattern word differently; same multisets)."""
    from hashcat_a5_table_generator_amd import Context, synth
    _, (data, offs) = synth.global_words("c5", 0, 4000, seed=0x71 + mode)
    words = [bytes(data[int(offs[i]):int(offs[i + 1])]) for i in range(len(offs) - 1)]
    with Context(0) as c:
        c.load_tables([table_path("greek-hebrew")])
        big = c.expand_words(words, mode, mn, 15)
        small = []
        for i in range(0, len(words), 16):
            small += c.expand_words(words[i:i + 16], mode, mn, 15)
    os.environ["A5X_NO_VSUB"] = "1"
    try:
        with Context(0) as c:
            c.load_tables([table_path("greek-hebrew")])
            plain = c.expand_words(words, mode, mn, 15)
    finally:
        os.environ.pop("A5X_NO_VSUB")
    differ = 0
    for i, (w, b, s, p) in enumerate(zip(words, big, small, plain)):
        assert b == s, (mode, i, w.decode(), "candidate order differs between batches")
        assert sorted(b) == sorted(p), (mode, i, w.decode())
        differ += b != p
    assert differ > 0, "no word took the virtual split"


@pytest.mark.parametrize("mode", [2, 3])
def test_virtual_ranges_concatenate(gpu_ctx, vtab, mode):
    """a5x_expand_device over random candidate sub-ranges == the full expansion, byte
    for byte (range starts inside sub-words: k_mode_locate's virtual branch)."""
    from hashcat_a5_table_generator_amd import DeviceBuffer, pack_words
    gpu_ctx.clear_table()
    gpu_ctx.load_tables([vtab])
    rng = np.random.default_rng(40 + mode)
    words = _words(rng, 3000)
    data, offs = pack_words(words)
    dw = DeviceBuffer.from_array(gpu_ctx, data)
    do = DeviceBuffer.from_array(gpu_ctx, offs)
    tc, tb = gpu_ctx.keyspace_device(dw.ptr, do.ptr, len(words), mode=mode)
    full = DeviceBuffer(gpu_ctx, tb)
    st = gpu_ctx.expand_device(dw.ptr, do.ptr, len(words), full.ptr, tb, mode=mode)
    assert st["candidates"] == tc and st["bytes"] == tb
    ref = full.to_array()
    cuts = sorted(set([0, tc] + [int(x) for x in rng.integers(0, tc, size=11)]))
    parts = []
    for a, b in zip(cuts[:-1], cuts[1:]):
        buf = DeviceBuffer(gpu_ctx, tb)
        st = gpu_ctx.expand_device(dw.ptr, do.ptr, len(words), buf.ptr, tb, mode=mode, cand_begin=a, cand_end=b)
        assert st["candidates"] == b - a
        parts.append(buf.to_array(count=st["bytes"]))
    assert np.array_equal(np.concatenate(parts), ref)
    want = _oracle(vtab, words, mode, 0, 15)
    assert sorted(bytes(ref).split(b"\n")[:-1]) == sorted(x for ws in want for x in ws)


@pytest.mark.parametrize("mode,mn", [(2, 0), (3, 1)])
def test_virtual_fused_md5_hits(vtab, mode, mn):
    """Fused MD5 over a batch with virtual words, every candidate of a third of the words
    a target: each hit (word, candidate) names the candidate whose MD5 it reports, every
    target is found, and a5x_format_hits regenerates the plains."""
    from hashcat_a5_table_generator_amd import Context, pack_words
    rng = np.random.default_rng(90 + mode)
    words = _words(rng, 1200)
    with Context(0) as ctx:
        ctx.load_tables([vtab])
        per_word = ctx.expand_words(words, mode, mn, 15)
        want = set()
        for w in range(0, len(words), 3):
            for i, cnd in enumerate(per_word[w]):
                want.add((w, i))
        ctx.set_targets(0, b"".join({hashlib.md5(per_word[w][i]).digest() for w, i in want}))
        d, o = pack_words(words)
        hits, _ = ctx.expand_digest(d, o, mode, mn, 15, hit_cap=1 << 20)
        for w, cidx, dg in hits:
            assert hashlib.md5(per_word[w][cidx]).digest() == dg, (mode, w, cidx)
        got = {(w, cidx) for w, cidx, _ in hits}
        assert want <= got
        text = ctx.format_hits(d, o, hits[:500], mode, mn, 15)
    for line in text.split(b"\n")[:-1]:
        hx, plain = line.split(b":", 1)
        if plain.startswith(b"$HEX[") and plain.endswith(b"]"):
            plain = binascii.unhexlify(plain[5:-1])
        assert hashlib.md5(plain).hexdigest().encode() == hx, line


@pytest.mark.parametrize("mode,mn", [(2, 0), (2, 1), (3, 0), (3, 1)])
def test_virtual_one_byte_ties(tmp_path, mode, mn):
    """One-byte keys with one-byte values (every sub-word shares one layout: one build
    writes all sub-word records, patching the tied bytes), words whose pieces hold many
    tied occurrences (runs of one letter) -- against the C oracle."""
    from hashcat_a5_table_generator_amd import Context
    p = tmp_path / "ascii.table"
    p.write_bytes(b"a=@\na=4\ns=$\ne=3\no=0\ni=!\nt=7\n")
    rng = np.random.default_rng(7 + mode + 10 * mn)
    alpha = "aseoitxyz"
    words = ["".join(alpha[int(x)] for x in rng.integers(0, len(alpha), size=int(rng.integers(1, 20)))).encode()
             for _ in range(1500)]
    words += [b"a" * n for n in range(1, 30)] + [b"sassafras", b"essentials", b"tattoo", b"aaaaeeeeoooo"]
    want = _oracle(str(p), words, mode, mn, 15)
    with Context(0) as c:
        c.load_tables([str(p)])
        got = c.expand_words(words, mode, mn, 15)
    for w, g, e in zip(words, got, want):
        assert sorted(g) == e, (mode, mn, w, len(g), len(e))


@pytest.mark.parametrize("mode,mn", [(2, 0), (3, 1)])
def test_virtual_fused_ntlm_every_candidate(mode, mn):
    """Fused NTLM over C5-shaped words (virtual words in k_expand_fast_ntlm: Go's UTF-16LE of
    sub-word entries, hits mapped back to (word, index)), every candidate a target: each
    reported once with the RFC 1320 MD4 of its UTF-16LE (oracle/digest_oracle.py)."""
    from hashcat_a5_table_generator_amd import Context, pack_words
    from oracle import digest_oracle as dg
    rng = np.random.default_rng(120 + mode)
    words = [("".join(LETTERS[int(x)] for x in rng.integers(0, 12, size=int(rng.integers(3, 10))))).encode()
             for _ in range(800)]
    with Context(0) as ctx:
        ctx.load_tables([table_path("greek-hebrew")])
        per_word = ctx.expand_words(words, mode, mn, 15)
        want = {}
        for w, cs in enumerate(per_word):
            for i, c in enumerate(cs):
                want.setdefault(dg.ntlm(c), set()).add((w, i))
        ctx.set_targets(1, b"".join(want))
        hits, _ = ctx.expand_digest(*pack_words(words), mode, mn, 15, hit_cap=1 << 20)
    got = {}
    for w, c, d in hits:
        assert dg.ntlm(per_word[w][c]) == d, (mode, w, c)
        got.setdefault(d, set()).add((w, c))
    assert sum(len(v) for v in got.values()) == len(hits)
    assert got == want


@pytest.mark.parametrize("mode,mn", [(2, 0), (2, 1), (3, 0), (3, 1)])
def test_virtual_fixed_width_long_words(tmp_path, mode, mn):
    """Fixed-width words (every key and value of a word the same length: k_keyspace_vsub's
    descriptor, records written by k_vwords_fill without the planner) up to 64 bytes, with up
    to four tied patterns, units of 2 and 3 choices (one or two per piece), literal runs cut at
    7 bytes and tied occurrences straddling pieces; 1- and 2-byte keys -- against the C oracle,
    counts and bytes included, and each word's order equal to its order in a 16-word batch."""
    from hashcat_a5_table_generator_amd import Context, pack_words
    p = tmp_path / "fixed.table"
    p.write_bytes("a=4\na=@\ns=$\ne=3\no=0\nt=7\nt=+\nα=ש\nβ=נ\nγ=ע\nγ=ק\n".encode())
    rng = np.random.default_rng(300 + 10 * mode + mn)
    alpha = ["a", "s", "e", "o", "t", "x", "y", "α", "β", "γ", "z"]
    words = []
    for _ in range(1200):
        w = ""
        target = int(rng.integers(8, 65))
        while len(w.encode()) < target:
            w += alpha[int(rng.integers(0, len(alpha)))]
        while len(w.encode()) > 64:
            w = w[:-1]
        words.append(w.encode())
    words += [("xyzxyzx" * 9)[:n].encode() + b"aa" for n in range(5, 62, 7)]
    words += ["αxxxxxxβxxxxxxαxxxxxxβ".encode(), "γγγγ".encode(), ("aseot" * 12).encode()]
    want = _oracle(str(p), words, mode, mn, 15)
    with Context(0) as c:
        c.load_tables([str(p)])
        cnt, byt = c.keyspace(*pack_words(words), mode, mn, 15)
        got = c.expand_words(words, mode, mn, 15)
        small = []
        for i in range(0, len(words), 16):
            small += c.expand_words(words[i:i + 16], mode, mn, 15)
    for w, k, b, g, s, e in zip(words, cnt, byt, got, small, want):
        assert sorted(g) == e, (mode, mn, w.decode(), len(g), len(e))
        assert int(k) == len(e) and int(b) == sum(len(x) + 1 for x in e), (mode, mn, w.decode())
        assert g == s, (mode, mn, w.decode(), "candidate order differs between batches")
