"""GPU parity of the fused digest + lookup stage (a5x_digest.hip) through the C ABI.

Digests are checked bit-exact against hashlib MD5 (== Go crypto/md5) and the RFC 1320
MD4 restatement of oracle/digest_oracle.py (NTLM) on every candidate of expanded
batches; lookups against planted targets must return exactly the planted
(word, candidate) pairs and nothing else.
"""
import numpy as np
import pytest

from conftest import table_path

pytestmark = pytest.mark.gpu


def _rw(rng, alpha, n):
    return np.asarray(rng.choice(alpha, size=int(n)), dtype=np.uint8).tobytes()


def _words(seed, n, greek=False):
    rng = np.random.default_rng(seed)
    alpha = list("αβγδεζηθικλμνξοπρστυφχψω".encode()) if greek else list(b"abcdefghijklmnopqrstuvwxyzs")
    out = [_rw(rng, alpha, rng.integers(1, 13)) for _ in range(n)]
    return out + [b"", b"a", b"strasse", b"\xff\xfe", "😀ab".encode()]


@pytest.mark.parametrize("algo", [0, 1])
@pytest.mark.parametrize("tabs", [["czech", "german"], ["greek-hebrew"], ["qwerty-cyrillic"]])
def test_digest_every_candidate(gpu_ctx, algo, tabs):
    """a5x_digest_lines_device over an expanded batch == oracle digest of every line."""
    from hashcat_a5_table_generator_amd import DeviceBuffer, pack_words
    from oracle import digest_oracle as dg
    gpu_ctx.clear_table()
    gpu_ctx.load_tables([table_path(t) for t in tabs])
    words = _words(algo * 7 + len(tabs), 1500, greek=tabs == ["greek-hebrew"])
    # MD5 block edges (55/56/63/64/119/120 bytes) with one substitutable letter each
    # (and lines past the 256 B staging margin -- hashed from HBM -- up to a pass-G word)
    words += [b"1" * (n - 1) + b"a" for n in (54, 55, 56, 63, 64, 119, 120, 200, 600, 1500, 3000)]
    data, offs = pack_words(words)
    dw = DeviceBuffer.from_array(gpu_ctx, data)
    do = DeviceBuffer.from_array(gpu_ctx, offs)
    tc, tb = gpu_ctx.keyspace_device(dw.ptr, do.ptr, len(words))
    out = DeviceBuffer(gpu_ctx, tb + 64)
    gpu_ctx.expand_device(dw.ptr, do.ptr, len(words), out.ptr, tb)
    stream = bytes(out.to_array(count=tb))
    lines = stream.split(b"\n")[:-1]
    dig = DeviceBuffer(gpu_ctx, 16 * len(lines) + 16)
    n = gpu_ctx.digest_lines_device(algo, out.ptr, len(stream), dig.ptr, len(lines))
    assert n == len(lines)
    got = dig.to_array(count=16 * n).reshape(n, 16)
    f = dg.ALGOS[algo]
    bad = [i for i, ln in enumerate(lines) if bytes(got[i]) != f(ln)]
    assert not bad, [(lines[i], bytes(got[i]).hex(), f(lines[i]).hex()) for i in bad[:5]]


@pytest.mark.parametrize("algo", [0, 1])
@pytest.mark.parametrize("mode", [0, 2])
def test_lookup_planted_targets(gpu_ctx, algo, mode):
    """Planted digests are found at their (word, candidate) and random digests never hit."""
    from hashcat_a5_table_generator_amd import pack_words
    from oracle import digest_oracle as dg
    gpu_ctx.clear_table()
    gpu_ctx.load_tables([table_path("czech"), table_path("german")])
    words = _words(100 + algo, 800)
    per_word = gpu_ctx.expand_words(words, mode, 0, 15)
    rng = np.random.default_rng(9)
    f = dg.ALGOS[algo]
    planted = {}
    for w in rng.choice(len(words), size=40, replace=False):
        if per_word[w]:
            c = int(rng.integers(0, len(per_word[w])))
            planted[f(per_word[w][c])] = (int(w), c)
    targets = list(planted) + [bytes(rng.integers(0, 256, size=16, dtype=np.uint8)) for _ in range(5000)]
    gpu_ctx.set_targets(algo, b"".join(targets))
    data, offs = pack_words(words)
    hits, st = gpu_ctx.expand_digest(data, offs, mode, 0, 15)
    assert st["candidates"] == sum(len(x) for x in per_word)
    got = {}
    for w, c, d in hits:
        assert f(per_word[w][c]) == d  # the reported candidate really has that digest
        got.setdefault(d, set()).add((w, c))
    for d, (w, c) in planted.items():
        assert (w, c) in got.get(d, set()), (per_word[w][c], d.hex())
    assert set(got) == set(planted)


def test_lookup_small_scratch_ranges(gpu_ctx, monkeypatch):
    """The two-pass range loop (scratch smaller than the batch output) finds the same hits."""
    monkeypatch.setenv("A5X_NO_FUSED_DIGEST", "1")  # (the fused path needs no scratch)
    from hashcat_a5_table_generator_amd import DeviceBuffer, pack_words
    from oracle import digest_oracle as dg
    gpu_ctx.clear_table()
    gpu_ctx.load_tables([table_path("czech"), table_path("german")])
    words = _words(5, 3000)
    per_word = gpu_ctx.expand_words(words, 0, 0, 15)
    pl = [(w, len(per_word[w]) - 1) for w in range(0, len(words), 97) if per_word[w]]
    gpu_ctx.set_targets(0, b"".join(dg.md5(per_word[w][c]) for w, c in pl))
    data, offs = pack_words(words)
    dw = DeviceBuffer.from_array(gpu_ctx, data)
    do = DeviceBuffer.from_array(gpu_ctx, offs)
    hits, st = gpu_ctx.expand_digest_device(dw.ptr, do.ptr, len(words), 0, 0, 15, scratch_bytes=50_000)
    assert st["expand_launches"] > 3
    tg = {dg.md5(per_word[w][c]) for w, c in pl}
    want = sorted((w, c) for w, cs in enumerate(per_word) for c, x in enumerate(cs) if dg.md5(x) in tg)
    assert sorted((w, c) for w, c, _ in hits) == want  # every candidate with a target digest, once


@pytest.mark.parametrize("algo", [0, 1])
def test_digest_long_candidates_cross_block_edges(gpu_ctx, algo):
    """250-300 B candidates (BIG-path words) whose lines straddle the digest stream's
    4 KiB / 2 KiB block edges at many offsets: the line must be hashed from staged bytes
    only (in_lds = e <= sl), bit-exact vs hashlib / RFC 1320 MD4."""
    from hashcat_a5_table_generator_amd import DeviceBuffer, pack_words
    from oracle import digest_oracle as dg
    gpu_ctx.clear_table()
    gpu_ctx.load_tables([table_path("czech")])
    rng = np.random.default_rng(11 + algo)
    # (NTLM streams its UTF-16LE into the MD4 blocks: no length limit, same lines as MD5)
    words = [b"1" * int(rng.integers(250, 300)) + b"a" for _ in range(200)]
    data, offs = pack_words(words)
    dw, do = DeviceBuffer.from_array(gpu_ctx, data), DeviceBuffer.from_array(gpu_ctx, offs)
    tc, tb = gpu_ctx.keyspace_device(dw.ptr, do.ptr, len(words))
    out = DeviceBuffer(gpu_ctx, tb + 64)
    gpu_ctx.expand_device(dw.ptr, do.ptr, len(words), out.ptr, tb)
    lines = bytes(out.to_array(count=tb)).split(b"\n")[:-1]
    assert len(lines) == tc and tb > 3 * (4096 if algo == 0 else 2048)  # several stream blocks
    dig = DeviceBuffer(gpu_ctx, 16 * tc + 16)
    assert gpu_ctx.digest_lines_device(algo, out.ptr, tb, dig.ptr, tc) == tc
    got = dig.to_array(count=16 * tc).reshape(tc, 16)
    f = dg.ALGOS[algo]
    bad = [i for i, ln in enumerate(lines) if bytes(got[i]) != f(ln)]
    assert not bad, [(len(lines[i]), bytes(got[i]).hex()) for i in bad[:5]]


def test_lookup_with_a_full_32_bit_prefilter(gpu_ctx, monkeypatch):
    """A 2^32-bit prefilter (what > 2^26 targets get): the device mask must be
    0xffffffff, not (1 << 32) - 1 = 0.  Forced with the sizing test hook."""
    from hashcat_a5_table_generator_amd import pack_words
    from oracle import digest_oracle as dg
    monkeypatch.setenv("A5X_TARGET_BM_LOG2", "32")
    gpu_ctx.clear_table()
    gpu_ctx.load_tables([table_path("czech"), table_path("german")])
    words = _words(77, 400)
    per_word = gpu_ctx.expand_words(words, 0, 0, 15)
    pl = [(w, len(per_word[w]) // 2) for w in range(0, 400, 13) if per_word[w]]
    gpu_ctx.set_targets(0, b"".join(dg.md5(per_word[w][c]) for w, c in pl))
    hits, _ = gpu_ctx.expand_digest(*pack_words(words), 0, 0, 15)
    got = {(w, c) for w, c, _ in hits}
    assert set(pl) <= got


def test_fused_ntlm_multi_block_candidates(gpu_ctx):
    """Fused NTLM (k_expand_fast_ntlm) on candidates of 20-64 UTF-16 units: MD4 message
    blocks past the first (the 0x80 pad and the bit length in a second / third block),
    2-byte and 4-byte UTF-8 (surrogate pairs) and invalid bytes (U+FFFD), bit-exact vs the
    RFC 1320 restatement over Go's UTF-16LE."""
    from hashcat_a5_table_generator_amd import pack_words
    from oracle import digest_oracle as dg
    gpu_ctx.clear_table()
    gpu_ctx.load_tables([table_path("czech")])
    # FAST words (the fused path needs every candidate-bearing word FAST: <= 8 pieces)
    words = [b"x" * n + b"a" for n in range(19, 48)]                 # 20-48 units: pads in block 1 / 2
    words += [("β" * n + "a").encode() for n in range(10, 24)]       # 2-byte UTF-8
    words += [("😀" * n + "ea").encode() for n in range(5, 12)]      # surrogate pairs, 12-24 units
    words += [b"\xff\xfe" * 10 + b"ae", b"\xce" + b"q" * 30 + b"e"]  # invalid UTF-8 -> U+FFFD
    per_word = gpu_ctx.expand_words(words, 0, 0, 15)
    assert all(per_word)
    targets = {dg.ntlm(c): (w, i) for w, cs in enumerate(per_word) for i, c in enumerate(cs)}
    gpu_ctx.set_targets(1, b"".join(targets))
    hits, st = gpu_ctx.expand_digest(*pack_words(words), 0, 0, 15)
    assert st["ms_total"] - st["ms_keyspace"] - st["ms_expand"] < 1e-3  # the fused path ran
    got = {(w, c) for w, c, _ in hits}
    assert got == {(w, i) for w, cs in enumerate(per_word) for i in range(len(cs))}
    for w, c, d in hits:
        assert dg.ntlm(per_word[w][c]) == d


def test_format_hits_word_past_4gib_of_output(gpu_ctx):
    """a5x_format_hits regenerates only the hit candidates (located, expanded as short
    ranges), so a hit in a word whose output is past 2^32 bytes -- "a" x 32 with a -> b,
    1.85e9 candidates, 61 GB -- still yields its exact plain (the whole-word
    re-expansion truncated its uint32 line offsets and exhausted host memory)."""
    from hashcat_a5_table_generator_amd import DeviceBuffer, pack_words
    from oracle import digest_oracle as dg
    word = b"a" * 32
    plains = [b"b" * 15 + b"a" * 17, b"a" * 31 + b"b", b"ab" * 7 + b"a" * 18]
    gpu_ctx.clear_table()
    gpu_ctx.set_table({b"a": [b"b"]})
    try:
        d, o = pack_words([b"qq", word, b"a"])
        dw, do = DeviceBuffer.from_array(gpu_ctx, d), DeviceBuffer.from_array(gpu_ctx, o)
        tc, tb = gpu_ctx.keyspace_device(dw.ptr, do.ptr, 3)
        assert tb > (1 << 32) and tc == 1846943452 + 1
        gpu_ctx.set_targets(0, b"".join(dg.md5(p) for p in plains))
        hits, _ = gpu_ctx.expand_digest_device(dw.ptr, do.ptr, 3, 0, 0, 15, scratch_bytes=8 << 30)
        assert sorted(w for w, _, _ in hits) == [1, 1, 1]
        lines = gpu_ctx.format_hits(d, o, hits).split(b"\n")[:-1]
        assert sorted(lines) == sorted(dg.md5(p).hex().encode() + b":" + p for p in plains)
    finally:
        gpu_ctx.clear_table()


@pytest.mark.parametrize("algo", [0, 1])
def test_fused_slot_path_every_candidate_mixed_utf8(gpu_ctx, algo):
    """The fused kernels' slot path (one candidate per 64-B message block, '\\n' turned into
    the 0x80 pad; NTLM on big entries pre-converted to UTF-16LE) beside their general path
    (windows with candidates past one block, or with a piece boundary inside a rune: the
    UTF-8 walk): every candidate of every word is a target, so each (word, candidate) must
    come back once with its MD5 / NTLM bit-exact vs the oracle (hashlib, RFC 1320 over Go's
    UTF-16LE).  Words mix ASCII, 2/3/4-byte runes (surrogate pairs), literal runs of 3-byte
    runes (the 7-byte literal pieces cut them) and invalid bytes (U+FFFD)."""
    from hashcat_a5_table_generator_amd import pack_words
    from oracle import digest_oracle as dg
    sub = {b"a": ["€".encode(), b"A"], b"e": ["é".encode(), "😀".encode()], b"o": [b"0", "ö".encode()]}
    gpu_ctx.set_table(sub)
    rng = np.random.default_rng(41 + algo)
    parts = [b"a", b"e", b"o", b"x", b"y", "日".encode(), "😀".encode(), b"\xff", b"\xc3", "é".encode(), "本語".encode()]
    words = [b"".join(parts[int(i)] for i in rng.integers(0, len(parts), size=int(rng.integers(1, 9))))
             for _ in range(1500)]
    words += [("日本語" * 3 + "ae").encode(), b"q" * 40 + b"ao", ("β" * 20 + "eo").encode()]  # long: general path
    per_word = gpu_ctx.expand_words(words, 0, 0, 15)
    f = dg.ALGOS[algo]
    want = {}
    for w, cs in enumerate(per_word):
        for i, c in enumerate(cs):
            want.setdefault(f(c), set()).add((w, i))
    gpu_ctx.set_targets(algo, b"".join(want))
    hits, st = gpu_ctx.expand_digest(*pack_words(words), 0, 0, 15, hit_cap=1 << 18)
    got = {}
    for w, c, d in hits:
        assert f(per_word[w][c]) == d, (algo, w, c, per_word[w][c])
        got.setdefault(d, set()).add((w, c))
    assert sum(len(v) for v in got.values()) == len(hits)  # each (word, candidate) once
    assert got == want


@pytest.mark.parametrize("algo,mode,tabs", [(0, 0, ["czech", "german"]), (1, 0, ["czech", "german"]),
                                            (0, 1, ["greek-hebrew"]), (0, 2, ["greek-hebrew"]),
                                            (1, 3, ["greek-hebrew"])])
def test_digest_ranges_partition_the_hits(gpu_ctx, algo, mode, tabs):
    """a5x_expand_digest_range_device: the batch's
    candidates cut into ranges at arbitrary candidates -- inside FAST words, slow / BIG
    words and mode-engine items -- give exactly the whole batch's hits, each range only
    the hits of its own candidates (every 7th candidate of the batch is a target)."""
    from hashcat_a5_table_generator_amd import DeviceBuffer, pack_words
    from oracle import digest_oracle as dg
    gpu_ctx.clear_table()
    gpu_ctx.load_tables([table_path(t) for t in tabs])
    greek = tabs == ["greek-hebrew"]
    words = _words(31 + algo + 3 * mode, 600, greek=greek)
    if greek:
        words += ["αλφαβητα".encode() * 2, "ααααααααα".encode()]  # repeated patterns (-s virtual words)
    else:
        # cluster words, a 20-letter word past the FAST piece limits (slow path), words
        # longer than 64 B (BIG path); keyspaces of 11..3455 candidates
        words += [b"sassas", b"abcdefghijklmnopqrst", b"q" * 64 + b"abcdes", b"qq" * 40 + b"strasse",
                  b"q" * 100 + b"sss" + b"q" * 30]
    data, offs = pack_words(words)
    cnt, _ = gpu_ctx.keyspace(data, offs, mode, 0, 15)
    coff = np.concatenate([[0], np.cumsum(cnt.astype(np.int64))])
    tc = int(coff[-1])
    per_word = gpu_ctx.expand_words(words, mode, 0, 15)
    f = dg.ALGOS[algo]
    flat = [c for w in per_word for c in w]
    assert len(flat) == tc
    targets = {f(flat[g]) for g in range(0, tc, 7)}
    gpu_ctx.set_targets(algo, b"".join(sorted(targets)) + bytes(range(16)))
    dw = DeviceBuffer.from_array(gpu_ctx, data)
    do = DeviceBuffer.from_array(gpu_ctx, offs)

    def hits(cb=0, ce=None):
        h, st = gpu_ctx.expand_digest_device(dw.ptr, do.ptr, len(words), mode, 0, 15, hit_cap=1 << 18,
                                             cand_begin=cb, cand_end=ce)
        assert st["candidates"] == (tc if ce is None else ce) - cb
        return {(int(w), int(c)) for w, c, _ in h}

    full = hits()
    want = {(w, c) for w, cs in enumerate(per_word) for c, x in enumerate(cs) if f(x) in targets}
    assert full == want
    rng = np.random.default_rng(5 + mode)
    cuts = sorted({0, tc, *(int(x) for x in rng.integers(1, tc, size=5))})
    big = int(np.argmax(cnt))  # also cut inside the largest word
    cuts = sorted(set(cuts) | {int(coff[big]) + int(cnt[big]) // 3})
    union = set()
    for a, b in zip(cuts, cuts[1:]):
        part = hits(a, b)
        assert all(a <= coff[w] + c < b for w, c in part), (a, b)
        assert not (part & union)
        union |= part
    assert union == full
