"""A word's candidate NUMBERING does not depend on the batch it is in.

The reference emits a word's candidates in a nondeterministic interleaving
(/root/reference/main.go:77-93), so parity is per-word multisets; but this library
also names candidates by (word, index) -- fused-digest hits, a5x_format_hits
regenerating a hit's plain from a sub-batch of the hit words, candidate ranges,
shards.  Those agree only if the index -> candidate map of a word is the same in
every batch.  The engines decide per word between the FAST plan (k_expand_fast
numbering) and the per-word paths; the decisions that used to depend on the word's
neighbours -- a keyspace tile whose record budget (FW_TILE_REC) runs out, a tile
too large to stage in LDS, the complex-word slot cap -- are exercised here by
batches built to hit them, and each word's ordered candidate list is compared with
the same word expanded in a small batch.
"""
import binascii
import hashlib
import os
import tempfile

import numpy as np
import pytest

from conftest import table_path

pytestmark = pytest.mark.gpu

KEYS = "abcdefghijklmnop"


def _table_text():
    # 16 one-byte keys, 3 values each: subs[0] keeps the key length (the -r FAST probe),
    # values are valid UTF-8 holding no key (-s positional words)
    lines = []
    for i, k in enumerate(KEYS):
        lines += [f"{k}={k.upper()}", f"{k}={chr(0xE0 + i)}", f"{k}={i % 10}"]
    return "\n".join(lines) + "\n"


@pytest.fixture(scope="module")
def wide_table():
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "wide.table")
        with open(p, "w", encoding="utf-8") as f:
            f.write(_table_text())
        yield p


def _words(mode, n, seed):
    """Distinct-letter words whose FAST records are ~52 u64 (> the 40 per word a tile
    budgets): 6 four-choice units (default, -s) or 12 two-choice units (-r, -s -r)."""
    rng = np.random.default_rng(seed)
    k = 6 if mode in (0, 2) else 12
    return [bytes(rng.permutation(np.frombuffer(KEYS.encode(), dtype=np.uint8))[:k]) for _ in range(n)]


def _expand_small(ctx, words, mode, mn, mx, per=16):
    out = []
    for i in range(0, len(words), per):
        out += ctx.expand_words(words[i:i + per], mode, mn, mx)
    return out


def _c_oracle_sorted(tpaths, words, mode, mn, mx):
    from oracle import c_oracle as co
    t = co.CTable(tpaths)
    data, offs = co.pack_words(words)
    out, wb = t.expand_batch(data, offs, mode, mn, mx)
    res, pos = [], 0
    for b in wb:
        seg = out[pos:pos + int(b)]
        pos += int(b)
        res.append(sorted(seg.split(b"\n")[:-1]) if seg else [])
    return res


@pytest.mark.parametrize("mode", [0, 1, 2, 3])
def test_order_independent_of_batch(wide_table, mode):
    """300 words with oversize FAST records (the first tile's budget runs out) behind a
    9000-byte word (the first tile cannot be staged): every word's ordered candidate list
    equals its list in a 16-word batch, and the multisets are the C oracle's."""
    from hashcat_a5_table_generator_amd import Context
    words = [b"z" * 9000] + _words(mode, 300, 0xB0 + mode)
    with Context(0) as ctx:
        ctx.load_tables([wide_table])
        big = ctx.expand_words(words, mode, 0, 15)
        small = _expand_small(ctx, words, mode, 0, 15)
    want = _c_oracle_sorted([wide_table], words, mode, 0, 15)
    for i, (w, b, s, e) in enumerate(zip(words, big, small, want)):
        assert sorted(b) == e, (mode, i, w[:20], len(b), len(e))
        assert b == s, (mode, i, w[:20], "candidate order differs between batches")


def test_cluster_words_past_the_complex_slot_cap():
    """czech + german words with s/ss clusters: 3000 of them overflow k_keyspace_cplx's
    FAST slot cap (nw/16 + 1024); the overflow words take the DP path in the big batch
    and the FAST plan alone -- their ordered lists must agree."""
    from hashcat_a5_table_generator_amd import Context
    rng = np.random.default_rng(0x55)
    alpha = np.frombuffer(b"aeioutrs", dtype=np.uint8)
    words = []
    for _ in range(3000):
        w = bytes(rng.choice(alpha, size=int(rng.integers(3, 8))))
        j = int(rng.integers(0, len(w) + 1))
        words.append(w[:j] + b"ss" + w[j:])
    tabs = [table_path("czech"), table_path("german")]
    with Context(0) as ctx:
        ctx.load_tables(tabs)
        big = ctx.expand_words(words, 0, 0, 15)
        small = _expand_small(ctx, words, 0, 0, 15)
    want = _c_oracle_sorted(tabs, words, 0, 0, 15)
    for i, (w, b, s, e) in enumerate(zip(words, big, small, want)):
        assert sorted(b) == e, (i, w, len(b), len(e))
        assert b == s, (i, w, "candidate order differs between batches")


@pytest.mark.parametrize("mode,mn", [(0, 0), (1, 0), (2, 0), (3, 1)])
def test_hits_of_overflowing_batch_regenerate_their_plains(wide_table, mode, mn):
    """Fused MD5 over the budget-overflowing batch, then a5x_format_hits (which re-runs
    a sub-batch of only the hit words, where no budget runs out): every hit's digest is
    the MD5 of the candidate its index names in the batch, every printed plain hashes to
    its digest, and every planted candidate is found."""
    from hashcat_a5_table_generator_amd import Context, pack_words
    words = [b"z" * 9000] + _words(mode, 300, 0xC0 + mode)
    rng = np.random.default_rng(7 + mode)
    with Context(0) as ctx:
        ctx.load_tables([wide_table])
        cands = ctx.expand_words(words, mode, mn, 15)
        planted = {}
        for w in rng.choice(np.arange(1, len(words)), size=120, replace=False):
            if cands[w]:
                c = cands[w][int(rng.integers(0, len(cands[w])))]
                planted[hashlib.md5(c).digest()] = c
        ctx.set_targets(0, b"".join(planted))
        d, o = pack_words(words)
        hits, _ = ctx.expand_digest(d, o, mode, mn, 15, hit_cap=1 << 14)
        for w, c, dg in hits:
            assert hashlib.md5(cands[w][c]).digest() == dg, (mode, w, c)
        text = ctx.format_hits(d, o, hits, mode, mn, 15)
    seen = set()
    for line in text.split(b"\n")[:-1]:
        hx, plain = line.split(b":", 1)
        if plain.startswith(b"$HEX[") and plain.endswith(b"]"):
            plain = binascii.unhexlify(plain[5:-1])
        assert hashlib.md5(plain).hexdigest().encode() == hx, line
        seen.add(bytes.fromhex(hx.decode()))
    assert set(planted) <= seen


@pytest.mark.parametrize("fast_waves,waves", [(6, 8), (16, 16)])
def test_oversized_workgroup_knobs_are_clamped(fast_waves, waves):
    """A5X_FAST_WAVES / A5X_WAVES beyond a kernel's __launch_bounds__ (256 threads for
    k_expand_fast*, k_expand_slow) used to launch 384-1024-thread workgroups that fail
    ("unspecified launch failure"); a5x_launch_expand now clamps each launch to the
    kernel's compiled maxThreadsPerBlock.  C3 words (FAST + slow + complex words) and
    the fused MD5 path, both against the C oracle."""
    from hashcat_a5_table_generator_amd import Context, pack_words, synth
    from oracle import c_oracle as co
    from test_gpu_configs import _check, _gpu_digest
    os.environ["A5X_FAST_WAVES"], os.environ["A5X_WAVES"] = str(fast_waves), str(waves)
    try:
        ctx = Context(0)
    finally:
        os.environ.pop("A5X_FAST_WAVES")
        os.environ.pop("A5X_WAVES")
    tabs = [table_path("czech"), table_path("german")]
    with ctx:
        ctx.load_tables(tabs)
        _, (data, offs) = synth.global_words("c3", 0, 50_000, seed=0x3C)
        tc, tb, got = _gpu_digest(ctx, data, offs)
        want = co.CTable(tabs).digest_batch(data, offs, 0, 0, 15)
        _check(got, want, data, offs)
        words = [bytes(data[int(offs[i]):int(offs[i + 1])]) for i in range(2000)]
        cands = ctx.expand_words(words, 0, 0, 15)
        planted = {hashlib.md5(c[len(c) // 2]).digest() for c in cands[::17] if c}
        ctx.set_targets(0, b"".join(planted))
        d, o = pack_words(words)
        hits, _ = ctx.expand_digest(d, o, 0, 0, 15, hit_cap=1 << 14)
    assert planted <= {dg for _, _, dg in hits}
    for w, c, dg in hits:
        assert hashlib.md5(cands[w][c]).digest() == dg
