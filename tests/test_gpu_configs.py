"""BASELINE.json config shapes on the HIP path (C4 shard, C5 lookup), checked against
the C oracle (oracle/a5_oracle.c, the restatement of main.go:168-205 / :308-440) by
per-word order-independent digests {count, bytes, sum h, sum h^2}.

C4 = configs[3]: qwerty-cyrillic x length-10 [a-z] words, 1023 candidates per word,
one global list split across GPUs by output bytes (bench.py shard_for_rank).
"""
import os

import numpy as np
import pytest

from conftest import table_path

pytestmark = pytest.mark.gpu

NTH = min(16, os.cpu_count() or 1)  # the GPU box's CPU share


def _gpu_digest(ctx, data, offs, mode=0, mn=0, mx=15):
    """Expand the batch into one HBM buffer and digest every word on the device."""
    from hashcat_a5_table_generator_amd import DeviceBuffer
    n = len(offs) - 1
    dw = DeviceBuffer.from_array(ctx, data)
    do = DeviceBuffer.from_array(ctx, offs)
    tc, tb = ctx.keyspace_device(dw.ptr, do.ptr, n, mode, mn, mx)
    out = DeviceBuffer(ctx, max(tb, 16))
    boff = DeviceBuffer(ctx, (n + 1) * 8)
    st = ctx.expand_device(dw.ptr, do.ptr, n, out.ptr, tb, mode, mn, mx, d_byte_off=boff.ptr)
    assert st["candidates"] == tc and st["bytes"] == tb
    dig = DeviceBuffer(ctx, n * 32)
    ctx.digest_device(out.ptr, boff.ptr, 0, n, dig.ptr)
    got = dig.to_array(np.uint64).reshape(n, 4)
    for b in (out, boff, dig, dw, do):
        b.free()
    return tc, tb, got


def _check(got, want, data, offs):
    bad = np.nonzero((got != want).any(axis=1))[0]
    assert len(bad) == 0, [(bytes(data[int(offs[i]):int(offs[i + 1])]), got[i], want[i]) for i in bad[:5]]


@pytest.fixture(scope="module")
def c4_ctx():
    from hashcat_a5_table_generator_amd import Context
    c = Context(0)
    c.load_tables([table_path("qwerty-cyrillic")])
    yield c
    c.close()


def test_c4_shape_one_million_words(c4_ctx):
    """1M length-10 words x qwerty-cyrillic (1.02e9 candidates, ~16 GB) == C oracle."""
    from hashcat_a5_table_generator_amd import synth
    from oracle import c_oracle as co
    _, (data, offs) = synth.global_words("c4", 0, 1_000_000, seed=0xC4)
    tc, tb, got = _gpu_digest(c4_ctx, data, offs)
    assert tc == 1023 * 1_000_000  # every [a-z] letter has exactly one cyrillic value
    want = co.CTable([table_path("qwerty-cyrillic")]).digest_batch(data, offs, 0, 0, 15, nthreads=NTH)
    _check(got, want, data, offs)


def test_c4_shard_past_u32_limits(c4_ctx):
    """A C4 shard past 2^32 candidates and 64 GiB of output in ONE call (the per-GPU
    shard of the 100M-word run is 1.28e10 candidates): counts, offsets and chunk
    indices must not wrap.  Words [w0, w1) of the global list, as bench.py's partition
    hands them to a rank."""
    from hashcat_a5_table_generator_amd import synth
    from oracle import c_oracle as co
    w0, w1 = 3_000_000, 7_300_000
    _, (data, offs) = synth.global_words("c4", w0, w1, seed=0xC4)
    n = w1 - w0
    tc, tb, got = _gpu_digest(c4_ctx, data, offs)
    assert tc == 1023 * n and tc > (1 << 32) and tb > (64 << 30)
    want = co.CTable([table_path("qwerty-cyrillic")]).digest_batch(data, offs, 0, 0, 15, nthreads=NTH)
    _check(got, want, data, offs)


def test_c4_partition_shards_cover_the_list(c4_ctx):
    """The north_star split on one device: the keyspace prefix of the whole list, split
    for 8 ranks (a5x_partition); the 8 shards expanded separately give the same per-word
    digests as the whole list, and the shards' output bytes are balanced."""
    from hashcat_a5_table_generator_amd import DeviceBuffer, partition, synth
    _, (data, offs) = synth.global_words("c3", 0, 400_000, seed=0xC3)
    c4_ctx.clear_table()
    c4_ctx.load_tables([table_path("czech"), table_path("german")])
    try:
        n = len(offs) - 1
        dw, do = DeviceBuffer.from_array(c4_ctx, data), DeviceBuffer.from_array(c4_ctx, offs)
        pre = DeviceBuffer(c4_ctx, (n + 1) * 8)
        tc, tb = c4_ctx.keyspace_device(dw.ptr, do.ptr, n, d_byte_off=pre.ptr)
        prefix = pre.to_array(np.uint64, count=n + 1)
        assert int(prefix[-1]) == tb
        split = partition(prefix, 8)
        _, _, whole = _gpu_digest(c4_ctx, data, offs)
        parts, sizes = [], []
        for r in range(8):
            a, b = int(split[r]), int(split[r + 1])
            sd = np.zeros(int(offs[b] - offs[a]) + 16, dtype=np.uint8)
            sd[: int(offs[b] - offs[a])] = data[int(offs[a]):int(offs[b])]
            so = (offs[a:b + 1] - offs[a]).astype(np.uint64)
            _, sb, g = _gpu_digest(c4_ctx, sd, so)
            parts.append(g)
            sizes.append(sb)
        assert np.array_equal(np.concatenate(parts), whole)
        assert sum(sizes) == tb and max(sizes) - min(sizes) < 0.01 * tb
    finally:
        c4_ctx.clear_table()
        c4_ctx.load_tables([table_path("qwerty-cyrillic")])


@pytest.mark.parametrize("algo", [0, 1])
def test_c5_shape_lookup_one_million_targets(algo):
    """C5 = configs[4]: greek-hebrew x Greek words, fused expansion + MD5 (0) / NTLM (1)
    + lookup against 1M targets (1000 planted candidates + random digests).  Every
    planted (word, candidate) is found; every hit is a real candidate whose digest is a
    target; no random target hits."""
    from hashcat_a5_table_generator_amd import Context, DeviceBuffer, synth
    from oracle import digest_oracle as dg
    f = dg.ALGOS[algo]
    _, (data, offs) = synth.global_words("c5", 0, 200_000, seed=0xC5 + algo)
    n = len(offs) - 1
    rng = np.random.default_rng(0xC5 + algo)
    with Context(0) as ctx:
        ctx.load_tables([table_path("greek-hebrew")])
        wsample = sorted(set(int(x) for x in rng.choice(n, size=1200, replace=False)))
        words = [bytes(data[int(offs[i]):int(offs[i + 1])]) for i in wsample]
        cands = ctx.expand_words(words, 0, 0, 15)
        planted, plains = {}, set()
        for w, cs in zip(wsample, cands):
            if cs and len(planted) < 1000:
                c = int(rng.integers(0, len(cs)))
                planted[(w, c)] = f(cs[c])
                plains.add(cs[c])
        rand = rng.integers(0, 256, size=(1_000_000 - len(planted), 16), dtype=np.uint8)
        targets = np.concatenate([np.frombuffer(b"".join(planted.values()), dtype=np.uint8).reshape(-1, 16), rand])
        ctx.set_targets(algo, targets)
        dw, do = DeviceBuffer.from_array(ctx, data), DeviceBuffer.from_array(ctx, offs)
        tc, _ = ctx.keyspace_device(dw.ptr, do.ptr, n)
        hits, st = ctx.expand_digest_device(dw.ptr, do.ptr, n, 0, 0, 15, scratch_bytes=1 << 30, hit_cap=1 << 16)
        assert st["candidates"] == tc and tc > 200_000_000
        got = {(w, c): d for w, c, d in hits}
        assert len(got) == len(hits)  # no duplicate reports
        missing = [k for k in planted if k not in got]
        assert not missing, missing[:5]
        tset = set(planted.values())
        hw = sorted({w for w, _ in got})
        hc = dict(zip(hw, ctx.expand_words([bytes(data[int(offs[w]):int(offs[w + 1])]) for w in hw], 0, 0, 15)))
        for (w, c), d in got.items():
            assert f(hc[w][c]) == d and d in tset, (w, c, d.hex())
        # zero false hits: a hit beyond the planted pairs is another occurrence of a planted
        # plain (the same candidate text from another word or position), never a random target
        assert all(hc[w][c] in plains for w, c in set(got) - set(planted))


@pytest.mark.parametrize("mode,mn", [(2, 0), (3, 0), (3, 1), (2, 2), (1, 0), (1, 2)])
def test_c5_shape_substitute_all_modes(mode, mn):
    """-s / -s -r / -r at the C5 shape (README.MD:159,163: greek-hebrew -s, -s -r -m 1):
    100k Greek words (positional fast paths: single-codepoint patterns, repeated letters
    tie their occurrences; -r with length-preserving subs[0]) == C oracle per-word digests."""
    from hashcat_a5_table_generator_amd import Context, synth
    from oracle import c_oracle as co
    _, (data, offs) = synth.global_words("c5", 0, 100_000, seed=0x55 + mode)
    with Context(0) as ctx:
        ctx.load_tables([table_path("greek-hebrew")])
        tc, tb, got = _gpu_digest(ctx, data, offs, mode, mn, 15)
    want = co.CTable([table_path("greek-hebrew")]).digest_batch(data, offs, mode, mn, 15, nthreads=NTH)
    assert tc == int(want[:, 0].sum()) and tc > 10_000_000
    _check(got, want, data, offs)


@pytest.mark.parametrize("algo,wl,tabs", [(0, "c3", ["czech", "german"]), (1, "c3", ["czech", "german"]),
                                         (1, "c5", ["greek-hebrew"])])
def test_fused_equals_two_pass(algo, wl, tabs):
    """The fused paths (k_expand_fast_md5 / k_expand_fast_ntlm: candidates hashed in the
    LDS ring, NTLM's UTF-16LE produced while the MD4 blocks fill) and the two-pass path
    (HBM scratch + k_digest_stream) report the same hits."""
    from hashcat_a5_table_generator_amd import Context, DeviceBuffer, synth
    from oracle import digest_oracle as dg
    _, (data, offs) = synth.global_words(wl, 0, 50_000, seed=0xF5)
    n = len(offs) - 1
    rng = np.random.default_rng(3)
    f = dg.ALGOS[algo]
    with Context(0) as ctx:
        ctx.load_tables([table_path(t) for t in tabs])
        ws = sorted(set(int(x) for x in rng.choice(n, size=300, replace=False)))
        cands = ctx.expand_words([bytes(data[int(offs[i]):int(offs[i + 1])]) for i in ws], 0, 0, 15)
        tg = [f(cs[int(rng.integers(0, len(cs)))]) for cs in cands if cs]
        ctx.set_targets(algo, b"".join(tg) + bytes(rng.integers(0, 256, 16 * 20000, dtype=np.uint8)))
        dw, do = DeviceBuffer.from_array(ctx, data), DeviceBuffer.from_array(ctx, offs)
        fused, st = ctx.expand_digest_device(dw.ptr, do.ptr, n, 0, 0, 15, hit_cap=1 << 14)
        os.environ["A5X_NO_FUSED_DIGEST"] = "1"
        try:
            two, st2 = ctx.expand_digest_device(dw.ptr, do.ptr, n, 0, 0, 15, hit_cap=1 << 14)
        finally:
            os.environ.pop("A5X_NO_FUSED_DIGEST")
    assert st["candidates"] == st2["candidates"]
    assert st["ms_total"] - st["ms_keyspace"] - st["ms_expand"] < 1e-3 < st2["ms_total"] - st2["ms_keyspace"] - st2["ms_expand"]
    assert sorted(fused) == sorted(two) and len(fused) >= len(tg)


@pytest.mark.parametrize("algo", [0, 1])
def test_hybrid_fused_digest_mixed_batch(algo):
    """A batch with non-FAST words (more than 8 pieces, BIG and pass-G lines)
    among FAST ones: the fused kernel hashes the FAST words and the others go through the
    two-pass path as a gathered sub-batch; the hits equal the all-two-pass run's and
    include every planted (word, candidate)."""
    from hashcat_a5_table_generator_amd import Context, DeviceBuffer, pack_words, synth
    from oracle import digest_oracle as dg
    _, (data, offs) = synth.global_words("c3", 0, 20_000, seed=0xB7)
    words = [bytes(data[int(offs[i]):int(offs[i + 1])]) for i in range(len(offs) - 1)]
    rng = np.random.default_rng(17 + algo)
    digits = list(b"0123456789")

    def spread(L, keys):
        w = bytearray(np.asarray(rng.choice(digits, size=L), dtype=np.uint8).tobytes())
        for p in rng.choice(L, size=len(keys), replace=False):
            w[p] = keys[int(rng.integers(0, len(keys)))]
        return bytes(w)

    extra = [spread(int(rng.integers(57, 62)), b"aeu") for _ in range(300)]   # > 8 pieces: not FAST
    extra += [spread(L, b"ae") for L in (100, 700, 2100, 5000)]                # BIG and pass-G lines
    pos = sorted(rng.choice(len(words) + len(extra), size=len(extra), replace=False))
    for p, w in zip(pos, extra):
        words.insert(int(p), w)
    f = dg.ALGOS[algo]
    with Context(0) as ctx:
        ctx.load_tables([table_path("czech"), table_path("german")])
        pick = sorted(set(int(x) for x in rng.choice(len(words), size=200, replace=False)) | set(int(p) for p in pos))
        cands = ctx.expand_words([words[i] for i in pick], 0, 0, 15)
        planted = {}
        for i, cs in zip(pick, cands):
            if cs:
                c = int(rng.integers(0, len(cs)))
                planted[(i, c)] = f(cs[c])
        ctx.set_targets(algo, b"".join(planted.values()) + bytes(rng.integers(0, 256, 16 * 5000, dtype=np.uint8)))
        d, o = pack_words(words)
        dw, do = DeviceBuffer.from_array(ctx, d), DeviceBuffer.from_array(ctx, o)
        fused, st = ctx.expand_digest_device(dw.ptr, do.ptr, len(words), 0, 0, 15, hit_cap=1 << 14)
        os.environ["A5X_NO_FUSED_DIGEST"] = "1"
        try:
            two, st2 = ctx.expand_digest_device(dw.ptr, do.ptr, len(words), 0, 0, 15, hit_cap=1 << 14)
        finally:
            os.environ.pop("A5X_NO_FUSED_DIGEST")
    assert st["candidates"] == st2["candidates"]
    assert sorted(fused) == sorted(two)
    got = {(w, c) for w, c, _ in fused}
    assert set(planted) <= got
    assert any(w in set(int(p) for p in pos) for w, _ in got)  # hits in the non-FAST words too


def test_hybrid_digest_hit_cap_below_hits():
    """Regression for the hybrid path's host-side hit handling (round-2 segfault record,
    gpurun_out/th.log at 02:01): the caller's buffer smaller than the hits
    found -- hit_cap 0 with a null buffer, hit_cap filled by the fused FAST words alone
    (the non-FAST sub-batch gets room == 0), and room for only some of the sub-batch's
    hits.  Every call reports the full count with A5X_E_CAPACITY, writes only inside
    the buffer, and returns a subset of the uncapped run's hits."""
    import ctypes
    from hashcat_a5_table_generator_amd import Context, DeviceBuffer, _lib, pack_words, synth
    from oracle import digest_oracle as dg
    _, (data, offs) = synth.global_words("c3", 0, 4000, seed=0xB8)
    words = [bytes(data[int(offs[i]):int(offs[i + 1])]) for i in range(len(offs) - 1)]
    rng = np.random.default_rng(23)
    extra = [bytes(rng.choice(list(b"0123456789"), size=58).astype(np.uint8)) + b"aeu" for _ in range(40)]
    extra += [b"1" * 700 + b"ae", b"2" * 2100 + b"ea"]  # BIG and pass-G lines
    words += extra
    with Context(0) as ctx:
        ctx.load_tables([table_path("czech"), table_path("german")])
        cands = ctx.expand_words(words, 0, 0, 15)
        # every candidate of 30 FAST words and of every non-FAST word is a target: many
        # hits on both sides of the hybrid split
        pick = list(range(30)) + list(range(len(words) - len(extra), len(words)))
        tg = {dg.md5(c) for i in pick for c in cands[i][:64]}
        ctx.set_targets(0, b"".join(sorted(tg)))
        d, o = pack_words(words)
        dw, do = DeviceBuffer.from_array(ctx, d), DeviceBuffer.from_array(ctx, o)
        full, _ = ctx.expand_digest_device(dw.ptr, do.ptr, len(words), 0, 0, 15, hit_cap=1 << 16)
        fset = set(full)
        n_fast = sum(1 for w, _, _ in full if w < 30)
        assert n_fast > 0 and len(full) > n_fast
        for cap in (0, n_fast, n_fast + 3, len(full) - 1):
            arr = (_lib.Hit * (cap + 8))()  # 8 guard entries past the cap stay untouched
            for k in range(cap, cap + 8):
                arr[k].word = 0xDEADBEEF
            nh = ctypes.c_uint64()
            rc = ctx._L.a5x_expand_digest_device(ctx.h, dw.ptr, do.ptr, len(words), 0, 0, 15, 0,
                                                 arr if cap else None, cap, ctypes.byref(nh), None, None)
            assert rc == -8, (cap, rc)  # A5X_E_CAPACITY
            assert nh.value == len(full)
            assert all(arr[k].word == 0xDEADBEEF for k in range(cap, cap + 8))
            got = ctx._hits(arr, cap)
            assert set(got) <= fset and len(set(got)) == cap


def test_c2_shape_greek_and_ascii():
    """C2 = configs[1] (qwerty-greek.table; greek-dictionary.txt is not in the snapshot,
    .MISSING_LARGE_BLOBS:1): 1M synthetic Greek words give exactly 0 candidates (every
    qwerty-greek key is ASCII, so processWord never matches a Greek byte), and the
    ASCII variant -- 1M [a-z] words x qwerty-greek, ~971 multi-byte candidates per word --
    equals the C oracle's per-word digests."""
    from hashcat_a5_table_generator_amd import Context, DeviceBuffer, synth
    from oracle import c_oracle as co
    with Context(0) as ctx:
        ctx.load_tables([table_path("qwerty-greek")])
        _, (data, offs) = synth.global_words("c2", 0, 1_000_000, seed=0xC2)
        dw, do = DeviceBuffer.from_array(ctx, data), DeviceBuffer.from_array(ctx, offs)
        tc, tb = ctx.keyspace_device(dw.ptr, do.ptr, len(offs) - 1)
        assert (tc, tb) == (0, 0)
        dw.free()
        do.free()
        _, (data, offs) = synth.global_words("c2a", 0, 1_000_000, seed=0xC2A)
        tc, tb, got = _gpu_digest(ctx, data, offs)
    n = len(offs) - 1
    assert 900 * n < tc < 1050 * n and tb > 15 * tc
    want = co.CTable([table_path("qwerty-greek")]).digest_batch(data, offs, 0, 0, 15, nthreads=NTH)
    _check(got, want, data, offs)


@pytest.mark.parametrize("algo,mode,mn,wl,tabs,ntarget", [
    (0, 3, 1, "c5", ["greek-hebrew"], 1_000_000),   # README.MD:159,163: -s -r -m 1 | hashcat, C5 shape
    (1, 3, 1, "c5", ["greek-hebrew"], 1_000_000),
    (0, 2, 0, "c5", ["greek-hebrew"], 20_000),
    (1, 1, 0, "c5", ["greek-hebrew"], 20_000),
    (0, 2, 0, "c3", ["czech", "german"], 20_000),    # non-confluent s / ss: the byte builder
    (1, 1, 2, "c3", ["czech", "german"], 20_000),    # -r with the running-offset bug: builder
])
def test_mode_fused_digest_equals_two_pass(algo, mode, mn, wl, tabs, ntarget):
    """-r / -s / -s -r fused digest (op 2 of the mode engines: every candidate hashed in
    the positional ring or the builder's lane buffer, no length pass, no HBM stream)
    reports exactly the two-pass path's hits (expansion into HBM scratch +
    k_digest_stream), including every planted (word, candidate) -- with lines past the
    LDS engines' 128 B (mode pass G) in the batch."""
    from hashcat_a5_table_generator_amd import Context, DeviceBuffer, pack_words, synth
    from oracle import digest_oracle as dg
    _, (data, offs) = synth.global_words(wl, 0, 40_000, seed=0xF6 + mode)
    words = [bytes(data[int(offs[i]):int(offs[i + 1])]) for i in range(len(offs) - 1)]
    words[100:100] = [b"0" * 150 + words[7], words[9] + b"1" * 300]  # > 128 B: mode pass G
    n = len(words)
    rng = np.random.default_rng(5 + mode)
    f = dg.ALGOS[algo]
    with Context(0) as ctx:
        ctx.load_tables([table_path(t) for t in tabs])
        ws = sorted(set(int(x) for x in rng.choice(n, size=300, replace=False)) | {100, 101})
        cands = ctx.expand_words([words[i] for i in ws], mode, mn, 15)
        planted = {}
        for w, cs in zip(ws, cands):
            if cs:
                c = int(rng.integers(0, len(cs)))
                planted[(w, c)] = f(cs[c])
        rand = rng.integers(0, 256, size=(ntarget - len(planted), 16), dtype=np.uint8)
        ctx.set_targets(algo, b"".join(planted.values()) + rand.tobytes())
        d, o = pack_words(words)
        dw, do = DeviceBuffer.from_array(ctx, d), DeviceBuffer.from_array(ctx, o)
        fused, st = ctx.expand_digest_device(dw.ptr, do.ptr, n, mode, mn, 15, hit_cap=1 << 16)
        os.environ["A5X_NO_FUSED_DIGEST"] = "1"
        try:
            two, st2 = ctx.expand_digest_device(dw.ptr, do.ptr, n, mode, mn, 15, hit_cap=1 << 16)
        finally:
            os.environ.pop("A5X_NO_FUSED_DIGEST")
    assert st["candidates"] == st2["candidates"] > 0
    assert sorted(fused) == sorted(two)
    got = {(w, c) for w, c, _ in fused}
    assert set(planted) <= got
    assert (100, 0) in {(w, 0) for w, _ in got} or all(w != 100 for w, _ in planted)
