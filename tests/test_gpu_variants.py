"""The product's alternative paths give the same bytes (through the C ABI, vs the C oracle).

Round 5 added paths the default run picks by the batch's shape:
  * k_keyspace_thread<true>: UTF-8 batches walked by lead bytes when every key starts on one
    (A5xTableHdr::lead_only); A5X_NO_UTF_WALK=1 forces the byte walk;
  * k_keyspace_vsub in two lane-slot sizes (words <= 32 B first, the rest to the large one);
    A5X_VSUB_LARGE_ONLY=1 runs the large one alone;
  * 16384-candidate expansion chunks; A5X_CHUNK sets another size.
Each knob's path must match the oracle (/root/reference/main.go:168-205, :208-305,
:308-440 restated in oracle/a5_oracle.c) word for word, as the default path does in
test_gpu_configs.py.
"""
import os

import numpy as np
import pytest

from conftest import table_path

pytestmark = pytest.mark.gpu

NTH = min(16, os.cpu_count() or 1)


def _digests(data, offs, mode, mn, tables):
    from hashcat_a5_table_generator_amd import Context, DeviceBuffer
    n = len(offs) - 1
    with Context(0) as ctx:
        ctx.load_tables([table_path(t) for t in tables])
        dw = DeviceBuffer.from_array(ctx, data)
        do = DeviceBuffer.from_array(ctx, offs)
        tc, tb = ctx.keyspace_device(dw.ptr, do.ptr, n, mode, mn, 15)
        out = DeviceBuffer(ctx, max(tb, 16))
        boff = DeviceBuffer(ctx, (n + 1) * 8)
        st = ctx.expand_device(dw.ptr, do.ptr, n, out.ptr, tb, mode, mn, 15, d_byte_off=boff.ptr)
        assert st["candidates"] == tc and st["bytes"] == tb
        dig = DeviceBuffer(ctx, n * 32)
        ctx.digest_device(out.ptr, boff.ptr, 0, n, dig.ptr)
        got = dig.to_array(np.uint64).reshape(n, 4)
        for b in (out, boff, dig, dw, do):
            b.free()
    return got


@pytest.mark.parametrize("knob,val,mode,mn", [
    ("A5X_NO_UTF_WALK", "1", 0, 0),
    ("A5X_NO_UTF_WALK", "1", 1, 0),
    ("A5X_NO_UTF_WALK", "1", 2, 0),
    ("A5X_VSUB_LARGE_ONLY", "1", 2, 0),
    ("A5X_VSUB_LARGE_ONLY", "1", 3, 1),
    ("A5X_CHUNK", "8192", 0, 0),
    ("A5X_CHUNK", "4096", 2, 0),
])
def test_knob_path_equals_oracle(monkeypatch, knob, val, mode, mn):
    """C5-shaped Greek words (UTF-8, greek-hebrew: keys on lead bytes) through the knob's
    path == the C oracle's per-word digests {count, bytes, sum h, sum h^2}."""
    from hashcat_a5_table_generator_amd import synth
    from oracle import c_oracle as co
    _, (data, offs) = synth.global_words("c5", 0, 40_000, seed=0x77 + mode)
    monkeypatch.setenv(knob, val)
    got = _digests(data, offs, mode, mn, ["greek-hebrew"])
    want = co.CTable([table_path("greek-hebrew")]).digest_batch(data, offs, mode, mn, 15, nthreads=NTH)
    bad = np.nonzero((got != want).any(axis=1))[0]
    assert len(bad) == 0, [(bytes(data[int(offs[i]):int(offs[i + 1])]), got[i], want[i]) for i in bad[:5]]


def test_mixed_ascii_and_utf8_words():
    """A batch whose first 256 KiB are ASCII picks the byte walk, one that starts with UTF-8
    the lead-byte walk; either way the mixed words (ASCII, Greek, Czech letters) equal the
    oracle (the walks are exact: no key starts on a continuation byte)."""
    from hashcat_a5_table_generator_amd import pack_words
    from oracle import c_oracle as co
    rng = np.random.default_rng(5)
    ascii_w = ["".join(chr(97 + int(x)) for x in rng.integers(0, 26, size=int(rng.integers(3, 12)))) for _ in range(60_000)]
    utf_w = ["".join("aeiosčřžáéíαβγ"[int(x)] for x in rng.integers(0, 14, size=int(rng.integers(3, 10))))
             for _ in range(2_000)]
    tabs = ["czech", "german", "greek-hebrew"]
    for words in (ascii_w + utf_w, utf_w + ascii_w):
        enc = [w.encode() for w in words]
        data, offs = pack_words(enc)
        got = _digests(data, offs, 0, 0, tabs)
        want = co.CTable([table_path(t) for t in tabs]).digest_batch(data, offs, 0, 0, 15, nthreads=NTH)
        bad = np.nonzero((got != want).any(axis=1))[0]
        assert len(bad) == 0, [enc[i] for i in bad[:5]]
