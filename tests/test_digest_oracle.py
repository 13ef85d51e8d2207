"""Pin the digest oracle (oracle/digest_oracle.py): RFC 1320 MD4 suite, NTLM vectors,
MD5 (RFC 1321 appendix A.5), Go-style UTF-16 conversion."""
import pytest

from oracle import digest_oracle as dg

RFC1320 = [
    (b"", "31d6cfe0d16ae931b73c59d7e0c089c0"),
    (b"a", "bde52cb31de33e46245e05fbdbd6fb24"),
    (b"abc", "a448017aaf21d8525fc10ae87aa6729d"),
    (b"message digest", "d9130a8164549fe818874806e1c7014b"),
    (b"abcdefghijklmnopqrstuvwxyz", "d79e1c308aa5bbcdeea8ed63df412da9"),
    (b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789", "043f8582f241db351ce627e153e7f0e4"),
    (b"1234567890" * 8, "e33b4ddc9c38f2199c3e7b164fcc0536"),
]


@pytest.mark.parametrize("msg,hexd", RFC1320)
def test_md4_rfc1320(msg, hexd):
    assert dg.md4(msg).hex() == hexd


def test_md5_rfc1321():
    assert dg.md5(b"").hex() == "d41d8cd98f00b204e9800998ecf8427e"
    assert dg.md5(b"message digest").hex() == "f96b697d7cb7938d525a2f31aaf161d0"


def test_ntlm_vectors():
    assert dg.ntlm(b"password").hex() == "8846f7eaee8fb117ad06bdd830b7586c"
    assert dg.ntlm(b"").hex() == "31d6cfe0d16ae931b73c59d7e0c089c0"


def test_utf16_go_semantics():
    assert dg.utf16le_go("é".encode()) == b"\xe9\x00"
    assert dg.utf16le_go(b"\xff") == b"\xfd\xff"            # invalid byte -> U+FFFD
    assert dg.utf16le_go(b"\xe2\x82") == b"\xfd\xff\xfd\xff"  # truncated sequence: one U+FFFD per byte
    assert dg.utf16le_go("😀".encode()) == b"\x3d\xd8\x00\xde"  # surrogate pair


def test_c_digests_match_python_oracle():
    """oracle/a5_oracle.c's MD5 / NTLM (the C digest baseline, bench.py digest_cpu_baseline)
    equal hashlib MD5 and the RFC 1320-pinned Python NTLM, incl. invalid UTF-8, astral
    runes and multi-block messages."""
    import hashlib
    import random
    from oracle import c_oracle as co
    assert co.digest(1, b"password").hex() == "8846f7eaee8fb117ad06bdd830b7586c"
    rng = random.Random(7)
    samples = [b"", "é😀".encode(), b"\xe2\x82", b"\xff" * 70] + [
        bytes(rng.randrange(256) for _ in range(n)) for n in list(range(0, 130)) + [1000]]
    for s in samples:
        assert co.digest(0, s) == hashlib.md5(s).digest()
        assert co.digest(1, s) == dg.ntlm(s)


def test_c_digest_run_counts_planted_hits():
    """a5o_digest_run (threaded expansion + digest + probe) finds every planted target."""
    import os
    import numpy as np
    from conftest import ROOT
    from oracle import c_oracle as co
    t = co.CTable([os.path.join(ROOT, "tests", "golden", "tables", "greek-hebrew.table")])
    words = ["καλημέρα".encode(), "αλφα".encode(), b"xyz"]
    data, offs = co.pack_words(words)
    cands = [c for w in words for c in t.expand_word(w, 0, 0, 15)]
    for algo, f in ((0, dg.md5), (1, dg.ntlm)):
        tg = np.frombuffer(b"".join(f(c) for c in cands[::7]) + bytes(range(16)), dtype=np.uint8).reshape(-1, 16)
        for th in (1, 3):
            assert t.digest_run(data, offs, 0, 0, 15, algo, tg, th) == (len(cands), len(cands[::7]))
