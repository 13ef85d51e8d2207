"""The oracle itself, pinned (CPU only).

The reference has no tests or fixtures, and Go + kong
v1.12.1 are unavailable here, so the oracle is pinned by:
  * SURVEY.md Appendix B known-answer vectors (counts + sorted-stream sha256 for
    all four engines, the -r corruption and panic), produced by an independent
    restatement during the survey;
  * hand-verifiable identities (2^n - 1, sum_c C(17, c), the README "hello");
  * cross-checks between the Python and C restatements and the keyspace DP.
"""
import collections
import hashlib
import itertools
import json
import math
import os
import random

import pytest

from conftest import ROOT, table_path
from oracle import a5_oracle as o


def tabs(*names):
    return o.load_tables([table_path(n) for n in names])


def sha16(c):
    return hashlib.sha256(b"".join(sorted(x + b"\n" for x in c))).hexdigest()[:16]


README = {b"h": [b"H"], b"e": [b"E"], b"l": [b"L"], b"o": [b"O"]}

# (tables, word) -> [default, -r, -s, -s -r] as "n/sha16" or "n"
APPENDIX_B = [
    (None, "hello", ["31", "32", "16", "16"]),
    (("qwerty-cyrillic",), "hello", ["31/5dbbabec877a2f9b", "32/d524175277092a92", "16/2d6249badf48690f",
                                      "16/2d6249badf48690f"]),
    (("qwerty-cyrillic",), "password", ["255/410d9958f4ca2539", "256/44b3a069f0759aa1", "128/f773969eeba1e906",
                                         "128/f773969eeba1e906"]),
    (("qwerty-cyrillic",), "abcdefghijklmnopq", ["131053/65c59fec8bbbc880", "131054/b72110f7841a1ffa",
                                                  "131054/f86e68b03ed54559", "131054/f86e68b03ed54559"]),
    (("czech", "german"), "strasse", ["359/bdc9580ce35e77b6", "160/5182929de81f7628", "144/c2b34ecd857ee4bc",
                                       "64/a1dcc5e4a0a25560"]),
    (("czech", "german"), "hello", ["8/a5faf1933cc1466d", "4/981812473ea3531c", "9/ea287d1323a5f872",
                                     "4/985306f955f16c3f"]),
    (("qwerty-azerty",), "aqua", ["7/ce96b43f78a97c7a", "8/3400bfbb17322a66", "4/d0f40c65ddba3790",
                                   "4/d0f40c65ddba3790"]),
    (("qwerty-azerty",), "m,;1", ["95/4e4ff3b27c0c49af", "16/d7bbf8cf7b23b42c", "96/93af7a720dba66b5",
                                   "16/e11730de23456a01"]),
    (("qwerty-greek",), "kalimera", ["255/c91c2c1617c99287", "256/01dd100b47e0bc2f", "128/e4ae1f5819654ef5",
                                      "128/e4ae1f5819654ef5"]),
    (("greek-hebrew",), "καλημέρα", ["127/f96af7a4c3e5e3d5", "128/deae50758a8193c2", "64/f55bd990a15ed463",
                                      "64/f55bd990a15ed463"]),
    (("greek-hebrew",), "αλφα", ["15/2d63f69806d66bca", "16/3635dffe5076e0ec", "8/8896745e98dd0fac",
                                  "8/8896745e98dd0fac"]),
    (("qwerty-greek",), "καλημέρα;", ["1/cb8ea1464d41ce3b", "2/ec33f73bfd72c3cc", "2/ec33f73bfd72c3cc",
                                       "2/ec33f73bfd72c3cc"]),
    (("qwerty-cyrillic",), "", ["0", "1", "1", "1"]),
]


@pytest.mark.parametrize("tables,word,want", APPENDIX_B)
def test_appendix_b_vectors(tables, word, want):
    sub = README if tables is None else tabs(*tables)
    for mode in range(4):
        c = o.expand(word.encode(), sub, mode, 0, 15)
        exp = want[mode]
        got = f"{len(c)}/{sha16(c)}" if "/" in exp else str(len(c))
        assert got == exp, (tables, word, mode)


def test_appendix_b_reverse_bug_and_panic():
    cyr = tabs("qwerty-cyrillic")
    assert sorted(o.process_word_reverse(b"qw", cyr, 0, 15)) == sorted(
        [b"q\xd0\xb9\x86", b"q\xd1\x86", b"\xd0\xb9w", b"qw"])
    with pytest.raises(o.GoPanic):
        o.process_word_reverse("1é".encode(), tabs("qwerty-azerty"), 0, 15)


def test_appendix_b_identities():
    cyr = tabs("qwerty-cyrillic")
    assert len(o.process_word(b"hello", cyr, 0, 0)) == 0
    assert len(o.process_word(b"hello", cyr, 2, 3)) == 20
    assert len(o.process_word(b"hello", cyr, 5, 5)) == 1
    assert len(o.process_word(b"hello", cyr, 6, 15)) == 0
    c = o.process_word(b"hello", tabs("czech", "czech"), 0, 15)
    assert len(c) == 14 and len(set(c)) == 5  # duplicates kept (main.go:48)


def test_analytic_counts():
    cyr = tabs("qwerty-cyrillic")
    for n in range(1, 11):
        w = b"abcdefghijklmnop"[:n]
        assert len(o.process_word(w, cyr, 0, 15)) == 2 ** n - 1
    assert o.keyspace_default(b"abcdefghijklmnopq", cyr, 0, 15)[0] == sum(math.comb(17, c) for c in range(1, 16))


def test_keyspace_dp_matches_enumeration():
    rng = random.Random(1)
    for _ in range(400):
        m = {}
        for _ in range(rng.randint(1, 5)):
            k = bytes(rng.choice(b"abs") for _ in range(rng.randint(1, 3)))
            m.setdefault(k, []).append(bytes(rng.choice(b"absxy") for _ in range(rng.randint(0, 3))))
        w = bytes(rng.choice(b"abs") for _ in range(rng.randint(0, 9)))
        mn, mx = rng.randint(-1, 4), rng.randint(-1, 8)
        c = o.process_word(w, m, mn, mx)
        assert o.keyspace_default(w, m, mn, mx) == (len(c), sum(len(x) + 1 for x in c))


def test_c_oracle_matches_python_oracle():
    from oracle import c_oracle as co
    rng = random.Random(5)
    for _ in range(1500):
        m = {}
        for _ in range(rng.randint(1, 5)):
            k = bytes(rng.choice(b"abs") for _ in range(rng.randint(0, 3)))
            m.setdefault(k, []).append(bytes(rng.choice(b"absxy") for _ in range(rng.randint(0, 3))))
        ct = co.CTable.from_map(m)
        w = bytes(rng.choice(b"abs") for _ in range(rng.randint(0, 9)))
        mn, mx = rng.randint(-1, 4), rng.randint(-1, 8)
        for mode in range(4):
            try:
                a = collections.Counter(o.expand(w, m, mode, mn, mx))
            except o.GoPanic:
                a = None
            try:
                b = collections.Counter(ct.expand_word(w, mode, mn, mx))
            except RuntimeError:
                b = None
            assert a == b, (mode, w, m, mn, mx)


def test_c_oracle_parser_matches_python_on_shipped_tables():
    from oracle import c_oracle as co
    names = ["czech", "german", "greek-hebrew", "qwerty-azerty", "qwerty-cyrillic", "qwerty-greek"]
    for n in names:
        assert co.CTable([table_path(n)]).to_map() == tabs(n)
    assert co.CTable([table_path("czech"), table_path("german")]).to_map() == tabs("czech", "german")


def test_substitute_all_membership_for_nonconfluent():
    """-s leaves depend on Go map order (main.go:339-341); sorted order is one of them."""
    az = tabs("qwerty-azerty")
    for leaf in o.leaves_substitute_all(b"aqua", az, 0, 15, False):
        canon = o._apply_in_order(b"aqua", leaf)
        assert canon in o.substitute_all_possible(b"aqua", leaf)
    # 'aqua' has order-dependent leaves: {a:q, q:a} gives 'aaua' (a first) or 'qquq' (q first)
    assert o.substitute_all_possible(b"aqua", [(b"a", b"q"), (b"q", b"a")]) == {b"aaua", b"qquq"}


def test_golden_fixture_is_current():
    """tests/golden/golden.json was produced by the current oracle (spot check)."""
    with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as f:
        cases = json.load(f)["cases"]
    rng = random.Random(9)
    for c in rng.sample(cases, 300):
        sub = tabs(*c["tables"])
        w = bytes.fromhex(c["word"])
        try:
            got = o.expand(w, sub, c["mode"], c["min"], c["max"])
            err = None
        except o.GoPanic:
            got, err = [], "panic"
        assert err == c["error"]
        assert len(got) == c["count"]
        assert hashlib.sha256(b"".join(sorted(x + b"\n" for x in got))).hexdigest() == c["sha256"]


def test_go_stdlib_semantics():
    # bufio.ScanLines
    assert o.scan_lines(b"a\r\nb\n\nc", True) == [b"a", b"b", b"", b"c"]
    assert o.scan_lines(b"a\n", True) == [b"a"]
    assert o.scan_lines(b"x" * 65535 + b"\nz", True) == [b"x" * 65535, b"z"]
    with pytest.raises(o.ScanTooLong):
        o.scan_lines(b"x" * 65536 + b"\n", True)
    assert o.scan_lines(b"a\n" + b"x" * 70000, False) == [b"a"]
    # strings.TrimSpace keeps U+00E0 (C3 A0) and U+0160 (C5 A0): qwerty-azerty.table:19, czech.table:18
    assert o.trim_space("0=à".encode() + b"\r ") == "0=à".encode()
    assert o.trim_space("  x ".encode()) == b"x"
    assert o.trim_space(b"\x85x\xa0") == b"\x85x\xa0"  # invalid UTF-8 bytes are not spaces
    assert o.trim_space(b"\x1cx") == b"\x1cx"          # Python's strip() would remove \x1c
    # decodeHexNotation
    assert o.decode_hex_notation(b"$HEX[e282ac]") == "€".encode()
    assert o.decode_hex_notation(b"$HEX[F0 9F 98 9C]") == "😜".encode()
    assert o.decode_hex_notation(b"$HEX[]") == b"$HEX[]"
    assert o.decode_hex_notation(b"$HEX[abc]") is None
    assert o.decode_hex_notation(b"$HEX[zz]") is None
    # strings.ReplaceAll with an empty pattern
    assert o.replace_all(b"ab", b"", b"-") == b"-a-b-"
    assert o.replace_all("é".encode(), b"", b"-") == "-é-".encode()
    # SplitN on the first '='
    t = o.parse_table_bytes(b"==x\na=b=c\n#c=d\nnoeq\n")
    assert t == {b"": [b"=x"], b"a": [b"b=c"]}
