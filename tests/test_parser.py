"""The product's host-side table parser and word splitter (liba5x, no GPU needed)
against the oracle's restatement of readSubstitutionTable (main.go:108-162),
the -t merge (main.go:40-50) and the dictionary scanner (main.go:72-74)."""
import ctypes
import random

import numpy as np
import pytest

from conftest import table_path
from oracle import a5_oracle as o

NAMES = ["czech", "german", "greek-hebrew", "qwerty-azerty", "qwerty-cyrillic", "qwerty-greek"]


@pytest.fixture(scope="module")
def host_ctx():
    from hashcat_a5_table_generator_amd import _lib
    from hashcat_a5_table_generator_amd.engine import Context
    c = Context.__new__(Context)
    c._L = _lib.load()
    h = ctypes.c_void_p()
    assert c._L.a5x_create(-1, ctypes.byref(h)) == 0  # host-only context
    c.h = h
    c.device = -1
    yield c
    c.close()


@pytest.mark.parametrize("name", NAMES)
def test_shipped_tables(host_ctx, name):
    host_ctx.clear_table()
    host_ctx.load_tables([table_path(name)])
    assert host_ctx.table() == o.load_tables([table_path(name)])


@pytest.mark.parametrize("combo", [["czech", "german"], ["german", "czech"], ["czech", "czech"],
                                   ["qwerty-azerty", "qwerty-cyrillic", "qwerty-greek"]])
def test_merge_order(host_ctx, combo):
    host_ctx.clear_table()
    host_ctx.load_tables([table_path(n) for n in combo])
    assert host_ctx.table() == o.load_tables([table_path(n) for n in combo])


EDGE_TABLES = [
    b"a=b\r\nc=d\r\n",                      # CRLF
    b"  a = b  \n\t#x=y\n#\n\n=\n",        # spaces kept inside key/value, comments, empty key+value
    b"==x\nk=v=w\nnoequals\n",             # first '=' splits
    b"$HEX[6575726f]=$HEX[e2 82 ac]\n",    # README.MD:174
    b":P=$HEX[F0 9F 98 9C]\n",             # README.MD:175
    b"$HEX[zz]=a\nb=$HEX[abc]\nc=$HEX[]\n",  # bad hex skipped, short literal kept
    "0=à\nS=Š\n".encode(),                 # trailing C3 A0 / C5 A0 must survive TrimSpace
    "  x=y 　\n".encode(),   # unicode spaces trimmed
    b"\x85x=y\xa0\n",                      # invalid UTF-8 bytes are not spaces
    b"a=1\na=2\na=1\n",                    # duplicates kept in order
    b"last=line-without-newline",
]


@pytest.mark.parametrize("data", EDGE_TABLES)
def test_edge_tables(host_ctx, data):
    host_ctx.clear_table()
    host_ctx.parse_table(data)
    assert host_ctx.table() == o.parse_table_bytes(data)


def test_too_long_line_is_fatal(host_ctx):
    from hashcat_a5_table_generator_amd import A5xError
    host_ctx.clear_table()
    with pytest.raises(A5xError) as e:
        host_ctx.parse_table(b"a=b\n" + b"x" * 70000 + b"\n")
    assert "TOOLONG" in str(e.value)


def test_random_tables_fuzz(host_ctx):
    rng = random.Random(3)
    alphabet = b"ab=#$HEX[]0f \t\r\n" + "à€".encode()
    for _ in range(300):
        data = bytes(rng.choice(alphabet) for _ in range(rng.randint(0, 80)))
        host_ctx.clear_table()
        try:
            ref = o.parse_table_bytes(data)
        except o.ScanTooLong:
            continue
        host_ctx.parse_table(data)
        assert host_ctx.table() == ref, data


@pytest.mark.parametrize("data", [b"", b"a", b"a\n", b"a\r\nb", b"\n\n", b"x\r\r\n", "αβ\r\n".encode(),
                                  b"w\n" + b"x" * 65536 + b"\nafter", b"w\n" + b"y" * 65535 + b"\nz"])
def test_split_words(data):
    from hashcat_a5_table_generator_amd import split_words
    words, offs = split_words(data)
    got = [bytes(words[int(offs[i]):int(offs[i + 1])]) for i in range(len(offs) - 1)]
    assert got == o.read_words(data)


def _plan_rc(nkeys):
    """Compile a table of nkeys 2-byte keys (one 2-byte value each) on a host-only context."""
    import ctypes
    from hashcat_a5_table_generator_amd import _lib
    L = _lib.load()
    h = ctypes.c_void_p()
    assert L.a5x_create(-1, ctypes.byref(h)) == 0
    keys = [bytes([97 + i // 26, 97 + i % 26]) for i in range(nkeys)]
    txt = b"".join(k + b"=" + k.upper() + b"\n" for k in keys)
    assert L.a5x_parse_table(h, txt, len(txt)) == 0
    info = np.zeros(4, dtype=np.uint64)
    rc = L.a5x_debug_plan_word(h, b"ab" + b"\0" * 16, 2, 0, 15, None, 0, info.ctypes.data)
    err = L.a5x_last_error(h)
    L.a5x_destroy(h)
    return rc, err


def test_device_table_size_cap():
    """the compiled device table (keys, choices, the lookup arrays, blob) is staged
    into LDS per workgroup and capped at 32 KiB (A5X_TABLE_LDS_MAX): 409 two-byte keys with
    one two-byte value each fit, 410 are refused with A5X_E_UNSUPPORTED naming the size (no
    silent fallback); every shipped table and the czech+german merge are far below."""
    assert _plan_rc(409)[0] == 0
    rc, err = _plan_rc(410)
    assert rc == -9 and b"LDS staging max 32768" in err
