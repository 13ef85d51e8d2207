"""hashcat-style plain formatting (a5x_format_plain) -- pure host code.

hashcat writes "hash:plain" lines and hexifies plains it cannot print as $HEX[...]
(the notation README.MD:171-176 documents for input).  hashcat is not part of the
reference, so the rule is restated (parity unpinned): hexify when the plain is not
valid UTF-8 (Go utf8 rules), contains a control byte (< 0x20, 0x7f) or has the
$HEX[...] form itself."""
import pytest

CASES = [
    (b"hello", b"hello"),
    (b"", b""),
    ("straße".encode(), "straße".encode()),           # valid UTF-8 stays
    ("שמשצשך30".encode(), "שמשצשך30".encode()),  # README.MD:168
    ("�".encode(), "�".encode()),                   # a literal U+FFFD is valid
    (b"a\x01b", b"$HEX[610162]"),                               # control byte
    (b"tab\there", b"$HEX[7461620968657265]"),
    (b"del\x7f", b"$HEX[64656c7f]"),
    (b"\xff", b"$HEX[ff]"),                                     # invalid byte
    (b"\xc3", b"$HEX[c3]"),                                     # truncated sequence
    (b"\xed\xa0\x80", b"$HEX[eda080]"),                         # UTF-16 surrogate
    (b"\xc0\xaf", b"$HEX[c0af]"),                               # overlong
    (b"$HEX[41]", b"$HEX[244845585b34315d]"),                   # would read back as 'A'
    (b"p:ss", b"p:ss"),                                          # the first ':' ends the hash
]


@pytest.mark.parametrize("plain,want", CASES)
def test_format_plain(plain, want):
    from hashcat_a5_table_generator_amd import format_plain
    assert format_plain(plain) == want


def test_format_plain_capacity():
    import ctypes
    from hashcat_a5_table_generator_amd import _lib
    L = _lib.load()
    n = ctypes.c_size_t()
    out = ctypes.create_string_buffer(4)
    assert L.a5x_format_plain(b"\xff\xfe", 2, out, 4, ctypes.byref(n)) == _lib.E_CAPACITY
    assert n.value == len(b"$HEX[fffe]")
