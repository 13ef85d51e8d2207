"""The streamed dictionary (engine.iter_word_batches; the CLI's DictStream is the same
rule in C++): ScanLines over bounded chunks must give exactly the words of a scan over
the whole file (a5x_split_words, main.go:72-74), at every chunk and batch size --
CRLF across chunk edges, empty lines, an unterminated last line, and the first line
with no newline in 64 KiB ending the input (bufio.ErrTooLong, never checked)."""
import io

import numpy as np
import pytest

from hashcat_a5_table_generator_amd import engine, split_words


def _words(data):
    w, o = split_words(data)
    return [bytes(w[int(o[i]):int(o[i + 1])]) for i in range(len(o) - 1)]


def _streamed(data, batch, chunk):
    out = []
    for w, o in engine.iter_word_batches(io.BytesIO(data), batch, chunk):
        assert len(o) - 1 <= batch and len(w) == int(o[-1]) + 16
        out += [bytes(w[int(o[i]):int(o[i + 1])]) for i in range(len(o) - 1)]
    return out


def _dict(rng, n):
    parts = []
    for _ in range(n):
        r = rng.random()
        if r < 0.05:
            parts.append(b"")
        else:
            parts.append(bytes(rng.integers(97, 123, size=int(rng.integers(1, 14)), dtype=np.uint8)))
        if rng.random() < 0.1:
            parts[-1] += b"\r"
    return b"\n".join(parts)


@pytest.mark.parametrize("chunk", [1, 3, 7, 64, 1000, 1 << 20])
@pytest.mark.parametrize("batch", [1, 5, 333, 1 << 22])
def test_stream_equals_whole_scan(chunk, batch):
    rng = np.random.default_rng(chunk * 31 + batch)
    data = _dict(rng, 400)
    for tail in (b"", b"\n", b"\r\n", b"end"):
        d = data + tail
        assert _streamed(d, batch, chunk) == _words(d)


@pytest.mark.parametrize("chunk", [100, 4099, 70000, 1 << 20])
def test_stream_stops_at_a_64k_line(chunk):
    rng = np.random.default_rng(5)
    head = _dict(rng, 300) + b"\n"
    for L in (65535, 65536, 200000):
        d = head + b"x" * L + b"\nafter\n"
        want = _words(d)
        assert _streamed(d, 64, chunk) == want
        assert (b"after" in want) == (L < 65536)
