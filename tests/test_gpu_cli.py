"""End to end through the CLI replica (csrc/a5x_cli.cpp, main.go:17-100) and
engine.generate: a C1-shaped dictionary FILE (configs[0]: qwerty-azerty x 10k
[a-z0-9] words) in all four modes; stdout must hold, word after word, exactly the
C oracle's candidate multiset of each word (oracle/a5_oracle.c: main.go:168-440).
Also the --hashes mode: "hash:plain" lines for planted MD5 / NTLM
targets, as hashcat would report them (README.MD:74-106)."""
import io
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, table_path

pytestmark = pytest.mark.gpu

CLI = os.path.join(ROOT, "hashcat_a5_table_generator_amd", "_build", "a5x_generator")
MODES = [(0, []), (1, ["-r"]), (2, ["-s"]), (3, ["-s", "-r"])]


@pytest.fixture(scope="module")
def dict_file(tmp_path_factory):
    """10k C1 words plus the scanner's edge cases: a CRLF line, an empty line, a
    line with spaces (kept: main.go:73 uses scanner.Text() without trimming)."""
    from hashcat_a5_table_generator_amd import synth
    _, (d, o) = synth.config_words("c1", 10000, seed=0xC1)
    words = [bytes(d[int(o[i]):int(o[i + 1])]) for i in range(len(o) - 1)]
    body = b"\n".join(words[:5000]) + b"\nqwerty\r\n\nazerty qwerty\n" + b"\n".join(words[5000:]) + b"\n"
    p = tmp_path_factory.mktemp("c1") / "dict.txt"
    p.write_bytes(body)
    return str(p), body


def _oracle_words(body):
    from hashcat_a5_table_generator_amd import split_words
    return split_words(body)


def _per_word_check(stdout, words, offs, mode, tables, mn=0, mx=15):
    from oracle import c_oracle as co
    want, wb = co.CTable([table_path(t) for t in tables]).expand_batch(words, offs, mode, mn, mx)
    assert len(stdout) == len(want), (len(stdout), len(want))
    pos = 0
    for i in range(len(offs) - 1):
        n = int(wb[i])
        g, w = stdout[pos:pos + n], want[pos:pos + n]
        if g != w:  # same multiset per word (the library's order inside a word may differ)
            assert sorted(g.split(b"\n")) == sorted(w.split(b"\n")), bytes(words[int(offs[i]):int(offs[i + 1])])
        pos += n


@pytest.mark.parametrize("mode,flags", MODES)
def test_cli_replica_end_to_end(dict_file, mode, flags):
    path, body = dict_file
    r = subprocess.run([CLI, path, "-t", table_path("qwerty-azerty"), *flags], stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, timeout=120)
    assert r.returncode == 0, r.stderr.decode(errors="replace")[-2000:]
    words, offs = _oracle_words(body)
    _per_word_check(r.stdout, words, offs, mode, ["qwerty-azerty"])


@pytest.mark.parametrize("mode", [0, 2])
def test_engine_generate_end_to_end(dict_file, mode):
    from hashcat_a5_table_generator_amd import generate
    path, body = dict_file
    out = io.BytesIO()
    n = generate(path, [table_path("qwerty-azerty")], substitute_all=mode >= 2, reverse_sub=bool(mode & 1), out=out,
                 batch_words=3000, chunk=4099)  # several batches, read in many small chunks
    words, offs = _oracle_words(body)
    _per_word_check(out.getvalue(), words, offs, mode, ["qwerty-azerty"])
    assert n == out.getvalue().count(b"\n")


@pytest.mark.parametrize("algo", ["md5", "ntlm"])
def test_cli_hashes_mode_reports_hash_plain(tmp_path, algo):
    """--hashes: every planted digest is reported once as hash:plain (first candidate in
    stream order), random digests never; non-printable plains come out as $HEX[...]."""
    from hashcat_a5_table_generator_amd import Context, format_plain
    from oracle import digest_oracle as dg
    f = dg.ALGOS[0 if algo == "md5" else 1]
    rng = np.random.default_rng(7)
    words = [bytes(rng.choice(list(b"abcdefghijklmnopqrstuvwxyz"), size=int(rng.integers(3, 10))).astype(np.uint8))
             for _ in range(3000)]
    words += [b"za\x01q", b"\xffqa"]  # plains with a control byte / invalid UTF-8
    (tmp_path / "d.txt").write_bytes(b"\n".join(words) + b"\n")
    with Context(0) as c:
        c.load_tables([table_path("qwerty-azerty")])
        per_word = c.expand_words(words, 0, 0, 15)
    planted = {}
    for w in list(rng.choice(3000, size=60, replace=False)) + [3000, 3001]:
        if per_word[w]:
            cand = per_word[w][int(rng.integers(0, len(per_word[w])))]
            planted[f(cand)] = cand
    lines = [d.hex() for d in planted] + [bytes(rng.integers(0, 256, 16, dtype=np.uint8)).hex() for _ in range(500)]
    lines += ["not-a-hash", planted and next(iter(planted)).hex().upper() + ":potfile-plain"]
    (tmp_path / "h.txt").write_text("\n".join(lines) + "\n")
    r = subprocess.run([CLI, str(tmp_path / "d.txt"), "-t", table_path("qwerty-azerty"), "--hashes",
                        str(tmp_path / "h.txt"), "--algo", algo], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                       timeout=120)
    assert r.returncode == 0, r.stderr.decode(errors="replace")[-2000:]
    got = r.stdout.split(b"\n")[:-1]
    want = {d.hex().encode() + b":" + format_plain(p) for d, p in planted.items()}
    assert set(got) == want and len(got) == len(want)
    assert any(b"$HEX[" in x for x in got)
    assert b"1 line(s)" in r.stderr


def test_cli_streams_dictionary_in_chunks(tmp_path):
    """The dictionary is read in bounded chunks (ScanLines across chunk edges, CRLF,
    empty lines) and expanded in small batches by the two-context pipeline, in batch
    order; the first line with no newline in 64 KiB ends the input silently, as the
    reference's unchecked bufio.Scanner does (main.go:72-74)."""
    from hashcat_a5_table_generator_amd import synth
    _, (d, o) = synth.config_words("c1", 6000, seed=0xC11)
    words = [bytes(d[int(o[i]):int(o[i + 1])]) for i in range(len(o) - 1)]
    body = b"\n".join(words[:4000]) + b"\nab\r\n\n" + b"\n".join(words[4000:]) + b"\n"
    long_line = b"q" * (64 * 1024) + b"\n"
    full = body + long_line + b"never\nseen\n"
    p = tmp_path / "d.txt"
    p.write_bytes(full)
    env = dict(os.environ, A5X_CLI_CHUNK="4099", A5X_CLI_BATCH="700")
    r = subprocess.run([CLI, str(p), "-t", table_path("qwerty-azerty")], stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, timeout=120, env=env)
    assert r.returncode == 0, r.stderr.decode(errors="replace")[-2000:]
    ow, oo = _oracle_words(full)  # split_words stops at the long line too
    assert len(oo) - 1 == 6002  # 6000 words + "ab" + ""
    # batch order is kept, so the stream is the per-word concatenation
    _per_word_check(r.stdout, ow, oo, 0, ["qwerty-azerty"])


def test_cli_hashes_long_potfile_line(tmp_path):
    """A --hashes line longer than any fixed buffer (a potfile line with a 10 KB plain)
    is one line: its digest is loaded once, no piece of it becomes a target."""
    from oracle import digest_oracle as dg
    (tmp_path / "d.txt").write_bytes(b"qa\n")
    d = dg.md5(b"aa")  # qwerty-azerty: q -> a
    piece = dg.md5(b"zz").hex()
    lines = [d.hex() + ":" + "x" * 5000 + piece + ":" + "y" * 5000]
    (tmp_path / "h.txt").write_text("\n".join(lines) + "\n")
    r = subprocess.run([CLI, str(tmp_path / "d.txt"), "-t", table_path("qwerty-azerty"), "--hashes",
                        str(tmp_path / "h.txt")], stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=120)
    assert r.returncode == 0, r.stderr.decode(errors="replace")[-2000:]
    assert r.stdout == d.hex().encode() + b":aa\n"
    assert b"line(s)" not in r.stderr


@pytest.mark.parametrize("mode,flags", [(0, []), (2, ["-s"]), (3, ["-s", "-r"])])
def test_cli_resume_cursor(dict_file, mode, flags):
    """--keyspace prints the stream's candidate count; --skip N --limit M prints exactly
    lines [N, N + M) of the full stream (SURVEY §5 checkpoint / resume), whatever the
    batching: the cursor run uses other batch sizes than the full run, so this also pins
    the batch-independent candidate order of every word."""
    path, _ = dict_file
    base = [CLI, path, "-t", table_path("qwerty-azerty"), *flags]
    full = subprocess.run(base, stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=120)
    assert full.returncode == 0, full.stderr.decode(errors="replace")[-2000:]
    lines = full.stdout.split(b"\n")[:-1]
    env = dict(os.environ, A5X_CLI_BATCH="1500", A5X_CLI_CHUNK="9001")
    ks = subprocess.run(base + ["--keyspace"], stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=120, env=env)
    assert ks.returncode == 0 and int(ks.stdout) == len(lines)
    n = len(lines)
    for skip, limit in [(0, 1), (1, 1000), (n // 3, n // 2), (n - 7, 100), (n + 5, 10), (12345, None)]:
        args = ["--skip", str(skip)] + ([] if limit is None else [f"--limit={limit}"])
        r = subprocess.run(base + args, stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=120, env=env)
        assert r.returncode == 0, r.stderr.decode(errors="replace")[-2000:]
        want = lines[skip:] if limit is None else lines[skip:skip + limit]
        assert r.stdout == b"".join(x + b"\n" for x in want), (skip, limit)
    bad = subprocess.run(base + ["--skip", "-3"], stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=60)
    assert bad.returncode == 80


def test_expand_range_windows_concatenate(dict_file):
    """Context.expand over candidate windows (a5x_expand_range) cut inside words: the
    windows concatenate to the full batch output."""
    from hashcat_a5_table_generator_amd import Context, split_words
    _, body = dict_file
    words, offs = split_words(body)
    with Context(0) as c:
        c.load_tables([table_path("qwerty-azerty")])
        for mode in (0, 1, 2):
            full, st = c.expand(words, offs, mode)
            T = st["candidates"]
            cuts = sorted({0, T, 1, T // 7, T // 2 + 3, T - 1})
            parts = [c.expand(words, offs, mode, cand_begin=a, cand_end=b)[0] for a, b in zip(cuts, cuts[1:])]
            assert b"".join(parts) == full, mode
