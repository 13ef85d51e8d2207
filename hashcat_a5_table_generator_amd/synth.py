"""Seeded synthetic word lists for the BASELINE.json configs.

``greek-dictionary.txt`` is missing from the reference snapshot
(``.MISSING_LARGE_BLOBS:1``), and there is no network, so every benchmark and
scale test runs on these generators (numpy PCG64, fixed seeds).
Output layout = the ABI batch layout: contiguous bytes (+16 B pad) and n+1
u64 offsets.
"""
from __future__ import annotations

from typing import Tuple

import numpy as np

GREEK = np.array([0x3B1 + i for i in range(25)], dtype=np.int64)  # α..ω


def _pack(lengths: np.ndarray, data: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    offs = np.zeros(len(lengths) + 1, dtype=np.uint64)
    np.cumsum(lengths, out=offs[1:])
    out = np.zeros(len(data) + 16, dtype=np.uint8)
    out[: len(data)] = data
    return out, offs


def words_from_alphabet(n: int, lmin: int, lmax: int, alphabet: bytes, seed: int) -> Tuple[np.ndarray, np.ndarray]:
    rng = np.random.default_rng(seed)
    lengths = rng.integers(lmin, lmax + 1, size=n, dtype=np.int64)
    alpha = np.frombuffer(alphabet, dtype=np.uint8)
    data = alpha[rng.integers(0, len(alpha), size=int(lengths.sum()), dtype=np.int64)]
    return _pack(lengths, data)


def words_az(n: int, lmin: int = 6, lmax: int = 12, seed: int = 0x5A5) -> Tuple[np.ndarray, np.ndarray]:
    """[a-z] words, length U[lmin, lmax] (C3, C4 with lmin=lmax=10, C2 ASCII variant)."""
    return words_from_alphabet(n, lmin, lmax, b"abcdefghijklmnopqrstuvwxyz", seed)


def words_az09(n: int, lmin: int = 6, lmax: int = 12, seed: int = 0x5A5) -> Tuple[np.ndarray, np.ndarray]:
    """[a-z0-9] words (C1)."""
    return words_from_alphabet(n, lmin, lmax, b"abcdefghijklmnopqrstuvwxyz0123456789", seed)


def words_greek(n: int, lmin: int = 6, lmax: int = 12, seed: int = 0x5A5) -> Tuple[np.ndarray, np.ndarray]:
    """Greek [α-ω] words of lmin..lmax letters (2 UTF-8 bytes each; C2, C5)."""
    rng = np.random.default_rng(seed)
    letters = rng.integers(lmin, lmax + 1, size=n, dtype=np.int64)
    cps = GREEK[rng.integers(0, len(GREEK), size=int(letters.sum()), dtype=np.int64)]
    b0 = (0xC0 | (cps >> 6)).astype(np.uint8)
    b1 = (0x80 | (cps & 0x3F)).astype(np.uint8)
    data = np.stack([b0, b1], axis=1).reshape(-1)
    return _pack(letters * 2, data)


def words_az_huge(n: int, lmin: int = 10, lmax: int = 10, seed: int = 0x5A5, every: int = 20000,
                  huge: int = 24) -> Tuple[np.ndarray, np.ndarray]:
    """C4's length-10 [a-z] words with every ``every``-th word (by position in the block)
    ``huge`` letters long: 2^huge - 1 candidates under qwerty-cyrillic, one word larger than a
    rank's share (the intra-word split of SURVEY 8(e) e1)."""
    rng = np.random.default_rng(seed)
    lengths = rng.integers(lmin, lmax + 1, size=n, dtype=np.int64)
    lengths[every // 3::every] = huge
    alpha = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz", dtype=np.uint8)
    data = alpha[rng.integers(0, len(alpha), size=int(lengths.sum()), dtype=np.int64)]
    return _pack(lengths, data)


CONFIGS = {
    # name: (tables, generator, kwargs, description)
    "c1": (["qwerty-azerty"], words_az09, {"lmin": 6, "lmax": 12},
           "qwerty-azerty x 10k [a-z0-9] words len U[6,12] (configs[0], CPU plumbing)"),
    "c2": (["qwerty-greek"], words_greek, {"lmin": 6, "lmax": 12},
           "qwerty-greek x synthetic Greek words len U[6,12] (configs[1]; 0 candidates: keys are ASCII)"),
    "c2a": (["qwerty-greek"], words_az, {"lmin": 6, "lmax": 12},
            "qwerty-greek x [a-z] words len U[6,12] (configs[1] ASCII variant, multi-byte output)"),
    "c3": (["czech", "german"], words_az, {"lmin": 6, "lmax": 12},
           "czech+german x synthetic [a-z] words len U[6,12] (configs[2])"),
    "c4": (["qwerty-cyrillic"], words_az, {"lmin": 10, "lmax": 10},
           "qwerty-cyrillic x synthetic [a-z] words len 10 (configs[3], 1023 cand/word)"),
    "c4h": (["qwerty-cyrillic"], words_az_huge, {"lmin": 10, "lmax": 10},
            "qwerty-cyrillic x C4 words with a 24-letter word every 20000 (intra-word shard split test)"),
    "c5": (["greek-hebrew"], words_greek, {"lmin": 6, "lmax": 12},
           "greek-hebrew x synthetic Greek words len U[6,12] (configs[4] expansion stage)"),
}


def config_words(name: str, n: int, seed: int = 0x5A5):
    tables, gen, kw, _ = CONFIGS[name]
    return tables, gen(n, seed=seed, **kw)


GLOBAL_BLOCK = 1 << 20  # words per independently seeded block of a global list


def global_words(name: str, w0: int, w1: int, seed: int = 0x5A5):
    """Words [w0, w1) of ONE unbounded deterministic list for config ``name``.

    The list is made of GLOBAL_BLOCK-word blocks, block b generated with seed
    (seed, b), so any rank can build any slice of the global list without the
    rest (bench.py's north_star partition: one list, split by byte prefix)."""
    tables, gen, kw, _ = CONFIGS[name]
    parts, lens = [], []
    b = w0 // GLOBAL_BLOCK
    while b * GLOBAL_BLOCK < w1:
        data, offs = gen(GLOBAL_BLOCK, seed=int(np.random.SeedSequence([seed, b]).generate_state(1)[0]), **kw)
        lo = max(w0, b * GLOBAL_BLOCK) - b * GLOBAL_BLOCK
        hi = min(w1, (b + 1) * GLOBAL_BLOCK) - b * GLOBAL_BLOCK
        parts.append(data[int(offs[lo]):int(offs[hi])])
        lens.append(np.diff(offs[lo:hi + 1].astype(np.int64)))
        b += 1
    lengths = np.concatenate(lens) if lens else np.zeros(0, dtype=np.int64)
    body = np.concatenate(parts) if parts else np.zeros(0, dtype=np.uint8)
    return tables, _pack(lengths, body)
