"""Generate tests/golden/golden.json from the Python oracle (oracle/a5_oracle.py).

The reference ships no tests, so the oracle itself is pinned
by SURVEY.md Appendix B (tests/test_oracle_golden.py) and analytic identities;
this script freezes its outputs for the cases below so the GPU tests on the box
(where /root/reference does not exist) compare against committed data.

    python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from oracle import a5_oracle as o  # noqa: E402

TABLES = ["czech", "german", "greek-hebrew", "qwerty-azerty", "qwerty-cyrillic", "qwerty-greek"]


def load(names):
    return o.load_tables([os.path.join(HERE, "tables", n + ".table") for n in names])


def sha(cands):
    return hashlib.sha256(b"".join(sorted(c + b"\n" for c in cands))).hexdigest()


def main():
    rng = random.Random(0x5A5)
    words = {
        "ascii": [b"hello", b"password", b"abcdefghijklmnopq", b"strasse", b"aqua", b"m,;1", b"kalimera",
                  b"", b"a", b"ss", b"sss", b"Zz", b"1234567890", b"qwertyuiop", b"P@ssw0rd!", b"\xff\xfe",
                  b"mississippi", b"STRASSE", b"abc;'.,"],
        "greek": ["καλημέρα".encode(), "αλφα".encode(), "καλημέρα;".encode(), "ψυχή".encode()],
    }
    for _ in range(40):
        L = rng.randint(1, 12)
        words["ascii"].append(bytes(rng.choice(b"abcdefghijklmnopqrstuvwxyz0123456789;,.'") for _ in range(L)))
    cases = []
    combos = [[t] for t in TABLES] + [["czech", "german"], ["czech", "czech"], ["qwerty-azerty", "qwerty-cyrillic"]]
    windows = [(0, 15), (2, 3), (5, 5), (0, 1), (1, 2), (3, 15), (-1, 15), (0, 0)]
    for tabs in combos:
        sub = load(tabs)
        for w in words["ascii"] + words["greek"]:
            for (mn, mx) in windows:
                for mode in range(4):
                    if mode != 0 and (mn, mx) not in [(0, 15), (2, 3)]:
                        continue
                    try:
                        c = o.expand(w, sub, mode, mn, mx)
                        err = None
                    except o.GoPanic:
                        c, err = [], "panic"
                    if len(c) > 200000:
                        continue
                    cases.append({"tables": tabs, "word": w.hex(), "mode": mode, "min": mn, "max": mx,
                                  "count": len(c), "bytes": sum(len(x) + 1 for x in c), "sha256": sha(c),
                                  "error": err})
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py (oracle/a5_oracle.py)", "cases": cases}, f,
                  indent=0, separators=(",", ":"))
    print(len(cases), "cases")


if __name__ == "__main__":
    main()
