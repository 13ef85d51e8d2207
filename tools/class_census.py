"""Host-side class census of a workload's words (a5x_debug_plan_word, classification
only): how many words/candidates take the FAST kernel vs the per-word path, and a
sample of the non-FAST words with their counts.  CPU only.

    python tools/class_census.py c3 200000
"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from hashcat_a5_table_generator_amd import _lib, synth  # noqa: E402

FAST, DEFER, RADIX = 1 << 5, 1 << 4, 1 << 0


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "c3"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 200000
    tables, (data, offs) = synth.config_words(wl, n)
    L = _lib.load()
    h = ctypes.c_void_p()
    assert L.a5x_create(-1, ctypes.byref(h)) == 0
    root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden", "tables")
    for t in tables:
        assert L.a5x_load_table_file(h, os.path.join(root, t + ".table").encode()) == 0
    info = np.zeros(4, dtype=np.uint64)
    buf = data.tobytes()
    tot = {"fast": [0, 0], "slow": [0, 0], "defer": [0, 0]}
    slow = []
    nbh, nbc = {}, {}
    for i in range(n):
        w = buf[offs[i]:offs[i + 1]]
        wb = w + b"\0" * 16
        rc = L.a5x_debug_plan_word(h, wb, len(w), 0, 15, None, 0, info.ctypes.data)
        assert rc == 0, L.a5x_last_error(h)
        f = int(info[2]) & 0xFFFFFFFF
        if f & FAST:
            nb = (int(info[2]) >> 32) & 0xFF
            nbh[nb] = nbh.get(nb, 0) + 1
            nbc[nb] = nbc.get(nb, 0) + int(info[0])
        k = "fast" if f & FAST else ("defer" if f & DEFER else "slow")
        tot[k][0] += 1
        tot[k][1] += int(info[0])
        if k != "fast":
            slow.append((int(info[0]), w, f))
    for k, (a, b) in tot.items():
        print(f"{k:6s} words {a:8d}  candidates {b:12d}")
    for nb in sorted(nbh):
        print(f"  FAST words with {nb} big pieces: {nbh[nb]:8d} words, {nbc[nb]:12d} candidates")
    slow.sort(reverse=True)
    for c, w, f in slow[:25]:
        print(f"  {c:10d}  {w!r:20s} flags {f:#010x}")
    L.a5x_destroy(h)


if __name__ == "__main__":
    main()
