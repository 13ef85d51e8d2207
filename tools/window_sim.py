"""Window statistics of k_expand_fast on a workload (CPU simulation from the host
plan of every word): words / records / big entries / candidates per window, for
the window limits in a5x_kernels.hip (FX_WW words, FX_ZSLOT record u64, FX_ZBE big
entries) and the chunk size.

    python tools/window_sim.py c3 100000 [chunk] [ww] [wrec] [nbe]
"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from hashcat_a5_table_generator_amd import _lib, synth  # noqa: E402

FAST = 1 << 5


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "c3"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 100000
    CH = int(sys.argv[3]) if len(sys.argv) > 3 else 8192
    WW = int(sys.argv[4]) if len(sys.argv) > 4 else 32
    WREC = int(sys.argv[5]) if len(sys.argv) > 5 else 255
    NBE = int(sys.argv[6]) if len(sys.argv) > 6 else 255
    tables, (data, offs) = synth.config_words(wl, n)
    L = _lib.load()
    h = ctypes.c_void_p()
    assert L.a5x_create(-1, ctypes.byref(h)) == 0
    root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden", "tables")
    for t in tables:
        assert L.a5x_load_table_file(h, os.path.join(root, t + ".table").encode()) == 0
    info = np.zeros(4, dtype=np.uint64)
    buf = data.tobytes()
    cnt = np.zeros(n, np.int64)
    rs = np.zeros(n, np.int64)
    be = np.zeros(n, np.int64)
    fast = np.zeros(n, bool)
    for i in range(n):
        w = buf[offs[i]:offs[i + 1]]
        rc = L.a5x_debug_plan_word(h, w + b"\0" * 16, len(w), 0, 15, None, 0, info.ctypes.data)
        assert rc == 0
        f = int(info[2]) & 0xFFFFFFFF
        cnt[i] = int(info[0])
        if f & FAST and cnt[i] > 0:
            fast[i] = True
            np_, ne = (f >> 24) & 31, (f >> 16) & 255
            rs[i] = 1 + np_ + ne
            be[i] = (int(info[2]) >> 40) & 0xFFFF
    L.a5x_destroy(h)
    c0 = np.concatenate([[0], np.cumsum(cnt)])
    total = int(c0[-1])
    # walk chunks like k_expand_fast
    wins = []  # (words, rec, ents, cands)
    w = 0
    for ch in range((total + CH - 1) // CH):
        g0, g1 = ch * CH, min(total, (ch + 1) * CH)
        while c0[w + 1] <= g0:
            w += 1
        g = g0
        while g < g1:
            if not fast[w] or cnt[w] == 0:
                g = max(g, min(int(c0[w + 1]), g1))
                w += 1
                continue
            k, r, e = 0, 0, 0
            while (w + k < n and k < WW and fast[w + k] and c0[w + k] < g1 and cnt[w + k] > 0
                   and r + rs[w + k] < WREC and e + be[w + k] <= NBE):
                r += rs[w + k]; e += be[w + k]; k += 1
            k = max(k, 1)
            gend = min(g1, int(c0[w + k]))
            wins.append((k, r, e, gend - g))
            g = gend
            w += k
        w = max(w - 1, 0)
        while w > 0 and c0[w] > g1:
            w -= 1
    a = np.array(wins, dtype=np.float64)
    print(f"{wl}: {n} words, {total} candidates, chunk {CH}: {len(wins)} windows "
          f"({len(wins) / n:.3f} per word, {total / len(wins):.0f} candidates per window)")
    print(f"  mean words {a[:, 0].mean():.1f}  records {a[:, 1].mean():.0f} u64  big entries {a[:, 2].mean():.0f}"
          f"  | word mean rs {rs[fast].mean():.1f}  bent {be[fast].mean():.1f}")
    lim = {"words": (a[:, 0] >= WW).mean(), "rec": (a[:, 1] + 40 >= WREC).mean(), "ent": (a[:, 2] + 60 >= NBE).mean()}
    print("  near-limit fraction:", {k: round(v, 3) for k, v in lim.items()})


if __name__ == "__main__":
    main()
