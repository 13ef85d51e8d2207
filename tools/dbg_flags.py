"""Debug: device keyspace flags/counts of the parity test's random words (GPU)."""
import sys, zlib
import numpy as np
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests')
from conftest import table_path
from hashcat_a5_table_generator_amd import Context
from hashcat_a5_table_generator_amd.engine import pack_words
tabs = sys.argv[1].split(",")
lo, hi = int(sys.argv[2]), int(sys.argv[3])
rng = np.random.default_rng(zlib.crc32(",".join(tabs).encode()))
alpha = list(b"abcdefghijklmnopqrstuvwxyzAEOUSZ0123456789;,.'\"`-=")
alpha += list("αβγδεζηθικλμνξοπρστυφχψω".encode())
words = [np.asarray(rng.choice(alpha, size=int(rng.integers(0, 14))), dtype=np.uint8).tobytes() for _ in range(2000)]
c = Context(0)
c.load_tables([table_path(t) for t in tabs])
data, offs = pack_words(words)
for mn, mx in [(0, 15), (2, 4), (1, 3)]:
    cnt, byt = c.keyspace(data, offs, 0, mn, mx)
    fl = c.last_flags() if hasattr(c, "last_flags") else None
    c0 = np.concatenate([[0], np.cumsum(cnt)])
    print("case", mn, mx, "total", int(c0[-1]))
    for i in range(lo, hi):
        print(" ", i, int(c0[i]), int(cnt[i]), words[i])
