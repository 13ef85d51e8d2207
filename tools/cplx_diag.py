"""Which C3 words make k_keyspace_cplx slow (GPU box).  Needs a diagnostic liba5x built from a local
edit of k_keyspace_cplx (not kept in the sources): s_memtime at the top of the per-word loop, and at the end
count[w] = 0xC0FFEE, bytes[w] = the elapsed ticks.  Result: profiles/r06fz_cplx_word_cycles_c3.txt.

    A5X_LIB_PATH=.../_build_cdiag/liba5x.so python tools/cplx_diag.py [words]
"""
import collections
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hashcat_a5_table_generator_amd import Context, synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
tables, (data, offs) = synth.config_words("c3", n)
with Context(0) as c:
    c.load_tables([os.path.join(ROOT, "tests", "golden", "tables", t + ".table") for t in tables])
    cnt, byt = c.keyspace(data, offs, 0, 0, 15)
byt = np.asarray(byt, dtype=np.int64)
idx = np.nonzero(np.asarray(cnt, dtype=np.int64) == 0xC0FFEE)[0]
cyc = byt[idx]
print(f"{n} words, {len(idx)} complex; cycles: mean {cyc.mean():.0f} median {np.median(cyc):.0f} "
      f"p99 {np.percentile(cyc, 99):.0f} max {cyc.max()}; sum {cyc.sum():.3e}")
order = np.argsort(-cyc)
for k in order[:40]:
    w = int(idx[k])
    print(f"{cyc[k]:>10d}  {bytes(data[offs[w]:offs[w + 1]]).decode(errors='replace')}")
hist = collections.Counter(int(np.log2(max(1, x))) for x in cyc)
print("log2(cycles) histogram:", sorted(hist.items()))
