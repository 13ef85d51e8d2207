"""Debug helper (GPU box): expand a small synthetic batch on the device and print
the first words whose output differs from the oracle (byte-level)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hashcat_a5_table_generator_amd import Context, DeviceBuffer, synth  # noqa: E402
from oracle import a5_oracle as o  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "c3"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 300
tables, (data, offs) = synth.config_words(wl, n)
tp = [os.path.join(ROOT, "tests", "golden", "tables", t + ".table") for t in tables]
sub = o.load_tables(tp)
ctx = Context(0)
ctx.load_tables(tp)
dw, do = DeviceBuffer.from_array(ctx, data), DeviceBuffer.from_array(ctx, offs)
tc, tb = ctx.keyspace_device(dw.ptr, do.ptr, n)
out = DeviceBuffer(ctx, tb + 64)
boff = DeviceBuffer(ctx, (n + 1) * 8)
ctx.expand_device(dw.ptr, do.ptr, n, out.ptr, tb, d_byte_off=boff.ptr)
got = out.to_array(np.uint8, tb).tobytes()
bo = boff.to_array(np.uint64, n + 1)
co = DeviceBuffer(ctx, (n + 1) * 8)
ctx.keyspace_device(dw.ptr, do.ptr, n, d_cand_off=co.ptr) if False else None
import collections
cnts = [len(o.process_word(bytes(data[offs[i]:offs[i + 1]]), sub, 0, 15)) for i in range(n)]
cof = np.concatenate([[0], np.cumsum(cnts)])
bad = 0
for i in range(n):
    w = bytes(data[offs[i]:offs[i + 1]])
    ref = o.process_word(w, sub, 0, 15)
    seg = got[bo[i]:bo[i + 1]]
    want = b"".join(sorted(x + b"\n" for x in ref))
    if sorted(seg.split(b"\n")[:-1]) != sorted(ref) or not seg.endswith(b"\n") and ref:
        bad += 1
        if bad <= 4:
            print(f"word {i} {w!r}: {len(ref)} cands, {len(want)} B; got {len(seg)} B (off {bo[i]}) cand_off {cof[i]} chunk-rel {cof[i] % int(os.environ.get('A5X_CHUNK', '32768'))}")
            gl = seg.split(b"\n")
            print("   got first:", gl[:6])
            print("   ref first:", ref[:6])
print(f"{bad} bad words of {n}")
