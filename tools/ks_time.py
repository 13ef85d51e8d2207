"""Time the keyspace pass (device) for a table set over a synthetic word batch (GPU box).

    [KSMODE=m] python tools/ks_time.py [workload] [words] [table ...]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hashcat_a5_table_generator_amd import Context, DeviceBuffer, synth  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "c3"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 10_000_000
tables, (data, offs) = synth.config_words(wl, n)
if len(sys.argv) > 3:
    tables = sys.argv[3:]
ctx = Context(0)
ctx.load_tables([os.path.join(ROOT, "tests", "golden", "tables", t + ".table") for t in tables])
dw, do = DeviceBuffer.from_array(ctx, data), DeviceBuffer.from_array(ctx, offs)
mode = int(os.environ.get("KSMODE", "0"))
ctx.keyspace_device(dw.ptr, do.ptr, n, mode=mode)
best = 1e9
for _ in range(5):
    t0 = time.perf_counter()
    tc, tb = ctx.keyspace_device(dw.ptr, do.ptr, n, mode=mode)
    best = min(best, time.perf_counter() - t0)
print(f"{wl} {tables}: {n} words -> {tc} candidates; keyspace_device {best * 1e3:.2f} ms (host wall, incl. sync)")
