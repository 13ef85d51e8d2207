"""Per-phase cycle breakdown of k_expand_fast (diagnostic build: A5X_LIB_PATH=.../_build_diag/liba5x.so)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("A5X_LIB_PATH", os.path.join(ROOT, "hashcat_a5_table_generator_amd", "_build_diag", "liba5x.so"))
from hashcat_a5_table_generator_amd import Context, DeviceBuffer, _lib, synth  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "c3"
nwords = int(sys.argv[2]) if len(sys.argv) > 2 else 2_000_000
tables, (data, offs) = synth.config_words(wl, nwords)
ctx = Context(0)
ctx.load_tables([os.path.join(ROOT, "tests", "golden", "tables", t + ".table") for t in tables])
dw, do = DeviceBuffer.from_array(ctx, data), DeviceBuffer.from_array(ctx, offs)
n = len(offs) - 1
tc, tb = ctx.keyspace_device(dw.ptr, do.ptr, n)
out = DeviceBuffer(ctx, tb)
ctx.expand_device(dw.ptr, do.ptr, n, out.ptr, tb)
buf = (ctypes.c_ulonglong * 16)()
L = _lib.load()
assert L.a5x_debug_stamps(buf, 1) == 0, "not a diagnostic build"
st = ctx.expand_device(dw.ptr, do.ptr, n, out.ptr, tb)
assert L.a5x_debug_stamps(buf, 1) == 0
names = ["meta", "big entries", "prefix/open", "rounds", "records load", "fb_R/wi/prefetch", "close", "-", "-"]
tot = sum(buf[i] for i in range(9))
print(f"{wl}: {n} words {tc} cands, expand {st['ms_expand']:.2f} ms; wave-cycles total {tot:.3e}")
for i, nm in enumerate(names):
    print(f"  {nm:14s} {buf[i] / tot * 100:6.2f} %   {buf[i] / max(tc, 1) * 64:8.1f} cycles per 64 candidates")
