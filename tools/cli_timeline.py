#!/usr/bin/env python3
"""Host timeline of the CLI replica's stdout path (a5x_generator > /dev/null) on C3 words:
writes a dictionary of N synthetic words, runs the CLI with A5X_CLI_TIMELINE=1 and prints
its per-batch events plus the wall time and GB/s.  Usage: tools/cli_timeline.py [N] [extra CLI args]"""
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hashcat_a5_table_generator_amd import synth  # noqa: E402
from hashcat_a5_table_generator_amd.build import CLI  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
extra = sys.argv[2:]
tables, (data, offs) = synth.config_words("c3", n, seed=0x5A5)
lens = np.diff(offs.astype(np.int64))
body = np.frombuffer(bytes(data[: int(offs[-1])]), dtype=np.uint8)
text = np.empty(len(body) + n, dtype=np.uint8)
pos = np.arange(len(body)) + np.repeat(np.arange(n), lens)
text[pos] = body
text[np.cumsum(lens) + np.arange(n)] = 10
tp = [os.path.join(ROOT, "tests", "golden", "tables", t + ".table") for t in tables]
with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as td:
    d = os.path.join(td, "dict.txt")
    text.tofile(d)
    cmd = [CLI, d] + sum((["-t", t] for t in tp), []) + extra
    for rep in range(2):
        env = dict(os.environ, A5X_CLI_TIMELINE="1")
        t0 = time.perf_counter()
        with open(os.devnull, "wb") as dn:
            r = subprocess.run(cmd, stdout=dn, stderr=subprocess.PIPE, env=env)
        dt = time.perf_counter() - t0
        print(f"== run {rep}: rc {r.returncode} wall {dt:.3f} s", flush=True)
        print(r.stderr.decode(errors="replace"), flush=True)
