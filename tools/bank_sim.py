"""LDS bank model of k_expand_fast's ring placement on a workload's real candidate lengths
(CPU; MI355X_MICROARCH.md §LDS banking: ds_*_b32 in two 32-lane groups, bank (a/4) mod 32;
ds_*_b64 in four 16-lane groups; one cycle per extra address on a bank).

Rounds of 64 lanes x K=4 candidates, each candidate split into NB equal pieces (the plan's
big pieces), every piece OR-placed with wave-uniform dword counts (a5x_ring.h fx7_put).
Strategies: piece (the kernel), piece_swz (XOR-swizzled ring, FX_SWZ), piece_mask (exec-masked
ORs), piece_b64 (ds_or_b64), cand (whole candidates assembled in VGPRs), run (whole runs).

    python tools/bank_sim.py [workload] [words] [NB]
"""
import os
import random
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from hashcat_a5_table_generator_amd import synth  # noqa: E402
from oracle import a5_oracle as O  # noqa: E402  (test infrastructure: candidate lengths only)

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")


def swz(a):
    return a ^ ((a >> 3) & 0x70)


def cyc32(addrs):
    t = 0
    for h in (addrs[:32], addrs[32:]):
        bk = {}
        for a in h:
            if a is not None:
                bk.setdefault((a >> 2) & 31, set()).add(a)
        if bk:
            t += max(len(s) for s in bk.values())
    return t


def cyc64(addrs):
    t = 0
    for g in range(4):
        bk = {}
        for a in addrs[16 * g:16 * g + 16]:
            if a is not None:
                for d in (0, 4):
                    bk.setdefault(((a + d) >> 2) & 31, set()).add(a + d)
        if bk:
            t += max(len(s) for s in bk.values())
    return t


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "c3"
    nw = int(sys.argv[2]) if len(sys.argv) > 2 else 1200
    NB = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    tables, (data, offs) = synth.config_words(wl, nw)
    sub = O.load_tables([os.path.join(ROOT, "tests", "golden", "tables", t + ".table") for t in tables])
    b = data.tobytes()
    lens = np.array([len(c) + 1 for i in range(nw) for c in O.process_word(b[offs[i]:offs[i + 1]], sub, 0, 15)])
    random.seed(1)
    res = {}

    def add(k, arr, xfer):
        r = res.setdefault(k, [0, 0, 0])
        r[0] += 1
        r[1] += arr
        r[2] += max(arr, xfer)

    i = rounds = 0
    while i + 256 <= len(lens) and rounds < 300:
        L = lens[i:i + 256].reshape(64, 4)
        i += 256
        rounds += 1
        start = random.randrange(16)
        runlen = L.sum(1)
        P0 = start + np.concatenate([[0], np.cumsum(runlen)[:-1]])
        P = P0.copy()
        for c in range(4):
            pl = [[L[l, c] // NB + (1 if q < L[l, c] % NB else 0) for q in range(NB)] for l in range(64)]
            for q in range(NB):
                need = [((P[l] & 3) + pl[l][q] + 3) // 4 for l in range(64)]
                n32 = max(2, max(need))
                for j in range(n32):
                    a = [int((P[l] & ~3) + 4 * j) for l in range(64)]
                    add("piece", cyc32(a), 4)
                    add("piece_swz", cyc32([swz(x) for x in a]), 4)
                    add("piece_mask", cyc32([x if j < need[l] else None for l, x in enumerate(a)]), 4)
                n64 = max(2, max(((P[l] & 7) + pl[l][q] + 7) // 8 for l in range(64)))
                for j in range(n64):
                    add("piece_b64", cyc64([int((P[l] & ~7) + 8 * j) for l in range(64)]), 6)
                for l in range(64):
                    P[l] += pl[l][q]
        P = P0.copy()
        for c in range(4):
            need = [((P[l] & 3) + L[l, c] + 3) // 4 for l in range(64)]
            for j in range(max(need)):
                add("cand", cyc32([int((P[l] & ~3) + 4 * j) for l in range(64)]), 4)
            for l in range(64):
                P[l] += L[l, c]
        need = [((P0[l] & 3) + runlen[l] + 3) // 4 for l in range(64)]
        for j in range(max(need)):
            add("run", cyc32([int((P0[l] & ~3) + 4 * j) if j < need[l] else None for l in range(64)]), 4)
    print(f"{wl}: {nw} words, {len(lens)} candidates (mean {lens.mean():.1f} B), NB {NB}, {rounds} rounds of 256")
    print("strategy     instr/round  array cycles/instr  array cycles/round  max(array, transfer)/round")
    for k, (n, a, m) in res.items():
        print(f"{k:12s} {n / rounds:11.1f}  {a / n:18.2f}  {a / rounds:18.1f}  {m / rounds:26.1f}")


if __name__ == "__main__":
    main()
