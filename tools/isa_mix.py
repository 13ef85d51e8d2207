"""Issue-cost mix of the fused digests' VALU stream (CPU: hipcc -S for gfx950, no GPU).

The SIMD issue cost of an integer VALU wave64 instruction on MI355X is 2 or 4 cycles by
opcode (tools/mb_valu.hip, profiles/r06_mb_valu.txt, 4 waves per SIMD): v_add_u32 / v_xor_b32 /
v_bitop3_b32 / v_add_u32_e64 / v_cmp / v_cndmask issue in ~2 cycles (the chip's nominal
32 lanes per cycle), v_add3_u32 / v_alignbit_b32 / v_bfi_b32 / v_perm_b32 / v_alignbyte_b32 /
v_lshl_or_b32 / v_lshl_add_u32 / v_lshlrev_b32_e64 / v_mul_hi_u32 in ~4 (half rate).
This tool compiles md5_block / md4_block (csrc/a5x_md.h) on runtime data and the whole
k_expand_fast_md5 / _ntlm kernels, counts every VALU opcode and prices it, giving the mean
SIMD cycles per VALU instruction of each stream -> the mix-weighted VALU peak
(256 CUs x 4 SIMDs x 64 lanes x clock / mean cycles) that bench.py reports beside the nominal
2-cycle peak.  Opcodes the microbenchmark did not measure are priced by class (marked '~').

    python tools/isa_mix.py [out.json]
"""
import collections
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "hashcat_a5_table_generator_amd", "csrc")

MEASURED = {  # profiles/r06_mb_valu.txt, 4 waves per SIMD, rounded to the issue class
    "v_add_u32_e32": 2, "v_xor_b32_e32": 2, "v_bitop3_b32": 2, "v_add_u32_e64": 2, "v_cndmask_b32_e32": 2,
    "v_cmp_gt_u32_e32": 2, "v_add3_u32": 4, "v_xad_u32": 4, "v_bfi_b32": 4, "v_alignbit_b32": 4, "v_perm_b32": 4,
    "v_alignbyte_b32": 4, "v_lshl_or_b32": 4, "v_lshl_add_u32": 4, "v_mul_hi_u32": 4, "v_lshlrev_b32_e64": 4,
}
HALF = re.compile(r"^v_(add3|xad|bfi|align|perm|lshl_|lshr|ashr|mul|mad|bfe|lshl|lshlrev|lshrrev|ashrrev|alignbit|"
                  r"alignbyte|readlane|writelane|sad|cvt|bcnt|ffbh|ffbl|mbcnt)")


def price(op):
    if op in MEASURED:
        return MEASURED[op], False
    base = op[:-4] if op.endswith("_e32") or op.endswith("_e64") else op
    if base.startswith(("v_lshlrev", "v_lshrrev", "v_ashrrev")) and op.endswith("_e32"):
        return 4, True  # shifts: the e64 form measured half rate; assume the same unit
    return (4 if HALF.match(base) else 2), True


PROBE = r'''
#include <hip/hip_runtime.h>
#include "a5x_md.h"
__global__ void p_md5(const uint32_t* in, uint32_t* out) {
  uint32_t M[16], st[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
  for (int i = 0; i < 16; i++) M[i] = in[threadIdx.x * 16 + i];
  md5_block(st, M);
  for (int i = 0; i < 4; i++) out[threadIdx.x * 4 + i] = st[i];
}
__global__ void p_md4(const uint32_t* in, uint32_t* out) {
  uint32_t M[16], st[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
  for (int i = 0; i < 16; i++) M[i] = in[threadIdx.x * 16 + i];
  md4_block(st, M);
  for (int i = 0; i < 4; i++) out[threadIdx.x * 4 + i] = st[i];
}
'''


def asm(src_path, extra=()):
    out = tempfile.mktemp(suffix=".s")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only", "-S",
                    "-I", CSRC, "-I", os.path.join(ROOT, "include"), *extra, src_path, "-o", out],
                   check=True, stderr=subprocess.DEVNULL)
    text = open(out).read()
    os.remove(out)
    return text


def func_ops(text, sym):
    m = re.search(r"^" + re.escape(sym) + r":[^\n]*\n(.*?)^\.Lfunc_end", text, re.S | re.M)
    if not m:
        raise SystemExit("symbol not found: " + sym)
    return collections.Counter(re.findall(r"^\s+(v_[a-z0-9_]+)", m.group(1), re.M))


def mix(ops):
    n = sum(ops.values())
    cyc = sum(c * price(o)[0] for o, c in ops.items())
    est = sorted({o for o in ops if price(o)[1]})
    top = [(o, c, price(o)[0]) for o, c in ops.most_common(12)]
    return {"valu_instructions": n, "mean_issue_cycles": cyc / n, "half_rate_share": sum(c for o, c in ops.items()
            if price(o)[0] == 4) / n, "top": top, "priced_by_class": est}


def main():
    d = tempfile.mkdtemp()
    p = os.path.join(d, "probe.hip")
    open(p, "w").write(PROBE)
    t = asm(p)
    res = {"md5_block": mix(func_ops(t, "_Z5p_md5PKjPj")), "md4_block": mix(func_ops(t, "_Z5p_md4PKjPj"))}
    k = asm(os.path.join(CSRC, "a5x_kernels.hip"))
    res["k_expand_fast_md5 (static, whole kernel)"] = mix(func_ops(k, "_Z17k_expand_fast_md57ExpArgs"))
    res["k_expand_fast_ntlm (static, whole kernel)"] = mix(func_ops(k, "_Z18k_expand_fast_ntlm7ExpArgs"))
    res["costs"] = "tools/mb_valu.hip / profiles/r06_mb_valu.txt (2 = full rate, 4 = half rate per wave64 instruction)"
    for name, r in res.items():
        if isinstance(r, dict):
            print(f"{name:44s} {r['valu_instructions']:6d} VALU  mean {r['mean_issue_cycles']:.2f} cycles  "
                  f"half-rate share {r['half_rate_share']:.2f}  top {[(o, c) for o, c, _ in r['top'][:6]]}")
    if len(sys.argv) > 1:
        json.dump(res, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
