"""Build liba5x.so (HIP kernels for gfx950 + C++ host) and the CLI replica in-tree.

``python -m hashcat_a5_table_generator_amd.build`` or ``__graft_entry__.build()``.
Outputs go to ``hashcat_a5_table_generator_amd/_build/`` (git-ignored, but they
travel to the GPU box with the gpurun snapshot).
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
OUT = os.path.join(PKG, "_build")
LIB = os.path.join(OUT, "liba5x.so")
CLI = os.path.join(OUT, "a5x_generator")
ARCH = os.environ.get("A5X_OFFLOAD_ARCH", "gfx950")

LIB_SRCS = ["a5x_kernels.hip", "a5x_modes.hip", "a5x_digest.hip", "a5x_host.cpp"]
HEADERS = ["a5x_format.h", "a5x_gosem.h", "a5x_launch.h", "a5x_plan.h", "a5x_fx6.h", "a5x_ring.h", "a5x_md.h"]


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm is required to build liba5x)")


def _stale(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build_diag(verbose: bool = False) -> str:
    """Diagnostic variant in _build_diag/: per-phase s_memtime stamps of the fast kernel
    (-DA5X_STAMPS; tools/stamps.py).  Timing ablations are compile-time variants
    (build_variant(name, ["FX_ABL=<mask>"]), a5x_kernels.hip FX_ABL).  Never loaded by
    the product or the tests."""
    return build_variant("diag", ["A5X_STAMPS"], verbose)


def build_variant(name: str, defines, verbose: bool = False) -> str:
    """A5X tuning experiments: liba5x with extra -D defines in _build_<name>/ (never the product)."""
    out = os.path.join(PKG, "_build_" + name)
    os.makedirs(out, exist_ok=True)
    lib = os.path.join(out, "liba5x.so")
    srcs = [os.path.join(CSRC, s) for s in LIB_SRCS]
    cmd = [_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-fvisibility=hidden",
           *["-D" + d for d in defines], "-I", os.path.join(ROOT, "include"), "-I", CSRC, *srcs, "-o", lib]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    return lib


def build(force: bool = False, verbose: bool = False) -> str:
    os.makedirs(OUT, exist_ok=True)
    hipcc = _hipcc()
    srcs = [os.path.join(CSRC, s) for s in LIB_SRCS]
    deps = srcs + [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(ROOT, "include", "a5x.h")]
    inc = ["-I", os.path.join(ROOT, "include"), "-I", CSRC]
    if force or _stale(LIB, deps):
        cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
               "-fvisibility=hidden", *inc, *srcs, "-o", LIB + ".tmp"]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        os.replace(LIB + ".tmp", LIB)
    cli_src = os.path.join(CSRC, "a5x_cli.cpp")
    if os.path.exists(cli_src) and (force or _stale(CLI, [cli_src, LIB, os.path.join(CSRC, "a5x_gosem.h")])):
        cmd = [hipcc, "-O2", "-std=c++17", "-pthread", *inc, cli_src, "-o", CLI, "-L", OUT, "-la5x",
               "-Wl,-rpath,$ORIGIN"]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
