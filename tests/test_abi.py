"""The C ABI boundary (include/a5x.h) without a GPU: the library loads, exports every
declared symbol, and device entry points fail loudly instead of computing on the host."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import ROOT


def header_functions():
    with open(os.path.join(ROOT, "include", "a5x.h")) as f:
        src = f.read()
    return sorted(set(re.findall(r"A5X_API\s+[\w\s\*]+?\b(a5x_\w+)\s*\(", src)))


def test_header_declares_the_expected_api():
    from hashcat_a5_table_generator_amd import _lib
    assert header_functions() == sorted(_lib.EXPORTS)


def test_library_exports_every_declared_symbol():
    from hashcat_a5_table_generator_amd import _lib
    L = _lib.load()
    for name in header_functions():
        assert hasattr(L, name), name
    assert L.a5x_abi_version() == 1


def test_built_for_gfx950():
    from hashcat_a5_table_generator_amd import _lib
    with open(_lib.LIB_PATH, "rb") as f:
        blob = f.read()
    assert b"gfx950" in blob


def test_device_calls_fail_loudly_without_gpu():
    """No CPU fallback: a device context needs a GPU; host-only contexts refuse kernels."""
    from hashcat_a5_table_generator_amd import _lib
    L = _lib.load()
    h = ctypes.c_void_p()
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:
        has_gpu = False
    if not has_gpu:
        assert L.a5x_create(0, ctypes.byref(h)) != 0
    h = ctypes.c_void_p()
    assert L.a5x_create(-1, ctypes.byref(h)) == 0
    L.a5x_parse_table(h, b"a=b\n", 4)
    words = np.frombuffer(b"abc" + b"\0" * 16, dtype=np.uint8)
    offs = np.array([0, 3], dtype=np.uint64)
    cnt = np.zeros(1, dtype=np.uint64)
    rc = L.a5x_keyspace(h, words.ctypes.data, offs.ctypes.data, 1, 0, 0, 15, cnt.ctypes.data, cnt.ctypes.data)
    assert rc == -2  # A5X_E_HIP
    assert b"host-only" in L.a5x_last_error(h)
    L.a5x_destroy(h)


def test_context_without_gpu_raises():
    from hashcat_a5_table_generator_amd import A5xError, Context
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("a GPU is present")
    except Exception:
        pass
    with pytest.raises(A5xError):
        Context(0)


def test_partition_abi():
    from hashcat_a5_table_generator_amd import partition
    s = partition(np.array([0, 10, 20, 30, 40], dtype=np.uint64), 2)
    assert list(s) == [0, 2, 4]
    s = partition(np.array([0, 0, 0], dtype=np.uint64), 3)
    assert s[0] == 0 and s[-1] == 2


def test_cli_replica_usage():
    import subprocess
    from hashcat_a5_table_generator_amd import build
    if not os.path.exists(build.CLI):
        pytest.skip("CLI not built")
    r = subprocess.run([build.CLI, "--help"], capture_output=True, text=True)
    assert r.returncode == 0 and "--table-files" in r.stdout
    r = subprocess.run([build.CLI], capture_output=True, text=True)
    assert r.returncode != 0 and "table-files" in r.stderr


def test_create_failure_names_the_hip_call():
    """a5x_create with no visible device: the exception carries the failing HIP call and
    hipGetErrorString (a5x_create_error), not a bare A5X_E_HIP.  A child process, so that
    HIP_VISIBLE_DEVICES=-1 is seen before the HIP runtime initialises."""
    import subprocess
    import sys
    code = ("from hashcat_a5_table_generator_amd import Context, A5xError\n"
            "try:\n    Context(0)\nexcept A5xError as e:\n    print('ERR', e)\nelse:\n    print('OK')\n")
    env = dict(os.environ, HIP_VISIBLE_DEVICES="-1", ROCR_VISIBLE_DEVICES="-1")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    out = r.stdout.strip()
    assert out.startswith("ERR"), (out, r.stderr[-2000:])
    assert "A5X_E_HIP" in out and "a5x_create(device=0)" in out, out
    assert "hipGetDeviceCount" in out, out


def test_create_error_is_empty_after_success():
    from hashcat_a5_table_generator_amd import _lib
    L = _lib.load()
    h = ctypes.c_void_p()
    assert L.a5x_create(-7, ctypes.byref(h)) != 0
    assert L.a5x_create_error()  # the argument problem is named
    assert L.a5x_create(-1, ctypes.byref(h)) == 0
    assert L.a5x_create_error() == b""
    L.a5x_destroy(h)
