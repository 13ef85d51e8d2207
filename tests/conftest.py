import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

TABLES = os.path.join(ROOT, "tests", "golden", "tables")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    config.addinivalue_line("markers", "slow: long-running")


def table_path(name: str) -> str:
    return os.path.join(TABLES, name + ".table")


@pytest.fixture(scope="session")
def gpu_ctx():
    from hashcat_a5_table_generator_amd import Context
    c = Context(0)
    yield c
    c.close()
