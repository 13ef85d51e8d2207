"""pytest --junitxml of a GPU run -> profiles/<name>_<kernel_src_sha12>.txt (per-test outcomes).

    python tools/junit_record.py gpurun_out/junit_<tag>.xml <name>
"""
import os
import sys
import xml.etree.ElementTree as ET

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import kernel_src_sha  # noqa: E402

src, name = sys.argv[1], sys.argv[2]
root = ET.parse(src).getroot()
suite = root if root.tag == "testsuite" else root.find("testsuite")
sha = kernel_src_sha()[:12]
lines = [f"# pytest -m gpu on MI355X, kernel_src_sha {sha} (bench.kernel_src_sha of csrc/ at this run)",
         f"# junit: tests={suite.get('tests')} failures={suite.get('failures')} errors={suite.get('errors')} "
         f"skipped={suite.get('skipped')} time={suite.get('time')} s"]
for tc in suite.iter("testcase"):
    st = "passed"
    for k in ("failure", "error", "skipped"):
        if tc.find(k) is not None:
            st = {"failure": "FAILED", "error": "ERROR", "skipped": "skipped"}[k]
    lines.append(f"{st:8s} {tc.get('classname')}::{tc.get('name')}  ({float(tc.get('time', 0)):.2f} s)")
out = os.path.join(ROOT, "profiles", f"{name}_{sha}.txt")
with open(out, "w") as f:
    f.write("\n".join(lines) + "\n")
print(out, len(lines) - 2, "tests")
