"""Every measurement record DESIGN.md / README.md cite is committed under profiles/, and the
headline records carry the kernel-source sha they were measured at (CPU only)."""
import json
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CITED = re.compile(r"`((?:profiles/)?(?:r0\d\w*|pmc_\w+)\.(?:json|txt|csv))`")


def _cited():
    names = set()
    for doc in ("DESIGN.md", "README.md"):
        with open(os.path.join(ROOT, doc)) as f:
            names.update(os.path.basename(n) for n in CITED.findall(f.read()))
    return sorted(names)


def test_cited_profiles_exist():
    names = _cited()
    assert names, "no profiles cited"
    missing = [n for n in names if not os.path.exists(os.path.join(ROOT, "profiles", n))]
    assert not missing, missing


def test_cited_pmc_records_name_their_sources():
    for n in _cited():
        if n.startswith("pmc_") and n.endswith(".json"):
            with open(os.path.join(ROOT, "profiles", n)) as f:
                d = json.load(f)
            assert len(d.get("kernel_src_sha", "")) == 64, n
