"""Test configuration: `gpu` marker, repo on sys.path, built artefacts present."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device")
    need = [os.path.join(ROOT, "oracle", "liboracle.so"), os.path.join(ROOT, "cyclone_amd", "libcyaes.so")]
    if not all(os.path.exists(p) for p in need):
        subprocess.run(["make", "-C", ROOT, "-j8", "lib", "oracle"], check=True)


@pytest.fixture(scope="session")
def golden():
    import json
    with open(os.path.join(GOLDEN, "openssl_vectors.json")) as f:
        ov = json.load(f)
    with open(os.path.join(GOLDEN, "ref_kat.json")) as f:
        kat = json.load(f)
    with open(os.path.join(GOLDEN, "ref_tables.json")) as f:
        tables = json.load(f)
    return {"openssl": ov, "kat": kat, "tables": tables}
