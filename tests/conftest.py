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


def pytest_report_header(config):
    """Which build of the library this session tests (CYAES_LIBRARY selects a
    variant; the bounds-checked build exports cyaes_debug_bounds)."""
    import cyclone_amd
    path = cyclone_amd.LIB_PATH
    try:
        bounds = hasattr(cyclone_amd.load_library(), "cyaes_debug_bounds")  # (torch's HIP runtime first)
    except (OSError, ImportError) as e:
        return "cyaes library: %s (not loadable: %s)" % (path, e)
    return "cyaes library: %s (%s)" % (os.path.relpath(path, ROOT), "bounds-checked build" if bounds else "product build")


@pytest.fixture(autouse=True)
def _gpu_fault_guard(request):
    """After every `gpu` test: synchronise the device, so an asynchronous fault
    is charged to the test whose work caused it (not to the next test's first
    HIP call), and, on the bounds-checked build (CYAES_LIBRARY=
    build/variants/bounds.so), assert that no kernel access left its extent."""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    import ctypes
    import torch
    if not torch.cuda.is_available():
        return
    torch.cuda.synchronize()
    import cyclone_amd
    lib = cyclone_amd.load_library()
    # Host-memory registrations: nothing the library registered outlives the
    # test that made it, and every unregister took (cyaes_pins.cpp).
    pins = cyclone_amd.debug_pins()
    assert pins["live"] == 0 and pins["refs"] == 0, "library host registrations still live: %s" % pins
    assert pins["failed_unregisters"] == 0 and pins["stale"] == 0, "host unregister failed: %s" % pins
    # Every range registered this session (the library's registry and the
    # tests' own hipHostRegister calls, tests/hiprt.py), released or freed:
    # the runtime answers for none of them any more, and none was unregistered
    # after its memory was unmapped (host queries only).
    import hiprt
    ranges, outlived = cyclone_amd.debug_pin_history()
    assert outlived == 0 and hiprt.OUTLIVED[0] == 0, \
        "a host registration outlived its memory (library %d, tests %d)" % (outlived, hiprt.OUTLIVED[0])
    assert not hiprt.LIVE, "test host registrations still live: %s" % hiprt.LIVE
    stale = [(hex(lo), hi - lo) for lo, hi in ranges + hiprt.HISTORY if hiprt.answers_for(lo, hi)]
    assert not stale, "the runtime still answers for released host ranges: %s" % stale
    fn = getattr(lib, "cyaes_debug_bounds", None)
    if fn is not None:
        rec = (ctypes.c_ulonglong * 20)()
        assert fn(rec) == 0, "cyaes_debug_bounds failed (device error)"
        lines = {int(rec[i]): int(rec[i + 1]) for i in range(4, 20, 2) if rec[i + 1]}
        assert rec[0] == 0, ("bounds check: %d access(es) outside their extent; first at cyaes_kernels.hip:%d, "
                             "offset %d of a %d-byte extent; misses by line: %s"
                             % (rec[0], rec[1], ctypes.c_longlong(rec[2]).value, rec[3], lines))


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
