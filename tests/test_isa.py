"""CPU guard on the built kernels' instruction schedules (tools/isa_stats.py).

The AES kernels are LDS-bound: a step's 640 (decrypt) or 1,280-1,440
(encrypt) table lookups must go out in bursts, with few s_waitcnt between
them.  Twice a change elsewhere in a kernel body lost that schedule without
any test noticing (r05: the strided decrypt; r06: a runtime
branch in the flat decrypt's range loop, 232 -> 493 waits, the relay stream's
decrypt +7.8 %).  This reads the device code of the built
objects (no GPU) and checks, per throughput kernel, waits per LDS read and
scratch spills.  The latency-bound quad encrypt (a wait per round by design),
the A/B-only XCD-weighted decrypt and the keyed ragged decrypt (the batcher's
OPEN path, PCIe-bound) are listed apart.
"""
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

# (substring of the mangled name, max waits per LDS read, max scratch instructions)
GUARDS = [
    ("k_duplex", 0.20, 8),
    ("k_encrypt_lines", 0.22, 0),
    ("k_encrypt_rag_lines", 0.22, 24),
    ("9k_encryptILb", 0.22, 0),
    ("k_decrypt_raggedILb0", 0.20, 0),
    ("k_decrypt_flat_keyed", 0.22, 0),
]
EXEMPT = ("k_encrypt_quad", "k_decrypt_raggedILb1", "ELb1EEEvNS_7DecArgsE")  # see the docstring


def _stats():
    if not (shutil.which("hipcc") or os.path.exists("/opt/rocm/lib/llvm/bin/llvm-objdump")):
        pytest.skip("no ROCm LLVM tools")
    if not os.path.exists(os.path.join(ROOT, "build", "cyaes_dec_kernels.o")):
        pytest.skip("kernel objects not built (make)")
    import isa_stats
    return isa_stats.stats()


def test_lds_bound_kernels_keep_their_schedule():
    st = _stats()
    seen = set()
    bad = []
    for (tu, name), s in st.items():
        if s["lds"] < 600:
            continue  # not an AES step body
        flat = "decrypt_flat" in name and "keyed" not in name
        xw = flat and name.endswith("ELb1EEEvNS_7DecArgsE")
        if any(e in name for e in EXEMPT[:2]) or xw:
            continue
        lim = None
        for sub, w, scr in GUARDS:
            if sub in name:
                lim = (w, scr)
                seen.add(sub)
        if flat:
            lim = (0.22, 8)
            seen.add("flat")
        if lim is None:
            bad.append("%s %s: no guard" % (tu, name))
            continue
        ratio = s["waitcnt"] / s["lds"]
        if ratio > lim[0] or s["scratch"] > lim[1]:
            bad.append("%s %s: %.2f waits per LDS read (max %.2f), %d scratch (max %d)" % (
                tu, name, ratio, lim[0], s["scratch"], lim[1]))
    assert not bad, "\n".join(bad)
    assert seen >= {g[0] for g in GUARDS} | {"flat"}, seen


def test_flat_decrypt_instantiations_share_one_schedule():
    """Every unkeyed flat decrypt (uniform, strided, sessions, IV arrays, both
    progress divisors) within a few waits of the others: a body change that
    breaks one instantiation's schedule stands out here first."""
    st = _stats()
    waits = {name: s["waitcnt"] for (tu, name), s in st.items()
             if tu == "cyaes_dec_kernels" and "decrypt_flat" in name and not name.endswith("ELb1EEEvNS_7DecArgsE")}
    assert len(waits) >= 10, waits
    assert max(waits.values()) <= 1.15 * min(waits.values()), waits
