"""C-ABI boundary checks that need no GPU: the library loads, exports every
symbol include/cyaes.h declares, its host key schedule equals the oracle's
(Rijndael::Rijndael, cyr_rijndael.cpp:507-572), and argument errors are
reported the way DESIGN.md §2 documents instead of the reference's asserts."""
import ctypes
import os
import random
import subprocess

import pytest

import cyclone_amd as ca
import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_header_symbol():
    lib = ca.load_library()
    names = ca.header_functions()
    assert len(names) >= 40
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    # and the binding declares a signature for each of them
    assert sorted(ca._SIGS) == names


def test_mgpu_library_exports_its_header():
    lib = ca.load_mgpu_library()
    names = ca.header_functions([ca.MGPU_HEADER])
    assert names and all(hasattr(lib, n) for n in names)
    assert sorted(ca._MGPU_SIGS) == names
    assert ca.mgpu_shard(10, 3, 0) == (0, 3) and ca.mgpu_shard(10, 3, 2) == (6, 4)
    assert ca.mgpu_shard(1024, 4, 1, align=256) == (256, 256)
    covered = [ca.mgpu_shard(1000, 7, i, 16) for i in range(7)]
    assert covered[0][0] == 0 and sum(c for _, c in covered) == 1000
    assert all(a + c == b for (a, c), (b, _) in zip(covered, covered[1:]))


def test_every_include_header_is_checked():
    """Each include/*.h with a C-ABI is covered by one of the export checks above."""
    hdrs = sorted(f for f in os.listdir(os.path.join(ROOT, "include")) if f.endswith(".h"))
    assert hdrs == ["cyaes.h", "cyaes_adler32.h", "cyaes_batch.h", "cyaes_mgpu.h", "cyaes_relay.h"]


def test_key_expand_matches_oracle(golden):
    rng = random.Random(7)
    keys = [bytes.fromhex(golden["kat"]["key"])] + [bytes(rng.randrange(256) for _ in range(16)) for _ in range(64)]
    for k in keys:
        assert ca.key_expand(k).words() == oracle.key_expand(k).words()
    for s in golden["openssl"]["schedules"]:
        ke, kd = ca.key_expand(bytes.fromhex(s["key"])).words()
        assert ke == s["ke"] and kd == s["kd"]


def test_default_iv_and_strings():
    lib = ca.load_library()
    assert ctypes.string_at(lib.cyaes_default_iv(), 16) == bytes(range(16))
    assert ca.Rijndael.DefaultIV == bytes(range(16)) and ca.Rijndael.BLOCK_SIZE == 16
    assert ca.strerror(ca.CYAES_EINVAL) == "invalid argument"
    assert "gfx950" in ca.version()
    assert ctypes.sizeof(ca.CyaesKey) == 352  # == sizeof(m_Ke) + sizeof(m_Kd)


def test_argument_errors_without_device():
    """size % 16, NULL buffers -> CYAES_EINVAL; size 0 -> no-op (cyr_rijndael.cpp:590-591)."""
    lib = ca.load_library()
    k = ca.key_expand(bytes(16))
    buf = (ctypes.c_uint8 * 32)()
    iv = (ctypes.c_uint8 * 16)(*([7] * 16))
    for fn in (lib.cyaes_cbc_encrypt, lib.cyaes_cbc_decrypt):
        assert fn(ctypes.byref(k), buf, buf, 17, None) == ca.CYAES_EINVAL
        assert fn(ctypes.byref(k), None, buf, 16, None) == ca.CYAES_EINVAL
        assert fn(None, buf, buf, 16, None) == ca.CYAES_EINVAL
        assert fn(ctypes.byref(k), buf, buf, 0, iv) == ca.CYAES_OK
        assert list(iv) == [7] * 16
    assert lib.cyaes_key_expand(None, ctypes.byref(k)) == ca.CYAES_EINVAL
    assert lib.cyaes_gpu_encrypt_uniform(None, None, None, 1, 16, None, 0, None, None, None) == ca.CYAES_EINVAL
    assert lib.cyaes_gpu_fill_synthetic(None, 0, 1, 16, 0, None) == ca.CYAES_EINVAL
    for fn in (lib.cyaes_gpu_encrypt_host, lib.cyaes_gpu_decrypt_host):
        assert fn(None, buf, buf, 1, 16, 0, 0) == ca.CYAES_EINVAL
    assert lib.cyaes_batcher_submit_many(None, None, 0, None) == ca.CYAES_EINVAL


def _has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.mark.skipif(_has_gpu(), reason="checks the no-device path")
def test_create_without_device_fails_loudly():
    with pytest.raises(ca.CyaesError) as e:
        ca.GpuContext(0)
    assert e.value.status == ca.CYAES_ENODEV


def test_missing_library_fails_loudly(tmp_path):
    with pytest.raises(ImportError):
        ca.load_library(str(tmp_path / "libcyaes.so"))


def test_cpp_dropin_builds_and_links():
    """The cyclone::Rijndael drop-in header + C-ABI compile and link (relay-style client)."""
    subprocess.run(["make", "-C", ROOT, "-s", "cpptest"], check=True)
    exe = os.path.join(ROOT, "build", "test_rijndael")
    assert os.access(exe, os.X_OK)
    out = subprocess.run(["nm", "-D", "--undefined-only", exe], capture_output=True, text=True).stdout
    assert "_ZN7cyclone8Rijndael7encryptEPKhPhmS3_" in out  # Rijndael::encrypt from libcyaes.so
    exported = subprocess.run(["nm", "-D", "--defined-only", ca.LIB_PATH], capture_output=True, text=True).stdout
    for sym in ("_ZN7cyclone8RijndaelC1EPKh", "_ZN7cyclone8Rijndael7encryptEPKhPhmS3_",
                "_ZN7cyclone8Rijndael7decryptEPKhPhmS3_", "_ZN7cyclone8Rijndael9DefaultIVE"):
        assert sym in exported, sym


@pytest.mark.skipif(_has_gpu(), reason="checks the no-device path")
def test_mgpu_without_device_fails_loudly():
    with pytest.raises(ca.CyaesError) as e:
        ca.MultiGpu([0])
    assert e.value.status == ca.CYAES_ENODEV


def test_relay_call_expressions_compile():
    """samples/relay's Rijndael expressions, verbatim (tests/cpp/relay_calls.cpp:
    relay_local.cpp:204-207,329-334,343,363-366), compile and link against the
    drop-in header unchanged -- INTEGRATION.md §1's claim, as a build."""
    subprocess.run(["make", "-C", ROOT, "-s", "cpptest"], check=True)
    exe = os.path.join(ROOT, "build", "relay_calls")
    src = open(os.path.join(ROOT, "tests", "cpp", "relay_calls.cpp")).read()
    for expr in ("pipe->m_encrypt = new Rijndael(pipe->m_secretKey.bytes);",
                 "for (size_t i = 0; i < Rijndael::BLOCK_SIZE; i++)",
                 "pipe->m_encrypt->encrypt(buf, buf, buf_round_size);",
                 "pipe->m_decrypt->decrypt(buf, buf, packet.get_packet_size() - sizeof(RelayForwardMsg));",
                 "memset(pipe->m_secretKey.bytes, 0, Rijndael::BLOCK_SIZE);"):
        assert expr in src, expr
    assert subprocess.run([exe, "--compile"]).returncode == 0


def test_dropin_fails_closed():
    """A drop-in call that cannot run on the GPU aborts (NDEBUG build included)
    instead of returning with the relay's buffer still plaintext.  Here: a
    device index that does not exist (and, in this container, no GPU at all)."""
    subprocess.run(["make", "-C", ROOT, "-s", "cpptest"], check=True)
    p = subprocess.run([os.path.join(ROOT, "build", "relay_calls")], capture_output=True, text=True,
                       env=dict(os.environ, CYAES_DEVICE="99"), timeout=120)
    assert p.returncode == -6, (p.returncode, p.stdout, p.stderr)  # SIGABRT
    assert "aborting rather than leave the buffer unprocessed" in p.stderr
    assert "relay_calls: ok" not in p.stdout
