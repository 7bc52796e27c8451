"""GPU parity: the gfx950 HIP path (through the C-ABI) vs the oracle and the
committed goldens, bit-exact.  Mirrors the reference's Rijndael TEST_CASE
(thejinchao/cyclone test/unit/cyt_unit_crypt.cpp:173-248) and extends it to
the batched relay semantics (one chain per payload, relay_local.cpp:206,
relay_server.cpp:329) at every BASELINE.json config size."""
import os
import random
import subprocess

import numpy as np
import pytest

import cyclone_amd as ca
import hiprt
import oracle

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
K0 = oracle.KEY_00_0F


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "gpu tests need a ROCm device"
    return t


# Encrypt has two kernels: four lanes per chain for batches
# under CYAES_QUAD_MAX_CHAINS chains (every small test batch here), one lane
# per chain above.  "lane" forces the latter, so both run every test's paths
# (keys, IVs, ragged, in place); "run3" also makes each lane's work item a run
# of 3 consecutive payloads (k_encrypt RUNS, CYAES_ENC_RUN; the runtime keeps
# single payloads where runs do not apply: IV arrays, key index arrays,
# sessions that are not whole runs).  The full-size configs below use the
# runtime's own choice.
# Decrypt: waves take work ranges (flat kernel) and payload
# groups (ragged kernel) from a per-launch ticket counter once a wave has more
# than one; "dyn1" caps the decrypt grid at 3 workgroups with 1-step ranges,
# so even the small test batches hand out many ranges per wave, and "static1"
# runs the static per-wave split on a 2-workgroup grid.
KERNEL_MODES = {"auto": {}, "lane": {"CYAES_QUAD_MAX_CHAINS": "0"},
                "run3": {"CYAES_QUAD_MAX_CHAINS": "0", "CYAES_ENC_RUN": "3"},
                "dyn1": {"CYAES_DEC_GRID": "3", "CYAES_DEC_RANGE_STEPS": "1", "CYAES_DEC_GROUPS_PER_WAVE": "64",
                         "CYAES_DEC_DYN": "1"},
                "static1": {"CYAES_QUAD_MAX_CHAINS": "0", "CYAES_DEC_GRID": "2", "CYAES_DEC_DYN": "0"}}
_MODE_VARS = ("CYAES_QUAD_MAX_CHAINS", "CYAES_ENC_RUN", "CYAES_DEC_GRID", "CYAES_DEC_RANGE_STEPS",
              "CYAES_DEC_GROUPS_PER_WAVE", "CYAES_DEC_DYN")


def _set_mode(mode):
    old = {k: os.environ.get(k) for k in _MODE_VARS}
    for k in _MODE_VARS:
        os.environ.pop(k, None)
    os.environ.update(KERNEL_MODES[mode])
    return old


def _restore(old):
    for k, v in old.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v


@pytest.fixture(params=sorted(KERNEL_MODES))
def encrypt_kernel(request):
    """Contexts created inside the test use this encrypt-kernel mode."""
    old = _set_mode(request.param)
    yield request.param
    _restore(old)


@pytest.fixture(scope="module", params=sorted(KERNEL_MODES))
def ctx(torch, request):
    old = _set_mode(request.param)
    c = ca.GpuContext(0)
    _restore(old)
    c.set_keys(K0)
    yield c
    c.close()


def dev(torch, arr):
    a = np.ascontiguousarray(arr)
    return torch.from_numpy(a.view(np.uint8).reshape(-1).copy()).to("cuda")


def host(t):
    import torch as _t
    _t.cuda.synchronize()
    return t.cpu().numpy()


def empty(torch, n):
    return torch.empty(max(int(n), 1), dtype=torch.uint8, device="cuda")


# ---------------------------------------------------------------- drop-in --
def test_reference_testcase_cpp(torch):
    """The C++ re-expression of cyt_unit_crypt.cpp:173-248 against the drop-in class."""
    subprocess.run(["make", "-C", ROOT, "-s", "cpptest"], check=True)
    r = subprocess.run([os.path.join(ROOT, "build", "test_rijndael"), os.path.join(ROOT, "tests/golden/ref_kat.txt")],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "All tests passed" in r.stdout


def test_relay_call_expressions_run(torch):
    """relay_local.cpp's Rijndael expressions, verbatim, run on the GPU (in-place
    encrypt of a 0xCE-padded chunk, in-place decrypt of packet_size - 8 bytes)."""
    subprocess.run(["make", "-C", ROOT, "-s", "cpptest"], check=True)
    r = subprocess.run([os.path.join(ROOT, "build", "relay_calls")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "relay_calls: ok" in r.stdout


def test_dropin_python_kat_stream_inplace(golden):
    k = golden["kat"]
    aes = ca.Rijndael(bytes.fromhex(k["key"]))
    plain, cipher = bytes.fromhex(k["plaintext"]), bytes.fromhex(k["ciphertext"])
    assert bytes(aes.encrypt(plain)) == cipher
    assert bytes(aes.decrypt(cipher)) == plain
    for fn, src, want in ((aes.encrypt, plain, cipher), (aes.decrypt, cipher, plain)):
        iv = bytearray(aes.DefaultIV)
        out = bytearray()
        for i in range(0, 64, 16):
            out += fn(src[i:i + 16], None, 16, iv)
        assert bytes(out) == want and bytes(iv) == bytes.fromhex(k["iv_check"])
    buf = bytearray(plain)
    aes.encrypt(buf, buf)
    assert bytes(buf) == cipher
    aes.decrypt(buf, buf)
    assert bytes(buf) == plain


def test_dropin_random_roundtrips():
    rng = random.Random(3)
    for _ in range(20):
        key = bytes(rng.randrange(256) for _ in range(16))
        data = bytes(rng.randrange(256) for _ in range(128))
        aes, ref = ca.Rijndael(key), oracle.Rijndael(key)
        ct = bytes(aes.encrypt(data))
        assert ct == bytes(ref.encrypt(data))
        assert bytes(aes.decrypt(ct)) == data


def test_dropin_concurrent_threads():
    """Synchronous calls from many threads at once are combined into shared GPU
    batches (mixed directions, sizes, keys, IV in/out, in place): every call
    still gets exactly its own Rijndael::encrypt/decrypt result."""
    import threading

    errors = []

    def worker(t):
        rng = random.Random(100 + t)
        try:
            for _ in range(40):
                key = bytes(rng.randrange(256) for _ in range(16))
                size = 16 * rng.choice([1, 2, 5, 64, 92, 93, 300])
                data = bytes(rng.randrange(256) for _ in range(size))
                aes, ref = ca.Rijndael(key), oracle.Rijndael(key)
                use_iv = rng.random() < 0.5
                iv0 = bytes(rng.randrange(256) for _ in range(16))
                iv, riv = (bytearray(iv0), bytearray(iv0)) if use_iv else (None, None)
                if rng.random() < 0.5:
                    got = bytes(aes.encrypt(data, None, size, iv))
                    want = bytes(ref.encrypt(data, None, size, riv))
                else:
                    buf = bytearray(data)  # in place
                    aes.decrypt(buf, buf, size, iv)
                    got = bytes(buf)
                    want = bytes(ref.decrypt(data, None, size, riv))
                if got != want or iv != riv:
                    errors.append((t, size, use_iv))
        except Exception as e:  # noqa: BLE001 -- reported below
            errors.append((t, repr(e)))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(12)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors[:5]


def test_dropin_config_sizes(golden):
    """Single relay-sized calls (up to the 65280 B relay cap and 64 KiB)."""
    aes = ca.Rijndael(K0)
    for v in golden["openssl"]["sizes"]:
        if v["p"]:
            continue
        pt = oracle.synthetic(0, 1, v["payload_bytes"]).tobytes()
        ct = bytes(aes.encrypt(pt))
        assert ct[-16:].hex() == v["last_block"]
        assert ct == bytes(oracle.Rijndael(K0).encrypt(pt))
        assert bytes(aes.decrypt(ct)) == pt


# ------------------------------------------------------------- batch API --
@pytest.mark.parametrize("pb,n", [(16, 5000), (48, 3001), (64, 1000), (144, 777), (240, 513), (368, 300),
                                  (1024, 4096), (1472, 2047), (4096, 257), (65280, 65), (65536, 96)])
def test_uniform_batch_vs_oracle(torch, ctx, pb, n):
    pt = oracle.synthetic(11, n, pb)
    want = oracle.batch(False, [K0], 0, pt, pb, nthreads=16)
    d_pt, d_ct, d_rt = dev(torch, pt), empty(torch, pt.size), empty(torch, pt.size)
    ctx.encrypt_uniform(d_pt, d_ct, n, pb)
    got = host(d_ct)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, "encrypt mismatch at byte %d (payload %d)" % (bad[0], bad[0] // pb)
    ctx.decrypt_uniform(d_ct, d_rt, n, pb)
    assert np.array_equal(host(d_rt), pt)
    assert ctx.check() == ca.CYAES_OK


def test_in_place_batches(torch, ctx):
    """in == out: encrypt (lane-private) and decrypt (boundary snapshot across waves)."""
    pb, n = 1472, 30000
    pt = oracle.synthetic(5, n, pb)
    want = oracle.batch(False, [K0], 0, pt, pb, nthreads=16)
    d = dev(torch, pt)
    ctx.encrypt_uniform(d, d, n, pb)
    assert np.array_equal(host(d), want)
    ctx.decrypt_uniform(d, d, n, pb)
    assert np.array_equal(host(d), pt)


def test_in_place_decrypts_on_two_streams(torch, ctx):
    """Two in-place decrypts (boundary snapshots) and two aliased-IV decrypts of
    one context on two streams at once: each call's scratch is its own."""
    pb, n = 1472, 40000
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    pts = [oracle.synthetic(7 + 100000 * i, n, pb) for i in range(2)]
    cts = [oracle.batch(False, [K0], 0, pt, pb, nthreads=16) for pt in pts]
    ds = [dev(torch, ct) for ct in cts]
    ivs = [dev(torch, np.tile(np.frombuffer(bytes(range(16)), np.uint8), n)) for _ in range(2)]
    torch.cuda.synchronize()
    for rep in range(3):
        for i, s in enumerate((s1, s2)):
            ctx.decrypt_uniform(ds[i], ds[i], n, pb, stream=s.cuda_stream)
        for i, s in enumerate((s1, s2)):
            ctx.encrypt_uniform(ds[i], ds[i], n, pb, stream=s.cuda_stream)
        torch.cuda.synchronize()
    for i, s in enumerate((s1, s2)):  # aliased IV in/out: a per-call copy of the IVs
        ctx.decrypt_uniform(ds[i], ds[i], n, pb, iv_in=ivs[i], iv_out=ivs[i], stream=s.cuda_stream)
    torch.cuda.synchronize()
    for i in range(2):
        assert np.array_equal(host(ds[i]), pts[i])
        assert np.array_equal(host(ivs[i]).reshape(n, 16), cts[i].reshape(n, pb // 16, 16)[:, -1])
    assert ctx.check() == ca.CYAES_OK


@pytest.mark.parametrize("pb,n", [(1472, 65536), (65536, 2048), (1488, 40000)])
@pytest.mark.parametrize("inplace", [False, True])
def test_dynamic_ranges_full_grid(torch, pb, n, inplace):
    """Flat decrypt with the default grid on batches big enough that each wave
    takes several work ranges from the launch's ticket counter (DESIGN.md §3.3,
    VERDICT r03 next 2): MTU payloads (!BIG rows), 64 KiB payloads (one payload
    start per step at most), and a payload size that does not divide a step.
    In place, every range's C[begin-1] comes from the prepass snapshot.  The
    same batch under the static per-wave split gives the same bytes.  An
    all-dynamic split of one-step ranges makes waves prefetch the first step
    of their next range often, next to the batch's partial last range."""
    pt = oracle.synthetic(11, n, pb)
    ct = oracle.batch(False, [K0], 0, pt, pb, nthreads=16)
    outs = []
    for env in ({}, {"CYAES_DEC_DYN": "0"}, {"CYAES_DEC_DYN": "1", "CYAES_DEC_RANGE_STEPS": "1"},
                {"CYAES_DEC_DYN": "1", "CYAES_DEC_RANGE_STEPS": "5", "CYAES_DEC_DYN_PCT": "60"},
                {"CYAES_DEC_DYN": "1", "CYAES_DEC_RANGE_STEPS": "1", "CYAES_DEC_DYN_PCT": "100"}):
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        c = ca.GpuContext(0)
        _restore(old)
        c.set_keys(K0)
        d = dev(torch, ct)
        out = d if inplace else empty(torch, ct.size)
        c.decrypt_uniform(d, out, n, pb)
        outs.append(host(out))
        assert c.check() == ca.CYAES_OK
        c.close()
    for o in outs:
        assert np.array_equal(o, pt)


def test_context_cycles_with_torch_copies(torch):
    """Contexts created and destroyed back to back, each running in-place
    decrypts (work words and boundary snapshots from its scratch blocks) and
    an aliased-IV decrypt, with torch allocations and host-to-device copies
    in between: the pattern around r04's two illegal-address reports, which
    came from a torch copy right after a context and its stream-ordered
    scratch pool were destroyed.  Bit-exact every cycle."""
    n, pb = 96, 1472
    pt = oracle.synthetic(31, n, pb)
    ct = oracle.batch(False, [K0], 0, pt, pb, nthreads=4)
    last = ct.reshape(n, pb // 16, 16)[:, -1].copy()
    for cycle in range(120):
        c = ca.GpuContext(0)
        c.set_keys(K0)
        d = dev(torch, ct)
        c.decrypt_uniform(d, d, n, pb)
        ivs = dev(torch, np.zeros((n, 16), np.uint8))
        c.decrypt_uniform(dev(torch, ct), empty(torch, ct.size), n, pb, iv_in=ivs, iv_out=ivs)
        junk = dev(torch, np.full(1 << 20, cycle & 0xFF, np.uint8))  # torch's allocator and copies in between
        assert np.array_equal(host(d), pt), cycle
        assert np.array_equal(host(ivs).reshape(n, 16), last), cycle
        assert c.check() == ca.CYAES_OK
        c.close()
        del d, ivs, junk


def test_concurrent_flat_and_ragged_decrypts(torch):
    """A flat and a ragged decrypt (and two flat ones) on two streams at once,
    repeatedly: each launch has its own ticket counter and progress words
    (DecArgs.work), so neither disturbs the other (VERDICT r03 weak 7 / next 6;
    the relay decrypts on its loopers, relay_server.cpp:329, while a drop-in
    caller decrypts, cyr_rijndael.cpp:612-635)."""
    pb, n = 1472, 65536
    hdr, stride = 12, pb + 12
    c = ca.GpuContext(0)
    c.set_keys(K0)
    pt = oracle.synthetic(21, n, pb)
    ct = oracle.batch(False, [K0], 0, pt, pb, nthreads=16)
    flat = dev(torch, ct)
    flat2 = dev(torch, ct)
    stream_buf = np.full(n * stride + 16, 0xA5, np.uint8)
    stream_buf[:n * stride].reshape(n, stride)[:, hdr:hdr + pb] = ct.reshape(n, pb)
    rbuf = dev(torch, stream_buf)
    off = dev(torch, np.arange(n, dtype=np.uint64) * stride + hdr)
    nb = dev(torch, np.full(n, pb, np.uint32))
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    for rep in range(4):  # decrypt, then encrypt back, on both streams, both orders
        a, b = (s1, s2) if rep % 2 == 0 else (s2, s1)
        c.decrypt_uniform(flat, flat, n, pb, stream=a.cuda_stream)
        c.decrypt_ragged(rbuf, rbuf, off, nb, n, stream=b.cuda_stream)
        c.decrypt_uniform(flat2, flat2, n, pb, stream=b.cuda_stream)
        c.encrypt_uniform(flat, flat, n, pb, stream=a.cuda_stream)
        c.encrypt_ragged(rbuf, rbuf, off, nb, n, stream=b.cuda_stream)
        c.encrypt_uniform(flat2, flat2, n, pb, stream=b.cuda_stream)
        torch.cuda.synchronize()  # the next rep swaps the streams: a buffer's ops stay ordered
    c.decrypt_uniform(flat, flat, n, pb, stream=s1.cuda_stream)
    c.decrypt_ragged(rbuf, rbuf, off, nb, n, stream=s2.cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(host(flat), pt)
    assert np.array_equal(host(flat2), ct)
    got = host(rbuf)
    assert np.array_equal(got[:n * stride].reshape(n, stride)[:, hdr:hdr + pb].reshape(-1), pt)
    assert (got[:n * stride].reshape(n, stride)[:, :hdr] == 0xA5).all()
    assert c.check() == ca.CYAES_OK
    c.close()


def test_session_keys_payloads_per_key(torch, ctx):
    """Config D shape, scaled: keys grouped by payload (payload p uses key p / ppk)."""
    nk, ppk, pb = 24, 7, 1472
    n = nk * ppk
    keys = [oracle.session_key(s) for s in range(nk)]
    c = ca.GpuContext(0)
    c.set_keys(b"".join(keys))
    pt = oracle.synthetic(0, n, pb)
    want = oracle.batch(False, keys, ppk, pt, pb, nthreads=16)
    d_pt, d_ct, d_rt = dev(torch, pt), empty(torch, pt.size), empty(torch, pt.size)
    c.encrypt_uniform(d_pt, d_ct, n, pb, payloads_per_key=ppk)
    assert np.array_equal(host(d_ct), want)
    c.decrypt_uniform(d_ct, d_rt, n, pb, payloads_per_key=ppk)
    assert np.array_equal(host(d_rt), pt)
    with pytest.raises(ca.CyaesError):  # (n-1)/ppk >= nkeys
        c.encrypt_uniform(d_pt, d_ct, n + ppk, pb, payloads_per_key=ppk)
    c.close()


@pytest.mark.parametrize("pb,ppk,nk", [(1472, 256, 6), (65536, 3, 4), (208, 1000, 3), (4096, 1, 700), (1024, 16, 300)])
def test_session_keys_uniform_steps(torch, encrypt_kernel, pb, ppk, nk):
    """Sessions spanning many decrypt steps (config D: 256 x 1472 B per key).
    Sessions that are whole steps long (1472 x 256, 65536 x 3, 4096 x 1, 1024 x 16)
    take the session-aligned decrypt (schedule chosen per step, several sessions
    per wave); 208 x 1000 takes the per-lane one-key-per-step check and the
    waterfall of steps that straddle a session boundary."""
    n = nk * ppk - 5  # last session partial
    keys = [oracle.session_key(100 + s) for s in range(nk)]
    c = ca.GpuContext(0)
    c.set_keys(b"".join(keys))
    pt = oracle.synthetic(11, n, pb)
    want = oracle.batch(False, keys, ppk, pt, pb, nthreads=16)
    d_pt, d_ct, d_rt = dev(torch, pt), empty(torch, pt.size), empty(torch, pt.size)
    c.encrypt_uniform(d_pt, d_ct, n, pb, payloads_per_key=ppk)
    assert np.array_equal(host(d_ct), want)
    c.decrypt_uniform(d_ct, d_rt, n, pb, payloads_per_key=ppk)
    assert np.array_equal(host(d_rt), pt)
    c.decrypt_uniform(d_ct, d_ct, n, pb, payloads_per_key=ppk)  # in place
    assert np.array_equal(host(d_ct), pt)
    assert c.check() == ca.CYAES_OK
    c.close()


# ------------------------------------------------- host-resident batches --
@pytest.mark.parametrize("pinned", [True, False])
def test_host_batches_streamed(torch, encrypt_kernel, pinned):
    """cyaes_gpu_{en,de}crypt_host: host memory in and out, several chunks per
    call (3-slot ring wraps), per-session keys, pinned and pageable buffers."""
    nk, ppk, pb = 9, 40, 1472
    n = nk * ppk - 3
    keys = [oracle.session_key(s) for s in range(nk)]
    c = ca.GpuContext(0)
    c.set_keys(b"".join(keys))
    pt = oracle.synthetic(5, n, pb)
    want = oracle.batch(False, keys, ppk, pt, pb, nthreads=16)

    def buf(a=None):
        t = torch.empty(pt.size, dtype=torch.uint8, pin_memory=pinned)
        if a is not None:
            t.copy_(torch.from_numpy(a))
        return t
    h_pt, h_ct, h_rt = buf(pt), buf(), buf()
    chunk = 2 * ppk * pb  # 2 sessions per chunk -> 5 chunks
    c.encrypt_host(h_pt, h_ct, n, pb, payloads_per_key=ppk, chunk_bytes=chunk)
    assert np.array_equal(h_ct.numpy(), want)
    c.decrypt_host(h_ct, h_rt, n, pb, payloads_per_key=ppk, chunk_bytes=chunk)
    assert np.array_equal(h_rt.numpy(), pt)
    c.decrypt_host(h_ct, h_ct, n, pb, payloads_per_key=ppk, chunk_bytes=1)  # in place, one session per chunk
    assert np.array_equal(h_ct.numpy(), pt)
    c.encrypt_host(h_pt, h_ct, n, pb, payloads_per_key=ppk)  # default chunk: one
    assert np.array_equal(h_ct.numpy(), want)
    with pytest.raises(ca.CyaesError):  # (n-1)/ppk >= nkeys
        c.encrypt_host(h_pt, h_ct, n, pb, payloads_per_key=ppk // 4)
    with pytest.raises(ca.CyaesError):
        c.encrypt_host(h_pt, h_ct, n, pb + 8)
    c.close()


def _pin_delta(before):
    after = ca.debug_pins()
    return after, {k: after[k] - before[k] for k in after}


def test_host_batch_buffers_sharing_a_page(torch):
    """cyaes_gpu_{en,de}crypt_host on two pageable buffers that share a page (in
    != out, one heap block, the second starting on the first's last page): the
    first is registered for the call (its exact bytes), the second is not
    registered over the page the first's registration holds but bounced through
    the pipe's pinned staging (cyaes_pins.cpp; r04's illegal-address faults,
    DESIGN.md §4.2).  Bit-exact both ways and in place; nothing the library
    registered outlives a call; then a torch pageable copy above 1 MiB (the size
    from which the runtime pins a pageable copy on the fly) from a fresh buffer
    over the freed addresses, also bit-exact.  relay_local.cpp:188-217: socket
    buffer -> encrypt -> send."""
    n, pb = 1500, 1472  # 2.2 MB per buffer
    total = n * pb
    c = ca.GpuContext(0)
    c.set_keys(K0)
    pt = oracle.synthetic(3, n, pb)
    want = oracle.batch(False, [K0], 0, pt, pb, nthreads=16)
    arena = np.zeros(2 * total + 4 * 4096, dtype=np.uint8)  # pageable
    base = arena.ctypes.data
    a_off = (-base) % 4096 + 16
    b_off = a_off + total + 48
    assert (base + a_off + total - 1) // 4096 == (base + b_off) // 4096  # one shared page
    h_a, h_b = arena[a_off:a_off + total], arena[b_off:b_off + total]
    h_a[:] = pt
    for chunk in (0, 5 * 4096 * 1472 // 4096):  # one chunk; several (the 3-slot staging ring wraps)
        h_b[:] = 0
        before = ca.debug_pins()
        c.encrypt_host(h_a.ctypes.data, h_b.ctypes.data, n, pb, chunk_bytes=chunk)
        assert np.array_equal(h_b, want)
        after, d = _pin_delta(before)
        assert after["live"] == 0 and after["refs"] == 0
        assert d["registered"] == 1 and d["unregistered"] == 1 and d["conflicts"] == 1  # in registered, out bounced
        assert after["failed_unregisters"] == 0 and after["stale"] == 0
        h_a[:] = 0
        before = ca.debug_pins()
        c.decrypt_host(h_b.ctypes.data, h_a.ctypes.data, n, pb, chunk_bytes=chunk)  # the other way round
        assert np.array_equal(h_a, pt)
        after, d = _pin_delta(before)
        assert after["live"] == 0 and d["registered"] == 1 and d["conflicts"] == 1
    c.encrypt_host(h_a.ctypes.data, h_a.ctypes.data, n, pb, chunk_bytes=1 << 20)  # in place, registered
    assert np.array_equal(h_a, want)
    assert ca.debug_pins()["live"] == 0
    del h_a, h_b
    arena = None
    fresh = np.random.default_rng(5).integers(0, 256, 2 * total + 4 * 4096, dtype=np.uint8)
    d_fresh = torch.from_numpy(fresh).to("cuda")
    torch.cuda.synchronize()
    assert np.array_equal(d_fresh.cpu().numpy(), fresh)
    c.close()


def test_host_batch_in_foreign_registrations(torch):
    """Host batches over memory someone else registered: a buffer inside one
    foreign registration (torch pinned memory, hipHostMalloc) is used as it is,
    nothing registered; a pageable buffer part of which the caller registered
    itself (torch's cudaHostRegister over its middle pages) is bounced, never
    registered over that registration, which stays intact (its own unregister
    succeeds).  Bit-exact."""
    n, pb = 700, 1472
    total = n * pb
    c = ca.GpuContext(0)
    c.set_keys(K0)
    pt = oracle.synthetic(4, n, pb)
    want = oracle.batch(False, [K0], 0, pt, pb, nthreads=16)
    h_pin = torch.empty(total, dtype=torch.uint8, pin_memory=True)
    h_pin.copy_(torch.from_numpy(pt))
    before = ca.debug_pins()
    c.encrypt_host(h_pin, h_pin, n, pb)
    assert np.array_equal(h_pin.numpy(), want)
    after, d = _pin_delta(before)
    assert d["registered"] == 0 and d["conflicts"] == 0 and after["live"] == 0
    arena = np.zeros(total + 4 * 4096, dtype=np.uint8)
    off = (-arena.ctypes.data) % 4096 + 64
    buf = arena[off:off + total]
    buf[:] = pt
    lo = arena.ctypes.data + off - 64 + 2 * 4096  # pages 2..4 of the buffer, registered by "the caller"
    assert hiprt.host_register(lo, 3 * 4096) == 0
    try:
        before = ca.debug_pins()
        c.encrypt_host(buf.ctypes.data, buf.ctypes.data, n, pb, chunk_bytes=256 * 1472)
        assert np.array_equal(buf, want)
        after, d = _pin_delta(before)
        assert d["registered"] == 0 and d["conflicts"] == 1 and after["live"] == 0
        c.decrypt_host(buf.ctypes.data, buf.ctypes.data, n, pb)
        assert np.array_equal(buf, pt)
    finally:
        assert hiprt.host_unregister(lo) == 0
    c.close()


def test_set_keys_waits_only_for_its_own_streams(torch):
    """cyaes_gpu_set_keys waits for the streams that read its own context's key
    table, not for the device: while a long decrypt of
    context A runs on a stream, B.set_keys (a new session's context,
    relay_server.cpp:224,229) returns before that decrypt ends; A.update_keys,
    whose table the decrypt reads, returns only after it.  Both bit-exact."""
    n, pb = 65536, 65536  # 4 GiB; three decrypts queued: ~8 ms on the GPU
    a, b = ca.GpuContext(0), ca.GpuContext(0)
    a.set_keys(K0)
    ct = torch.empty(n * pb, dtype=torch.uint8, device="cuda")
    pt = torch.empty_like(ct)
    a.fill_synthetic(ct, 0, n, pb, oracle.PLAINTEXT_SEED)
    want = a.digest(ct, n * pb)
    a.encrypt_uniform(ct, ct, n, pb)
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    end = torch.cuda.Event()
    with torch.cuda.stream(s):
        for _ in range(3):
            a.decrypt_uniform(ct, pt, n, pb, stream=s.cuda_stream)
        end.record(s)
    keys_b = [oracle.session_key(i) for i in range(5)]
    b.set_keys(b"".join(keys_b))
    b_returned_early = not end.query()
    a.update_keys(0, K0)  # the running decrypts read this row
    a_waited = end.query()
    torch.cuda.synchronize()
    a.update_keys(1, oracle.session_key(9))  # appended (the table grows; the old one is kept until close)
    assert a.get_key(0).words() == ca.key_expand(K0).words()
    assert b_returned_early, "set_keys on another context waited for this context's decrypt"
    assert a_waited, "update_keys returned while a batch still read the rows it replaced"
    assert a.digest(pt, n * pb) == want
    small = oracle.synthetic(6, 64, 1024)
    d_in = torch.from_numpy(small.copy()).to("cuda")
    d_out = torch.empty_like(d_in)
    b.encrypt_uniform(d_in, d_out, 64, 1024, payloads_per_key=16)
    assert np.array_equal(host(d_out), oracle.batch(False, keys_b, 16, small, 1024))
    assert a.check() == ca.CYAES_OK
    a.close()
    b.close()


def test_set_keys_device_back_to_back_on_two_streams(torch):
    """Two cyaes_gpu_set_keys_device calls on two streams, the first queued
    behind an ~8 ms decrypt of another context: the second key set wins,
    bit-exactly (its expansion waits on the device for the first's; VERDICT r05
    weak 5).  Per-session keys arrive by broadcast and are expanded where they
    land (relay_server.cpp:218-240, a new Rijndael per session at :224,229)."""
    n, pb = 65536, 65536
    a, b = ca.GpuContext(0), ca.GpuContext(0)
    a.set_keys(K0)
    b.set_keys(K0)
    ct = torch.empty(n * pb, dtype=torch.uint8, device="cuda")
    pt = torch.empty_like(ct)
    b.fill_synthetic(ct, 0, n, pb, oracle.PLAINTEXT_SEED)
    keys1 = [oracle.session_key(100 + i) for i in range(6)]
    keys2 = [oracle.session_key(200 + i) for i in range(6)]
    d1 = torch.from_numpy(np.frombuffer(b"".join(keys1), np.uint8).copy()).to("cuda")
    d2 = torch.from_numpy(np.frombuffer(b"".join(keys2), np.uint8).copy()).to("cuda")
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    end = torch.cuda.Event()
    with torch.cuda.stream(s1):
        for _ in range(3):
            b.decrypt_uniform(ct, pt, n, pb, stream=s1.cuda_stream)  # b's table: a's writes need not wait for it
        a.set_keys_device(d1, 6, stream=s1.cuda_stream)
        end.record(s1)
    a.set_keys_device(d2, 6, stream=s2.cuda_stream)
    queued_behind = not end.query()
    for i in range(6):
        assert a.get_key(i).words() == ca.key_expand(keys2[i]).words(), i
    small = oracle.synthetic(7, 6 * 16, 1024)
    d_in = torch.from_numpy(small.copy()).to("cuda")
    d_out = torch.empty_like(d_in)
    a.encrypt_uniform(d_in, d_out, 6 * 16, 1024, payloads_per_key=16)
    assert np.array_equal(host(d_out), oracle.batch(False, keys2, 16, small, 1024))
    assert queued_behind, "the first expansion was not still queued when the second was issued"
    assert a.check() == ca.CYAES_OK
    a.close()
    b.close()


def test_key_uses_bounded_over_short_lived_streams(torch):
    """1,000 batches, each on a stream of its own created and destroyed around
    it (a caller that opens a stream per request): the context's record of
    streams reading its key table keeps only those with a batch in flight
    (cyaes_debug_ctx), and a key write afterwards waits for nothing stale.
    Every batch bit-exact."""
    c = ca.GpuContext(0)
    c.set_keys(K0)
    n, pb = 64, 1024
    pt = oracle.synthetic(8, n, pb)
    want = oracle.batch(False, [K0], 0, pt, pb)
    d_in = torch.from_numpy(pt.copy()).to("cuda")
    outs = [torch.empty_like(d_in) for _ in range(4)]
    torch.cuda.synchronize()
    peak = 0
    for i in range(1000):
        s = hiprt.stream_create()
        out = outs[i % 4]
        if i % 2:
            c.encrypt_uniform(d_in, out, n, pb, stream=s)
        else:
            c.encrypt_strided(d_in, out, 0, pb, n, pb, stream=s)
        if i % 97 == 0:
            hiprt.stream_sync(s)
            assert np.array_equal(host(out), want), i
        hiprt.stream_destroy(s)
        peak = max(peak, c.debug_state()["key_uses"])
    torch.cuda.synchronize()
    c.encrypt_uniform(d_in, outs[0], n, pb)
    torch.cuda.synchronize()
    st = c.debug_state()
    assert st["key_uses"] <= 1, st
    assert peak < 200, peak  # (bounded by the batches in flight, not by the 1,000 streams)
    c.update_keys(0, K0)  # waits for the one reader left
    assert c.debug_state()["key_uses"] == 0
    assert np.array_equal(host(outs[0]), want)
    c.close()


def test_host_batch_single_key_large(torch, ctx):
    """One key, 64 KiB payloads, 4 chunks of 4 MiB."""
    n, pb = 256, 65536
    pt = oracle.synthetic(0, n, pb)
    want = oracle.batch(False, [K0], 0, pt, pb, nthreads=16)
    h_ct = np.empty_like(pt)
    ctx.encrypt_host(pt.ctypes.data, h_ct.ctypes.data, n, pb, chunk_bytes=4 << 20)
    assert np.array_equal(h_ct, want)
    h_rt = np.empty_like(pt)
    ctx.decrypt_host(h_ct.ctypes.data, h_rt.ctypes.data, n, pb, chunk_bytes=4 << 20)
    assert np.array_equal(h_rt, pt)


def test_key_index_array_divergent_waves(torch, encrypt_kernel):
    """Arbitrary per-payload key indices: several keys inside one wave (waterfall)."""
    rng = np.random.default_rng(9)
    nk, pb, n = 37, 208, 3000
    keys = [bytes(rng.integers(0, 256, 16, dtype=np.uint8)) for _ in range(nk)]
    kidx = rng.integers(0, nk, n, dtype=np.uint32)
    c = ca.GpuContext(0)
    c.set_keys(b"".join(keys))
    pt = oracle.synthetic(3, n, pb)
    want = np.concatenate([oracle.batch(False, [keys[kidx[p]]], 0, pt[p * pb:(p + 1) * pb], pb) for p in range(n)])
    d_pt, d_ct, d_rt, d_k = dev(torch, pt), empty(torch, pt.size), empty(torch, pt.size), dev(torch, kidx)
    c.encrypt_uniform(d_pt, d_ct, n, pb, key_idx=d_k)
    assert np.array_equal(host(d_ct), want)
    c.decrypt_uniform(d_ct, d_rt, n, pb, key_idx=d_k)
    assert np.array_equal(host(d_rt), pt)
    assert c.check() == ca.CYAES_OK
    bad = kidx.copy()
    bad[17] = nk + 3
    c.encrypt_uniform(d_pt, d_ct, n, pb, key_idx=dev(torch, bad))
    assert c.check() == ca.CYAES_ERANGE  # reported, then cleared
    assert c.check() == ca.CYAES_OK
    # the stream-scoped check (waits for that stream only) reports and clears the same flag
    s = torch.cuda.Stream()
    d_bad = dev(torch, bad)
    s.wait_stream(torch.cuda.current_stream())
    c.encrypt_uniform(d_pt, d_ct, n, pb, key_idx=d_bad, stream=s.cuda_stream)
    assert c.check_stream(s.cuda_stream) == ca.CYAES_ERANGE
    assert c.check_stream(s.cuda_stream) == ca.CYAES_OK and c.check() == ca.CYAES_OK
    c.encrypt_uniform(d_pt, d_ct, n, pb, key_idx=d_k, stream=s.cuda_stream)
    assert c.check_stream(s.cuda_stream) == ca.CYAES_OK
    assert np.array_equal(host(d_ct), want)
    c.close()


@pytest.mark.parametrize("alias", [False, True])
def test_iv_in_out(torch, ctx, alias):
    """Per-payload IV in / final chain out (cyr_rijndael.cpp:594-598, 607-608, 633-634)."""
    rng = np.random.default_rng(1)
    pb, n = 1024 + 48, 1500
    pt = oracle.synthetic(9, n, pb)
    ivs = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    want_ct, want_iv = np.empty_like(pt), np.empty_like(ivs)
    for p in range(n):
        iv = bytearray(ivs[p].tobytes())
        want_ct[p * pb:(p + 1) * pb] = np.frombuffer(
            bytes(oracle.Rijndael(K0).encrypt(pt[p * pb:(p + 1) * pb].tobytes(), None, pb, iv)), np.uint8)
        want_iv[p] = np.frombuffer(bytes(iv), np.uint8)
    d_pt, d_ct, d_rt = dev(torch, pt), empty(torch, pt.size), empty(torch, pt.size)
    d_iv = dev(torch, ivs)
    d_ivo = d_iv if alias else empty(torch, ivs.size)
    ctx.encrypt_uniform(d_pt, d_ct, n, pb, iv_in=d_iv, iv_out=d_ivo)
    assert np.array_equal(host(d_ct), want_ct)
    assert np.array_equal(host(d_ivo).reshape(n, 16), want_iv)
    d_iv2 = dev(torch, ivs)
    d_ivo2 = d_iv2 if alias else empty(torch, ivs.size)
    ctx.decrypt_uniform(d_ct, d_rt, n, pb, iv_in=d_iv2, iv_out=d_ivo2)
    assert np.array_equal(host(d_rt), pt)
    assert np.array_equal(host(d_ivo2).reshape(n, 16), want_iv)  # last ciphertext block


@pytest.mark.parametrize("pb,n", [(16, 1), (16, 3), (4800, 3), (4800, 7), (65280, 2)])
@pytest.mark.parametrize("with_iv", [False, True])
@pytest.mark.parametrize("inplace", [False, True])
def test_decrypt_extent_edges(torch, ctx, pb, n, with_iv, inplace):
    """The two r02 over-reads of k_decrypt_flat's partial last step, pinned
    (VERDICT r02 "What's weak" 1): a 1-block batch, where lanes 1..63 read the
    block before the buffer, and payloads of >= 256 blocks (4,800 B = 300
    blocks; 65,280 B = the relay's largest chunk, 4,080 blocks) with IVs in and
    nblocks % 256 != 0, where the partial step read iv_in[npayloads], 16 B past
    the IV array.  The ciphertext sits at the start of its allocation and the
    IVs at the very end of theirs; the bounds build (tests/conftest.py) names
    any access outside.  Semantics: cyr_rijndael.cpp:612-635 (IV in, last
    ciphertext block out, in place)."""
    rng = np.random.default_rng(pb * 31 + n)
    nbytes = pb * n
    pt = rng.integers(0, 256, nbytes, dtype=np.uint8)
    ivs = rng.integers(0, 256, (n, 16), dtype=np.uint8) if with_iv else np.tile(np.arange(16, dtype=np.uint8), (n, 1))
    want_ct, want_iv = np.empty_like(pt), np.empty_like(ivs)
    for p in range(n):
        iv = bytearray(ivs[p].tobytes())
        want_ct[p * pb:(p + 1) * pb] = np.frombuffer(
            bytes(oracle.Rijndael(K0).encrypt(pt[p * pb:(p + 1) * pb].tobytes(), None, pb, iv)), np.uint8)
        want_iv[p] = np.frombuffer(bytes(iv), np.uint8)
    ct_alloc = torch.empty(nbytes + 4096, dtype=torch.uint8, device="cuda")
    d_ct = ct_alloc[:nbytes]
    d_ct.copy_(torch.from_numpy(want_ct).to("cuda"))
    d_out = d_ct if inplace else empty(torch, nbytes)
    iv_in = iv_out = None
    if with_iv:
        iv_alloc = torch.empty(16 * n + 1024, dtype=torch.uint8, device="cuda")
        iv_in = iv_alloc[-16 * n:]
        iv_in.copy_(torch.from_numpy(ivs.reshape(-1)).to("cuda"))
        iv_out = empty(torch, 16 * n)
    ctx.decrypt_uniform(d_ct, d_out, n, pb, iv_in=iv_in, iv_out=iv_out)
    assert np.array_equal(host(d_out), pt)
    if with_iv:
        assert np.array_equal(host(iv_out).reshape(n, 16), want_iv)  # last ciphertext block per payload
    assert ctx.check() == ca.CYAES_OK


def test_ragged_batches(torch, encrypt_kernel):
    """Relay packets of mixed sizes (0..65280 B), gaps between them, per-payload keys and IVs."""
    rng = np.random.default_rng(4)
    n = 700
    sizes = (rng.integers(0, 4081, n) * 16).astype(np.uint32)
    sizes[:6] = [0, 16, 65280, 1472, 32, 1024]
    gaps = rng.integers(0, 3, n) * 16
    offsets = np.zeros(n, dtype=np.uint64)
    pos = 0
    for p in range(n):
        pos += int(gaps[p])
        offsets[p] = pos
        pos += int(sizes[p])
    nk = 5
    keys = [bytes(rng.integers(0, 256, 16, dtype=np.uint8)) for _ in range(nk)]
    kidx = rng.integers(0, nk, n, dtype=np.uint32)
    ivs = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    data = rng.integers(0, 256, pos, dtype=np.uint8)
    want, want_iv = data.copy(), np.empty_like(ivs)
    for p in range(n):
        o, s = int(offsets[p]), int(sizes[p])
        iv = bytearray(ivs[p].tobytes())
        want[o:o + s] = np.frombuffer(bytes(oracle.Rijndael(keys[kidx[p]]).encrypt(data[o:o + s].tobytes(), None, s, iv)),
                                      np.uint8)
        want_iv[p] = np.frombuffer(bytes(iv), np.uint8)
    c = ca.GpuContext(0)
    c.set_keys(b"".join(keys))
    d_in, d_out = dev(torch, data), dev(torch, data)  # gaps keep their bytes
    d_off, d_nb, d_k = dev(torch, offsets), dev(torch, sizes), dev(torch, kidx)
    d_iv, d_ivo = dev(torch, ivs), empty(torch, ivs.size)
    c.encrypt_ragged(d_in, d_out, d_off, d_nb, n, key_idx=d_k, iv_in=d_iv, iv_out=d_ivo)
    assert np.array_equal(host(d_out), want)
    assert np.array_equal(host(d_ivo).reshape(n, 16), want_iv)
    d_back, d_ivo2 = dev(torch, data), empty(torch, ivs.size)
    c.decrypt_ragged(d_out, d_back, d_off, d_nb, n, key_idx=d_k, iv_in=d_iv, iv_out=d_ivo2)
    assert np.array_equal(host(d_back), data)
    got_iv = host(d_ivo2).reshape(n, 16)
    for p in range(n):
        o, s = int(offsets[p]), int(sizes[p])
        exp = want[o + s - 16:o + s] if s else ivs[p]
        assert np.array_equal(got_iv[p], exp), p
    c.decrypt_ragged(d_out, d_out, d_off, d_nb, n, key_idx=d_k, iv_in=d_iv)  # in place
    assert np.array_equal(host(d_out), data)
    c.close()


@pytest.fixture(params=["1", "3", "64", "auto"])
def ragged_group(request):
    """Payloads per wave group of the ragged decrypt: forced, or the runtime's choice."""
    old = os.environ.get("CYAES_RAGGED_GROUP")
    if request.param == "auto":
        os.environ.pop("CYAES_RAGGED_GROUP", None)
    else:
        os.environ["CYAES_RAGGED_GROUP"] = request.param
    yield request.param
    if old is None:
        os.environ.pop("CYAES_RAGGED_GROUP", None)
    else:
        os.environ["CYAES_RAGGED_GROUP"] = old


@pytest.mark.parametrize("keying", ["one", "index", "ppk"])
def test_ragged_decrypt_groups(torch, ragged_group, keying):
    """Relay-packet streams in HBM (payload at packet offset 12, 4-B aligned):
    mostly small packets with empty and one-block ones, a few 65,280-B ones;
    rows of a wave span several payloads (group > 1).  Keys per payload
    (index array, sessions of 7 payloads) or one key; IV in/out; in place."""
    rng = np.random.default_rng(21)
    n = 2500
    blocks = rng.choice([0, 1, 2, 5, 63, 64, 65, 92, 200], n).astype(np.uint32)
    blocks[rng.integers(0, n, 12)] = 4080
    sizes = blocks * 16
    offsets = np.zeros(n, dtype=np.uint64)
    pos = 0
    for p in range(n):
        offsets[p] = pos + 12  # packet header: 4-B head + 8-B forward msg
        pos += 12 + int(sizes[p])
    nk = 9
    keys = [bytes(rng.integers(0, 256, 16, dtype=np.uint8)) for _ in range(nk)]
    ppk = 7 if keying == "ppk" else 0
    if keying == "index":
        kidx = rng.integers(0, nk, n, dtype=np.uint32)
    elif keying == "ppk":
        kidx = (np.arange(n) // ppk % nk).astype(np.uint32)
        keys = [keys[(s) % nk] for s in range(n // ppk + 1)]
    else:
        kidx = np.zeros(n, dtype=np.uint32)
    ivs = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    plain = rng.integers(0, 256, pos, dtype=np.uint8)
    ct = plain.copy()
    for p in range(n):
        o, s = int(offsets[p]), int(sizes[p])
        k = keys[p // ppk] if ppk else keys[kidx[p]]
        ct[o:o + s] = np.frombuffer(bytes(oracle.Rijndael(k).encrypt(plain[o:o + s].tobytes(), None, s,
                                                                      bytearray(ivs[p].tobytes()))), np.uint8)
    c = ca.GpuContext(0)
    c.set_keys(b"".join(keys))
    d_off, d_nb = dev(torch, offsets), dev(torch, sizes)
    d_k = dev(torch, kidx) if keying == "index" else None
    d_iv, d_ivo = dev(torch, ivs), empty(torch, ivs.size)
    d_ct, d_back = dev(torch, ct), dev(torch, ct)  # headers / untouched bytes keep their values
    c.decrypt_ragged(d_ct, d_back, d_off, d_nb, n, key_idx=d_k, payloads_per_key=ppk, iv_in=d_iv, iv_out=d_ivo)
    got = host(d_back)
    for p in np.flatnonzero(sizes):
        o, s = int(offsets[p]), int(sizes[p])
        assert np.array_equal(got[o:o + s], plain[o:o + s]), (p, int(blocks[p]))
    hdr = np.ones(pos, dtype=bool)
    for p in range(n):
        hdr[int(offsets[p]):int(offsets[p]) + int(sizes[p])] = False
    assert np.array_equal(got[hdr], ct[hdr])  # nothing outside the payloads is written
    got_iv = host(d_ivo).reshape(n, 16)
    for p in range(n):
        o, s = int(offsets[p]), int(sizes[p])
        assert np.array_equal(got_iv[p], ct[o + s - 16:o + s] if s else ivs[p]), p
    c.decrypt_ragged(d_ct, d_ct, d_off, d_nb, n, key_idx=d_k, payloads_per_key=ppk, iv_in=d_iv)  # in place
    assert np.array_equal(host(d_ct), got)
    assert c.check() == ca.CYAES_OK
    c.close()


def test_ragged_offsets_beyond_4gib(torch, ragged_group, encrypt_kernel):
    """Payload offsets >= 2^31 and >= 2^32 (a batch base pointer far below the
    data): the 64-bit offset arithmetic of both ragged kernels."""
    rng = np.random.default_rng(5)
    n = 300
    sizes = (rng.choice([0, 1, 3, 92, 300], n) * 16).astype(np.uint32)
    offsets = np.zeros(n, dtype=np.uint64)
    pos = 0
    for p in range(n):
        offsets[p] = pos
        pos += int(sizes[p]) + 12
    data = rng.integers(0, 256, pos, dtype=np.uint8)
    want = data.copy()
    for p in range(n):
        o, s = int(offsets[p]), int(sizes[p])
        want[o:o + s] = np.frombuffer(bytes(oracle.Rijndael(K0).encrypt(data[o:o + s].tobytes())), np.uint8)
    c = ca.GpuContext(0)
    c.set_keys(K0)
    for bias in ((1 << 31) + 4, (5 << 32) + 1024):
        d = dev(torch, data)
        base = d.data_ptr() - bias  # in/out point `bias` bytes below the data
        d_off = dev(torch, offsets + np.uint64(bias))
        d_nb = dev(torch, sizes)
        c.encrypt_ragged(base, base, d_off, d_nb, n)
        assert np.array_equal(host(d), want)
        c.decrypt_ragged(base, base, d_off, d_nb, n)
        assert np.array_equal(host(d), data)
    assert c.check() == ca.CYAES_OK
    c.close()


def test_device_key_expansion(torch):
    """Keys already on the device (e.g. after the RCCL broadcast) are expanded there."""
    rng = np.random.default_rng(12)
    nk = 300
    raw = rng.integers(0, 256, (nk, 16), dtype=np.uint8)
    c = ca.GpuContext(0)
    c.set_keys_device(dev(torch, raw), nk)
    torch.cuda.synchronize()
    for i in list(range(5)) + [nk - 1]:
        assert c.get_key(i).words() == oracle.key_expand(raw[i].tobytes()).words()
    pb, n = 160, nk
    pt = oracle.synthetic(0, n, pb)
    want = np.concatenate([oracle.batch(False, [raw[p].tobytes()], 0, pt[p * pb:(p + 1) * pb], pb) for p in range(n)])
    d_ct = empty(torch, pt.size)
    c.encrypt_uniform(dev(torch, pt), d_ct, n, pb, payloads_per_key=1)
    assert np.array_equal(host(d_ct), want)
    c.close()


def test_fill_and_digest_match_oracle(torch, ctx):
    pb, n = 1472, 300
    d = empty(torch, pb * n)
    ctx.fill_synthetic(d, 77, n, pb, oracle.PLAINTEXT_SEED)
    want = oracle.synthetic(77, n, pb)
    assert np.array_equal(host(d), want)
    assert ctx.digest(d, pb * n) == oracle.digest(want)


# ------------------------------------------------- full BASELINE configs --
@pytest.mark.parametrize("name", ["B", "D", "C", "E_rank1"])
def test_full_config_digest(torch, golden, name):
    """Full-size configs on the device vs OpenSSL-derived goldens (checksum of
    checksums), the round trip, and sampled payloads vs the oracle."""
    cfg = golden["openssl"]["configs"][name]
    n, pb, ppk, p0 = cfg["npayloads"], cfg["payload_bytes"], cfg["payloads_per_key"], cfg["p0"]
    c = ca.GpuContext(0)
    if ppk:
        keys = [oracle.session_key(s) for s in range(n // ppk)]
        c.set_keys(b"".join(keys))
    else:
        keys = [K0]
        c.set_keys(K0)
    nbytes = n * pb
    d_pt, d_ct = empty(torch, nbytes), empty(torch, nbytes)
    c.fill_synthetic(d_pt, p0, n, pb, oracle.PLAINTEXT_SEED)
    assert ["%016x" % v for v in c.digest(d_pt, nbytes)] == cfg["plain_digest"]
    c.encrypt_uniform(d_pt, d_ct, n, pb, payloads_per_key=ppk)
    assert ["%016x" % v for v in c.digest(d_ct, nbytes)] == cfg["cipher_digest"]
    for p in (0, 1, n // 2 + 3, n - 1):
        pt = oracle.synthetic(p0 + p, 1, pb)
        want = oracle.batch(False, [keys[p // ppk] if ppk else K0], 0, pt, pb)
        torch.cuda.synchronize()
        assert np.array_equal(d_ct[p * pb:(p + 1) * pb].cpu().numpy(), want), p
    c.decrypt_uniform(d_ct, d_ct, n, pb, payloads_per_key=ppk)  # in place
    assert ["%016x" % v for v in c.digest(d_ct, nbytes)] == cfg["plain_digest"]
    assert c.check() == ca.CYAES_OK
    del d_pt, d_ct
    torch.cuda.empty_cache()
    c.close()


@pytest.mark.parametrize("run,pb,ppk,nk", [("1", 1472, 64, 9), ("2", 1472, 256, 5), ("4", 208, 256, 7),
                                           ("2", 1472, 192, 6), ("0", 1024, 128, 20)])
def test_encrypt_whole_wave_sessions_and_runs(torch, run, pb, ppk, nk):
    """k_encrypt SESS (sessions that hold whole waves of work items: the key
    is per wave, from the scalar position) with and without RUNS (R
    consecutive payloads per lane as one block stream, chain restarts at
    DefaultIV), forced onto small batches through the lane kernel, against the
    oracle; the last session and the last run are partial."""
    n = ppk * nk - 37
    keys = [oracle.session_key(s) for s in range(nk)]
    old = {k: os.environ.get(k) for k in ("CYAES_QUAD_MAX_CHAINS", "CYAES_ENC_RUN")}
    os.environ["CYAES_QUAD_MAX_CHAINS"] = "0"
    os.environ["CYAES_ENC_RUN"] = run
    try:
        c = ca.GpuContext(0)
    finally:
        _restore(old)
    c.set_keys(b"".join(keys))
    pt = oracle.synthetic(5, n, pb)
    want = oracle.batch(False, keys, ppk, pt, pb, nthreads=16)
    d_pt, d_ct, d_rt = dev(torch, pt), empty(torch, pt.size), empty(torch, pt.size)
    c.encrypt_uniform(d_pt, d_ct, n, pb, payloads_per_key=ppk)
    c.decrypt_uniform(d_ct, d_rt, n, pb, payloads_per_key=ppk)
    assert np.array_equal(host(d_ct), want)
    assert np.array_equal(host(d_rt), pt)
    assert c.check() == ca.CYAES_OK
    c.close()


@pytest.mark.parametrize("seed", range(12))
def test_duplex_sweep(torch, seed):
    """Seeded duplex launches (cyaes_gpu_duplex_uniform): random
    halves (sizes, payload lengths from one block to 64 KiB, key rows, in
    place or not) under random pool shares and range sizes of the decrypt phase
    (CYAES_DUPLEX_DYN_PCT, CYAES_DEC_RANGE_STEPS), against the two ordinary
    launches of reference contexts, bit-exact, and the round trip."""
    rng = np.random.default_rng(4000 + seed)
    keys = [K0, oracle.session_key(3), oracle.session_key(4)]
    epb = int(rng.choice([16, 64, 1472, 4096]))
    en = int(rng.choice([131072, 200003, 262144, 300000])) if epb <= 1472 else int(rng.choice([131072, 180000]))
    dpb = int(rng.choice([16, 1024, 1472, 65536]))
    dn = int(rng.choice([1000, 50000, 262144])) if dpb <= 1472 else int(rng.choice([257, 4000]))
    ek, dk = int(rng.integers(0, 3)), int(rng.integers(0, 3))
    e_inplace, d_inplace = bool(rng.integers(0, 2)), bool(rng.integers(0, 2))
    env = {"CYAES_DUPLEX_DYN_PCT": str(rng.choice([10, 25, 50, 100])),
           "CYAES_DEC_RANGE_STEPS": str(rng.choice([1, 4, 16]))}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        c = ca.GpuContext(0)
    finally:
        _restore(old)
    c.set_keys(b"".join(keys))
    ref = [ca.GpuContext(0) for _ in keys]
    for r, k in zip(ref, keys):
        r.set_keys(k)
    e_in, d_in = empty(torch, en * epb), empty(torch, dn * dpb)
    c.fill_synthetic(e_in, 3, en, epb, oracle.PLAINTEXT_SEED)
    c.fill_synthetic(d_in, 5, dn, dpb, oracle.PLAINTEXT_SEED)
    want_e, want_d = empty(torch, en * epb), empty(torch, dn * dpb)
    ref[ek].encrypt_uniform(e_in, want_e, en, epb)
    ref[dk].decrypt_uniform(d_in, want_d, dn, dpb)
    e_src, d_src = e_in.clone(), d_in.clone()
    e_out = e_in if e_inplace else empty(torch, en * epb)
    d_out = d_in if d_inplace else empty(torch, dn * dpb)
    c.duplex_uniform(e_in, e_out, en, epb, d_in, d_out, dn, dpb, enc_key=ek, dec_key=dk)
    assert torch.equal(e_out, want_e), (en, epb, ek, env)
    assert torch.equal(d_out, want_d), (dn, dpb, dk, env)
    back = empty(torch, en * epb)
    ref[ek].decrypt_uniform(e_out, back, en, epb)
    assert torch.equal(back, e_src)
    if not d_inplace:
        assert torch.equal(d_in, d_src)
    assert c.check() == ca.CYAES_OK
    for r in ref:
        r.close()
    c.close()
    torch.cuda.empty_cache()


@pytest.mark.parametrize("shape", ["relay", "relay_rest", "relay_big", "short", "aligned", "lists", "overlap",
                                   "empty_dec", "off", "relay_pool"])
def test_duplex_strided_matches_two_strided_calls(torch, shape):
    """cyaes_gpu_duplex_strided (two relay streams, one launch: relay_server.cpp
    :472 encrypts the sent stream while :329 decrypts the received one) against
    cyaes_gpu_encrypt_strided + cyaes_gpu_decrypt_strided of reference contexts
    (one per key row), bit-exact, bytes between payloads untouched, in place:
    relay packets (payload at offset 12, stride 1,484) with whole 1,024-payload
    line groups and a rest; >= 256-block payloads; shapes that fall back to the
    two calls (short streams, 16-B aligned back-to-back payloads, < 64-block
    decrypt payloads that take the ragged kernel, overlapping streams, an empty
    half, CYAES_DUPLEX=0); the decrypt's pool share forced to 100 %."""
    keys = [K0, oracle.session_key(5), oracle.session_key(6)]
    env = {"off": {"CYAES_DUPLEX": "0"}, "relay_pool": {"CYAES_DUPLEX_DYN_PCT": "100"}}.get(shape, {})
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        c = ca.GpuContext(0)
    finally:
        _restore(old)
    c.set_keys(b"".join(keys))
    ref = [ca.GpuContext(0) for _ in keys]
    for r, k in zip(ref, keys):
        r.set_keys(k)
    # (first, stride, n, payload bytes) per half
    e, d = {"relay": ((12, 1484, 1 << 20, 1472), (12, 1484, 300000, 1472)),
            "relay_rest": ((12, 1484, 262144 + 437, 1472), (44, 1500, 200003, 1472)),
            "relay_big": ((12, 4108, 262144, 4096), (12, 65548, 3000, 65536)),
            "short": ((12, 1484, 900, 1472), (12, 1484, 100000, 1472)),
            "aligned": ((0, 1472, 300000, 1472), (0, 2048, 300000, 2048)),
            "lists": ((12, 1484, 262144, 1472), (12, 524, 300000, 512)),
            "overlap": ((12, 1484, 262144, 1472), (12, 1484, 262144, 1472)),
            "empty_dec": ((12, 1484, 262144, 1472), (12, 1484, 0, 1472)),
            "off": ((12, 1484, 262144, 1472), (12, 1484, 300000, 1472)),
            "relay_pool": ((12, 1484, 1 << 20, 1472), (12, 1484, 1 << 20, 1472))}[shape]
    ek, dk = (1, 2) if shape in ("relay", "relay_big", "relay_rest") else (0, 0)

    def span(h):
        f, s, n, pb = h
        return ((f + (n - 1) * s + pb + 16) // 16 * 16) if n else 16
    e_buf = empty(torch, span(e))
    d_buf = e_buf if shape == "overlap" else empty(torch, span(d))
    c.fill_synthetic(e_buf, 3, e_buf.numel() // 16, 16, oracle.PLAINTEXT_SEED)
    if shape != "overlap":
        c.fill_synthetic(d_buf, 9, d_buf.numel() // 16, 16, oracle.PLAINTEXT_SEED)
    want_e, want_d = e_buf.clone(), (e_buf.clone() if shape == "overlap" else d_buf.clone())
    if shape == "overlap":  # encrypt-then-decrypt order on one buffer
        ref[ek].encrypt_strided(want_e, want_e, *e)
        want_d = want_e
        ref[dk].decrypt_strided(want_d, want_d, *d)
    else:
        ref[ek].encrypt_strided(want_e, want_e, *e)
        if d[2]:
            ref[dk].decrypt_strided(want_d, want_d, *d)
    c.duplex_strided(e_buf, e_buf, *e, d_buf, d_buf, *d, enc_key=ek, dec_key=dk)
    assert torch.equal(e_buf, want_e), (shape, e)
    assert torch.equal(d_buf, want_d), (shape, d)
    if shape != "overlap":  # the sent stream decrypts back
        ref[ek].decrypt_strided(e_buf, e_buf, *e)
        chk = empty(torch, span(e))
        c.fill_synthetic(chk, 3, chk.numel() // 16, 16, oracle.PLAINTEXT_SEED)
        assert torch.equal(e_buf, chk)
    with pytest.raises(ca.CyaesError):
        c.duplex_strided(e_buf, e_buf, 2, 1484, 4, 1472, d_buf, d_buf, 12, 1484, 4, 1472)  # first % 4
    with pytest.raises(ca.CyaesError):
        c.duplex_strided(e_buf, e_buf, 12, 1484, 4, 1472, d_buf, d_buf, 12, 1484, 4, 1472, dec_key=3)
    assert c.check() == ca.CYAES_OK
    for r in ref:
        r.close()
    c.close()
    torch.cuda.empty_cache()


@pytest.mark.parametrize("layout", ["relay_inplace", "relay_out", "gaps", "half_regular", "sizes", "rest_and_empty"])
def test_ragged_encrypt_by_lines(torch, layout):
    """Ragged encrypts through k_encrypt_rag_lines: waves
    whose 64 payloads (16 apart in a 1,024-payload group) share a line phase
    and a length walk aligned lines; every other wave is handed back to the
    ragged lane kernel through the device list; the rest past the last whole
    group runs as its own batch.  Against a context with the line walk off
    (CYAES_ENC_RAG_LINES=0), bytes outside the payloads untouched, the relay
    stream's first 2,048 payloads also against the oracle, and decrypted back.
    relay_local.cpp:206 encrypts each packet's payload in place."""
    n = 131072 + (437 if layout == "rest_and_empty" else 0)
    rng = np.random.default_rng(77)
    pb = 1472
    if layout in ("relay_inplace", "relay_out"):
        sizes = np.full(n, pb, np.uint32)
        gaps = np.full(n, 12, np.uint64)
    elif layout == "gaps":
        sizes = np.full(n, pb, np.uint32)
        gaps = 12 + 4 * rng.integers(0, 3, n).astype(np.uint64)
    elif layout == "half_regular":  # regular groups, then groups with random gaps
        sizes = np.full(n, pb, np.uint32)
        gaps = np.full(n, 12, np.uint64)
        gaps[n // 2:] += (4 * rng.integers(0, 3, n - n // 2)).astype(np.uint64)
    elif layout == "sizes":  # one phase pattern, lengths that differ inside some waves
        sizes = np.full(n, pb, np.uint32)
        sizes[rng.integers(0, n, 300)] = 16 * rng.integers(1, 200, 300)
        gaps = np.full(n, 12, np.uint64)
    else:
        sizes = np.full(n, pb, np.uint32)
        sizes[rng.integers(0, n, 50)] = 0
        gaps = np.full(n, 12, np.uint64)
    pkt = gaps + sizes.astype(np.uint64)
    offsets = (np.cumsum(pkt) - sizes.astype(np.uint64)).astype(np.uint64)
    total = int(offsets[-1] + sizes[-1]) + 64
    old = {"CYAES_ENC_RAG_LINES": os.environ.get("CYAES_ENC_RAG_LINES")}
    os.environ["CYAES_ENC_RAG_LINES"] = "0"
    try:
        ref = ca.GpuContext(0)
    finally:
        _restore(old)
    c = ca.GpuContext(0)
    c.set_keys(K0)
    ref.set_keys(K0)
    buf = empty(torch, (total + 15) // 16 * 16)
    c.fill_synthetic(buf, 0, buf.numel() // 16, 16, oracle.PLAINTEXT_SEED)
    d_off, d_nb = dev(torch, offsets), dev(torch, sizes)
    want = buf.clone()
    ref.encrypt_ragged(want, want, d_off, d_nb, n)
    if layout == "relay_out":
        out = torch.zeros_like(buf)
        want_out = torch.zeros_like(buf)
        ref.encrypt_ragged(buf, want_out, d_off, d_nb, n)
        c.encrypt_ragged(buf, out, d_off, d_nb, n)
        assert torch.equal(out, want_out)
    else:
        src = buf.clone()
        c.encrypt_ragged(buf, buf, d_off, d_nb, n)
        assert torch.equal(buf, want), layout
        if layout == "relay_inplace":  # synthetic payloads: the oracle on a prefix, then back
            view = buf[:n * 1484].view(n, 1484)[:, 12:12 + pb]
            pt_b = empty(torch, n * pb)
            c.fill_synthetic(pt_b, 0, n, pb, oracle.PLAINTEXT_SEED)
            view.copy_(pt_b.view(n, pb))
            c.encrypt_ragged(buf, buf, d_off, d_nb, n)
            ct = view.contiguous().reshape(-1)
            want_b = oracle.batch(False, [K0], 0, pt_b.cpu().numpy()[:2048 * pb], pb, nthreads=16)
            assert np.array_equal(host(ct[:2048 * pb]), want_b)
            c.decrypt_ragged(buf, buf, d_off, d_nb, n)
            assert torch.equal(view.contiguous().reshape(-1), pt_b)
        c.decrypt_ragged(want, want, d_off, d_nb, n)
        assert torch.equal(want, src)
    assert c.check() == ca.CYAES_OK
    ref.close()
    c.close()
    torch.cuda.empty_cache()


def test_mixed_relay_stream_against_golden(torch):
    """bench.py's relay_stream.mixed, full size: config B's bytes as a relay
    tunnel stream of 0xFF00-B chunks and the socket reads' tails (29,580
    packets, payload at packet offset 12; relay_local.cpp:188-206) encrypted
    then decrypted in place through the ragged entry points; whole-buffer
    digests against tests/golden/relay_mixed.json (the oracle's ragged batch,
    tests/golden/gen_relay_mixed.py).  Also forced onto the static split and
    the one-lane encrypt, which must give the same bytes."""
    import json
    import bench
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "relay_mixed.json")))
    offsets, nbytes, alloc = bench.mixed_stream_layout(g["chunk_bytes"])
    assert (int(offsets.size), alloc) == (g["packets"], g["stream_bytes"])
    d_off, d_nb = dev(torch, offsets), dev(torch, nbytes)
    buf = empty(torch, alloc)
    for env in ({}, {"CYAES_DEC_DYN": "0", "CYAES_QUAD_MAX_CHAINS": "0"}):
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            c = ca.GpuContext(0)
        finally:
            _restore(old)
        c.set_keys(K0)
        c.fill_synthetic(buf, 0, alloc // 16, 16, oracle.PLAINTEXT_SEED)
        assert _digest_hex(c, buf, alloc) == g["plain_digest"]
        c.encrypt_ragged(buf, buf, d_off, d_nb, int(offsets.size))
        assert _digest_hex(c, buf, alloc) == g["cipher_digest"], env
        c.decrypt_ragged(buf, buf, d_off, d_nb, int(offsets.size))
        assert _digest_hex(c, buf, alloc) == g["plain_digest"], env
        assert c.check() == ca.CYAES_OK
        c.close()
    torch.cuda.empty_cache()


@pytest.mark.parametrize("seed", range(12))
def test_duplex_ragged_random_layouts(torch, seed):
    """cyaes_gpu_duplex_ragged on random tunnel-stream layouts (relay_local.cpp
    :188-206 chunks of 0..0xFF00 B rounded to 16, random 4-B-aligned gaps,
    empty payloads, random key rows; relay_server.cpp:329 decrypts the other
    direction): against encrypt_ragged then decrypt_ragged of reference
    contexts, bit-exact, the gaps untouched.  Few payloads take the concurrent
    scheme (packed encrypt beside the decrypt); many take the two calls."""
    rng = np.random.default_rng(1000 + seed)
    keys = [oracle.session_key(20 + i) for i in range(3)]
    c = ca.GpuContext(0)
    c.set_keys(b"".join(keys))
    ref = [ca.GpuContext(0) for _ in keys]
    for r, k in zip(ref, keys):
        r.set_keys(k)

    def layout(n, maxb):
        nb = (16 * ((rng.integers(0, maxb + 1, n) + 15) // 16)).astype(np.uint32)
        nb[rng.random(n) < 0.05] = 0
        gaps = (4 * rng.integers(0, 8, n)).astype(np.uint64)
        pkt = gaps + nb.astype(np.uint64)
        off = (np.cumsum(pkt) - nb.astype(np.uint64)).astype(np.uint64)
        return off, nb, int(off[-1] + nb[-1]) + 64
    ne = int(rng.choice([1, 7, 300, 2000, 40000]))
    nd = int(rng.choice([1, 64, 5000, 30000]))
    eo, en, ea = layout(ne, int(rng.choice([256, 4096, 0xFF00])) if ne < 40000 else 1500)
    do, dn, da = layout(nd, int(rng.choice([256, 4096, 0xFF00])))
    ek, dk = int(rng.integers(0, 3)), int(rng.integers(0, 3))
    e_buf, d_buf = empty(torch, (ea + 15) // 16 * 16), empty(torch, (da + 15) // 16 * 16)
    c.fill_synthetic(e_buf, seed, e_buf.numel() // 16, 16, oracle.PLAINTEXT_SEED)
    c.fill_synthetic(d_buf, seed + 99, d_buf.numel() // 16, 16, oracle.PLAINTEXT_SEED)
    de_o, de_n, dd_o, dd_n = dev(torch, eo), dev(torch, en), dev(torch, do), dev(torch, dn)
    want_e, want_d = e_buf.clone(), d_buf.clone()
    ref[ek].encrypt_ragged(want_e, want_e, de_o, de_n, ne)
    ref[dk].decrypt_ragged(want_d, want_d, dd_o, dd_n, nd)
    c.duplex_ragged(e_buf, e_buf, de_o, de_n, ne, d_buf, d_buf, dd_o, dd_n, nd, enc_key=ek, dec_key=dk)
    assert torch.equal(e_buf, want_e), (seed, ne, nd)
    assert torch.equal(d_buf, want_d), (seed, ne, nd)
    assert c.check() == ca.CYAES_OK
    for r in ref:
        r.close()
    c.close()
    torch.cuda.empty_cache()


@pytest.mark.parametrize("weights", ["1,1,1,1,1,1,1,1", "1.05,0.97,1.02,0.9,1.1,1,0.95,1.01", "1,0,3,1,1,0.5,2,0",
                                     "0,0,0,0,0,0,0,1"])
@pytest.mark.parametrize("n,pb", [(1 << 20, 1472), (262144, 65536 // 16), (300001, 1024), (4096, 1024), (7, 16)])
def test_xcd_weighted_static_split(torch, weights, n, pb):
    """The XCD-weighted static decrypt split (A/B, CYAES_DEC_XCD_W; VERDICT r05
    next 7): every wave one range, workgroup slot x's waves w_x / sum(w) of
    the steps, slots laid out in order, the last ranges clipped or empty; zero
    weights leave a slot idle.  Out-of-place uniform decrypts against a context
    with the equal split, bit-exact, and back to the plaintext
    (cyr_rijndael.cpp:612-635)."""
    old = {"CYAES_DEC_XCD_W": os.environ.get("CYAES_DEC_XCD_W")}
    os.environ["CYAES_DEC_XCD_W"] = weights
    try:
        c = ca.GpuContext(0)
    finally:
        _restore(old)
    ref = ca.GpuContext(0)
    c.set_keys(K0)
    ref.set_keys(K0)
    pt = empty(torch, n * pb)
    c.fill_synthetic(pt, 0, n, pb, oracle.PLAINTEXT_SEED)
    ct = empty(torch, n * pb)
    ref.encrypt_uniform(pt, ct, n, pb)
    want, got = empty(torch, n * pb), empty(torch, n * pb)
    ref.decrypt_uniform(ct, want, n, pb)
    c.decrypt_uniform(ct, got, n, pb)
    assert torch.equal(got, want), (weights, n, pb)
    assert torch.equal(got, pt)
    assert c.check() == ca.CYAES_OK
    ref.close()
    c.close()
    torch.cuda.empty_cache()


@pytest.mark.parametrize("shape", ["mixed", "mixed_pack4", "many_short", "empty_enc", "empty_dec", "off",
                                   "keys"])
def test_duplex_ragged_matches_two_ragged_calls(torch, shape):
    """cyaes_gpu_duplex_ragged (the relay's sent stream encrypted,
    relay_local.cpp:206, while its received stream is decrypted,
    relay_server.cpp:329) against cyaes_gpu_encrypt_ragged then
    cyaes_gpu_decrypt_ragged of reference contexts (one per key row),
    bit-exact, bytes between payloads untouched: the mixed relay stream (few
    long payloads: packed encrypt beside the decrypt on the context's second
    stream, also at 4 waves per workgroup), many short payloads (the two
    calls), an empty half, CYAES_DUPLEX=0, key rows 1 and 2; the sent stream
    decrypts back; errors for a bad key row."""
    import bench
    keys = [K0, oracle.session_key(5), oracle.session_key(6)]
    env = {"off": {"CYAES_DUPLEX": "0"}, "mixed_pack4": {"CYAES_DUPLEX_PACK": "4"}}.get(shape, {})
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        c = ca.GpuContext(0)
    finally:
        _restore(old)
    c.set_keys(b"".join(keys))
    ref = [ca.GpuContext(0) for _ in keys]
    for r, k in zip(ref, keys):
        r.set_keys(k)

    def layout(kind, seed):
        if kind == "mixed":
            return bench.mixed_stream_layout(96 << 20, seed=seed)
        if kind == "short":
            rng = np.random.default_rng(seed)
            nb = (16 * rng.integers(0, 93, 400000)).astype(np.uint32)
            off = (np.cumsum(nb.astype(np.uint64) + 12) - nb).astype(np.uint64)
            return off, nb, int(off[-1] + nb[-1]) + 16
        return np.zeros(0, np.uint64), np.zeros(0, np.uint32), 16
    ekind, dkind = {"many_short": ("short", "short"), "empty_enc": (None, "mixed"),
                    "empty_dec": ("mixed", None)}.get(shape, ("mixed", "mixed"))
    eo, en, ea = layout(ekind, 11)
    do, dn, da = layout(dkind, 12)
    ek, dk = (1, 2) if shape == "keys" else (0, 0)
    e_buf, d_buf = empty(torch, (ea + 15) // 16 * 16), empty(torch, (da + 15) // 16 * 16)
    c.fill_synthetic(e_buf, 3, e_buf.numel() // 16, 16, oracle.PLAINTEXT_SEED)
    c.fill_synthetic(d_buf, 9, d_buf.numel() // 16, 16, oracle.PLAINTEXT_SEED)
    de_o, de_n = (dev(torch, eo), dev(torch, en)) if en.size else (None, None)
    dd_o, dd_n = (dev(torch, do), dev(torch, dn)) if dn.size else (None, None)
    e_src = e_buf.clone()
    want_e, want_d = e_buf.clone(), d_buf.clone()
    if en.size:
        ref[ek].encrypt_ragged(want_e, want_e, de_o, de_n, int(en.size))
    if dn.size:
        ref[dk].decrypt_ragged(want_d, want_d, dd_o, dd_n, int(dn.size))
    for _ in range(2):  # the second call reuses the context's second stream
        e_buf.copy_(e_src)
        c.fill_synthetic(d_buf, 9, d_buf.numel() // 16, 16, oracle.PLAINTEXT_SEED)
        c.duplex_ragged(e_buf, e_buf, de_o, de_n, int(en.size), d_buf, d_buf, dd_o, dd_n, int(dn.size),
                        enc_key=ek, dec_key=dk)
        assert torch.equal(e_buf, want_e), shape
        assert torch.equal(d_buf, want_d), shape
    if en.size:
        ref[ek].decrypt_ragged(e_buf, e_buf, de_o, de_n, int(en.size))
        assert torch.equal(e_buf, e_src)
    with pytest.raises(ca.CyaesError):  # a bad key row of a non-empty half (an empty half's row is not read)
        c.duplex_ragged(e_buf, e_buf, de_o, de_n, int(en.size), d_buf, d_buf, dd_o, dd_n, int(dn.size),
                        enc_key=3 if en.size else 0, dec_key=0 if en.size else 3)
    assert c.check() == ca.CYAES_OK
    for r in ref:
        r.close()
    c.close()
    torch.cuda.empty_cache()


def test_dropin_size_zero_and_pieces():
    """The drop-in's argument rules: size 0 is a no-op whatever the
    pointers (the reference's loop never runs, cyr_rijndael.cpp:600), and a call
    longer than one combined batch runs as consecutive pieces of one chain
    (CYAES_DROPIN_PIECE lowers the piece size here), IV in and out, in place."""
    import ctypes
    lib = ca.load_library()
    k = ca.key_expand(K0)
    assert lib.cyaes_cbc_encrypt(ctypes.byref(k), None, None, 0, None) == ca.CYAES_OK
    assert lib.cyaes_cbc_decrypt(ctypes.byref(k), None, None, 0, None) == ca.CYAES_OK
    assert lib.cyaes_cbc_encrypt(ctypes.byref(k), None, None, 16, None) == ca.CYAES_EINVAL
    code = ("import os, sys, random\n"
            "sys.path[:0] = [%r, %r]\n"
            "import cyclone_amd as ca, oracle\n"
            "rng = random.Random(5)\n"
            "for size in (4096 * 3 + 16, 4096 * 5, 16 * 1000):\n"
            "    data = bytes(rng.getrandbits(8) for _ in range(size))\n"
            "    iv0 = bytes(rng.getrandbits(8) for _ in range(16))\n"
            "    a, r = ca.Rijndael(%r), oracle.Rijndael(%r)\n"
            "    iv, riv = bytearray(iv0), bytearray(iv0)\n"
            "    buf = bytearray(data); a.encrypt(buf, buf, size, iv)\n"
            "    assert bytes(buf) == bytes(r.encrypt(data, None, size, riv)) and iv == riv\n"
            "    iv, riv = bytearray(iv0), bytearray(iv0); ct = bytes(buf)\n"
            "    a.decrypt(buf, buf, size, iv)\n"
            "    assert bytes(buf) == data and iv == bytearray(ct[-16:])\n"
            "print('pieces ok')\n" % (ROOT, os.path.join(ROOT, "oracle"), K0, K0))
    env = dict(os.environ, CYAES_DROPIN_PIECE="4096")
    r = subprocess.run([__import__("sys").executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "pieces ok" in r.stdout, r.stdout + r.stderr


# ------------------------------------------------------------ duplex launch --
def _digest_hex(c, d, nbytes):
    return ["%016x" % v for v in c.digest(d, nbytes)]


@pytest.mark.parametrize("inplace", [False, True])
def test_duplex_config_b_and_c_goldens(torch, golden, inplace):
    """cyaes_gpu_duplex_uniform (one grid: encrypt one batch, then decrypt
    another; relay_server.cpp:472 and :329, the two directions of a pipe):
    config B encrypted while config C's ciphertext is decrypted, and config C
    encrypted while B's is decrypted, against the committed OpenSSL digests
    (B's and C's ciphertext, the plaintexts back), in and out of place."""
    cfg = golden["openssl"]["configs"]
    c = ca.GpuContext(0)
    c.set_keys(K0)
    sz = {k: (cfg[k]["npayloads"], cfg[k]["payload_bytes"]) for k in ("B", "C")}
    nb = {k: n * pb for k, (n, pb) in sz.items()}
    pt = {k: empty(torch, nb[k]) for k in sz}
    for k, (n, pb) in sz.items():
        c.fill_synthetic(pt[k], 0, n, pb, oracle.PLAINTEXT_SEED)
    ct_c = empty(torch, nb["C"])
    c.encrypt_uniform(pt["C"], ct_c, *sz["C"])
    assert _digest_hex(c, ct_c, nb["C"]) == cfg["C"]["cipher_digest"]
    # B encrypted while C's ciphertext is decrypted
    ct_b = pt["B"] if inplace else empty(torch, nb["B"])
    rt_c = ct_c if inplace else empty(torch, nb["C"])
    c.duplex_uniform(pt["B"], ct_b, *sz["B"], ct_c, rt_c, *sz["C"])
    assert _digest_hex(c, ct_b, nb["B"]) == cfg["B"]["cipher_digest"]
    assert _digest_hex(c, rt_c, nb["C"]) == cfg["C"]["plain_digest"]
    # C encrypted while B's ciphertext is decrypted
    ct_c2 = rt_c if inplace else empty(torch, nb["C"])
    rt_b = ct_b if inplace else empty(torch, nb["B"])
    c.duplex_uniform(rt_c, ct_c2, *sz["C"], ct_b, rt_b, *sz["B"])
    assert _digest_hex(c, ct_c2, nb["C"]) == cfg["C"]["cipher_digest"]
    assert _digest_hex(c, rt_b, nb["B"]) == cfg["B"]["plain_digest"]
    assert c.check() == ca.CYAES_OK
    c.close()
    torch.cuda.empty_cache()


@pytest.mark.parametrize("shape", ["runs", "big", "small_enc", "small_dec", "overlap", "empty_enc", "empty_dec",
                                   "off"])
def test_duplex_shapes_match_separate_launches(torch, shape):
    """The duplex launch against the two ordinary launches (another context per
    key row), over the shapes that take the duplex grid (encrypt runs; BIG
    decrypt payloads; different key rows per half) and the ones that fall back
    to two launches: a half too small to fill the GPU, overlapping batches (the
    decrypt reads what the encrypt writes: encrypt-then-decrypt order), an empty
    half, CYAES_DUPLEX=0."""
    keys = [K0, oracle.session_key(1), oracle.session_key(2)]
    env = {"CYAES_DUPLEX": "0"} if shape == "off" else {}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        c = ca.GpuContext(0)
    finally:
        _restore(old)
    c.set_keys(b"".join(keys))
    ref = [ca.GpuContext(0) for _ in keys]
    for r, k in zip(ref, keys):
        r.set_keys(k)
    en, epb, dn, dpb = {"runs": (1 << 20, 1472, 300000, 1024), "big": (262144, 4096, 20000, 65536),
                        "small_enc": (5000, 1472, 400000, 1472), "small_dec": (262144, 2048, 100, 1472),
                        "overlap": (262144, 2048, 262144, 2048), "empty_enc": (0, 1472, 300000, 1472),
                        "empty_dec": (262144, 2048, 0, 1472), "off": (262144, 2048, 300000, 1472)}[shape]
    ek, dk = (1, 2) if shape in ("big", "runs") else (0, 0)
    e_in, e_out = empty(torch, en * epb), empty(torch, en * epb)
    d_in, d_out = empty(torch, dn * dpb), empty(torch, dn * dpb)
    if en:
        c.fill_synthetic(e_in, 7, en, epb, oracle.PLAINTEXT_SEED)
    if dn:
        c.fill_synthetic(d_in, 11, dn, dpb, oracle.PLAINTEXT_SEED)  # decrypted as it is: any bytes are a ciphertext
    if shape == "overlap":  # the decrypt reads the encrypt's output
        c.duplex_uniform(e_in, e_out, en, epb, e_out, d_out, dn, dpb)
        assert torch.equal(d_out, e_in)  # encrypt, then decrypt of its output
        want_e = empty(torch, en * epb)
        ref[0].encrypt_uniform(e_in, want_e, en, epb)
        assert torch.equal(e_out, want_e)
    else:
        c.duplex_uniform(e_in, e_out, en, epb, d_in, d_out, dn, dpb, enc_key=ek, dec_key=dk)
        if en:
            want_e = empty(torch, en * epb)
            ref[ek].encrypt_uniform(e_in, want_e, en, epb)
            assert torch.equal(e_out, want_e)
        if dn:
            want_d = empty(torch, dn * dpb)
            ref[dk].decrypt_uniform(d_in, want_d, dn, dpb)
            assert torch.equal(d_out, want_d)
    # spot checks against the oracle
    torch.cuda.synchronize()
    if en:
        p = en // 3
        want = oracle.batch(False, [keys[ek]], 0, oracle.synthetic(7 + p, 1, epb), epb)
        assert np.array_equal(e_out[p * epb:(p + 1) * epb].cpu().numpy(), want)
    assert c.check() == ca.CYAES_OK
    with pytest.raises(ca.CyaesError):  # key row out of range
        c.duplex_uniform(e_in, e_out, max(en, 1), epb, d_in, d_out, dn, dpb, enc_key=3)
    with pytest.raises(ca.CyaesError):  # size % 16
        c.duplex_uniform(e_in, e_out, max(en, 1), epb + 4, d_in, d_out, dn, dpb)
    for r in ref:
        r.close()
    c.close()
    torch.cuda.empty_cache()
