"""Batching adapter (include/cyaes_batch.h) and
device-resident relay streams (include/cyaes_relay.h, row 2) on the MI355X,
checked against the AES oracle and the relay restatement
(oracle/relay_oracle.py).  Each request must equal the reference's
synchronous Rijndael call with iv = nullptr (relay_local.cpp:206,365;
relay_server.cpp:329,472)."""
import os
import random
import struct
import threading

import pytest

import cyclone_amd as ca
import oracle
import relay_oracle as ro

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def batcher():
    b = ca.Batcher(0, max_batch_bytes=4 << 20, max_delay_us=200)
    yield b
    b.close()


def _keys(n, seed):
    rng = random.Random(seed)
    return [bytes(rng.randrange(256) for _ in range(16)) for _ in range(n)]


def test_mixed_requests_from_threads_match_oracle(batcher):
    keys = _keys(6, 1)
    slots = [batcher.session_open(k) for k in keys]
    results = []
    lock = threading.Lock()

    def worker(tid):
        rng = random.Random(100 + tid)
        for i in range(150):
            op = rng.choice([ca.OP_ENCRYPT, ca.OP_DECRYPT])
            k = rng.randrange(len(keys))
            size = 16 * rng.choice([0, 1, 2, 63, 64, 92, 255, 256, 1000, rng.randrange(0, 4081)])
            data = bytes(rng.randrange(256) for _ in range(size))
            inplace = rng.random() < 0.3
            out = bytearray(data) if inplace else bytearray(size)
            inp = out if inplace else data
            rec = {"op": op, "k": k, "data": data, "out": out, "status": None}

            def done(status, rec=rec):
                rec["status"] = status
            batcher.submit(op, slots[k], inp, out, size, done)
            with lock:
                results.append(rec)

    threads = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    assert batcher.flush() == ca.CYAES_OK
    assert len(results) == 600
    for r in results:
        assert r["status"] == ca.CYAES_OK
        aes = oracle.Rijndael(keys[r["k"]])
        want = (aes.decrypt if r["op"] == ca.OP_DECRYPT else aes.encrypt)(bytearray(r["data"]))
        assert bytes(r["out"]) == bytes(want)
    st = batcher.stats()
    assert st["pending"] == 0 and st["errors"] == 0 and st["batches"] >= 1
    for s in slots:
        batcher.session_close(s)


def test_session_churn_while_submitting(batcher):
    """Submitters read a per-thread snapshot of the session table, refreshed
    when an open or close bumps its version.  Each worker keeps reopening its
    own session with a new key while the others do the same, and submits in
    between: every request must use the key its slot held when it was
    submitted, and a submit to a closed slot must fail with CYAES_ERANGE."""
    results = []
    lock = threading.Lock()
    errors = []

    def worker(tid):
        rng = random.Random(500 + tid)
        try:
            for rnd in range(12):
                key = bytes(rng.randrange(256) for _ in range(16))
                slot = batcher.session_open(key)
                for _ in range(rng.randrange(1, 12)):
                    size = 16 * rng.choice([1, 7, 92, 300])
                    data = bytes(rng.randrange(256) for _ in range(size))
                    out = bytearray(size)
                    rec = {"key": key, "data": data, "out": out, "status": None}

                    def done(status, rec=rec):
                        rec["status"] = status
                    batcher.submit(ca.OP_ENCRYPT, slot, data, out, size, done)
                    with lock:
                        results.append(rec)
                batcher.session_close(slot)
                try:  # the slot is closed now (another thread may reopen it: then it is theirs)
                    batcher.submit(ca.OP_ENCRYPT, slot, b"\0" * 16, bytearray(16), 16, None)
                except ca.CyaesError as e:
                    assert e.status == ca.CYAES_ERANGE
        except Exception as e:  # noqa: BLE001 -- reported below
            errors.append(repr(e))

    threads = [threading.Thread(target=worker, args=(t,)) for t in range(6)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    assert not errors, errors[:3]
    assert batcher.flush() == ca.CYAES_OK
    for r in results:
        assert r["status"] == ca.CYAES_OK
        assert bytes(r["out"]) == bytes(oracle.Rijndael(r["key"]).encrypt(bytearray(r["data"])))


def test_relay_seal_open_round_trip(batcher):
    """SEAL = relay_local.cpp:189-206 (packet + 0xCE pad + encrypt); OPEN =
    relay_server.cpp:329 (decrypt in place)."""
    key = _keys(1, 2)[0]
    slot = batcher.session_open(key)
    rng = random.Random(3)
    sizes = [0, 1, 15, 16, 17, 1472, 4095, 0xFF00] + [rng.randrange(1, 0xFF01) for _ in range(40)]
    sealed = []
    for i, n in enumerate(sizes):
        chunk = bytes(rng.randrange(256) for _ in range(n))
        pkt = bytearray(ca.relay_packet_bytes(n))
        batcher.submit_seal(slot, 1000 + i, chunk, pkt)
        sealed.append((chunk, pkt))
    assert batcher.flush() == ca.CYAES_OK
    for i, (chunk, pkt) in enumerate(sealed):
        assert bytes(pkt) == ro.seal_forward(key, 1000 + i, chunk)
    # the receive side: a stream of sealed packets, parsed and opened in place
    stream = b"".join(bytes(p) for _, p in sealed)
    parsed, used = ca.relay_parse(stream)
    assert used == len(stream) and len(parsed) == len(sizes)
    opened = [bytearray(stream[o:o + 4 + s]) for o, s, _ in parsed]
    for p in opened:
        batcher.submit_open(slot, p)
    assert batcher.flush() == ca.CYAES_OK
    for (chunk, spkt), p in zip(sealed, opened):
        conn, payload, whole = ro.open_forward(key, bytes(spkt))
        assert bytes(p) == whole and payload == chunk
        size = struct.unpack("<i", bytes(p[8:12]))[0]
        assert bytes(p[12:12 + size]) == chunk
    batcher.session_close(slot)


def test_session_reopen_and_errors(batcher):
    k1, k2 = _keys(2, 4)
    s = batcher.session_open(k1)
    data = bytes(range(256)) * 4
    out1 = bytearray(len(data))
    batcher.submit(ca.OP_ENCRYPT, s, data, out1)
    batcher.session_close(s)  # the submitted request keeps k1
    s2 = batcher.session_open(k2)
    assert s2 == s  # lowest free slot is reused
    out2 = bytearray(len(data))
    batcher.submit(ca.OP_ENCRYPT, s2, data, out2)
    assert batcher.flush() == ca.CYAES_OK
    assert bytes(out1) == bytes(oracle.Rijndael(k1).encrypt(bytearray(data)))
    assert bytes(out2) == bytes(oracle.Rijndael(k2).encrypt(bytearray(data)))
    with pytest.raises(ca.CyaesError) as e:
        batcher.submit(ca.OP_ENCRYPT, s2, data, bytearray(len(data)), 17)
    assert e.value.status == ca.CYAES_EINVAL
    with pytest.raises(ca.CyaesError) as e:
        batcher.submit(ca.OP_ENCRYPT, 999, data, bytearray(len(data)))
    assert e.value.status == ca.CYAES_ERANGE
    with pytest.raises(ca.CyaesError) as e:  # larger than a batch
        big = bytes(8 << 20)
        batcher.submit(ca.OP_ENCRYPT, s2, big, bytearray(len(big)))
    assert e.value.status == ca.CYAES_EINVAL
    bad = bytearray(ca.relay_build_forward(1, b"x" * 20))
    bad[1] ^= 1  # packet_size no longer matches the buffer
    with pytest.raises(ca.CyaesError):
        batcher.submit_open(s2, bad)
    batcher.session_close(s2)


def test_large_requests_fill_several_batches():
    b = ca.Batcher(0, max_batch_bytes=1 << 20, max_delay_us=50, inflight=2)
    try:
        key = _keys(1, 9)[0]
        s = b.session_open(key)
        rng = random.Random(9)
        reqs = []
        for i in range(24):
            n = 16 * rng.randrange(1, 65536 // 16 * 8)  # up to 512 KiB
            data = bytes(rng.getrandbits(8) for _ in range(n)) if i < 2 else bytes([i]) * n
            out = bytearray(n)
            b.submit(ca.OP_DECRYPT if i % 2 else ca.OP_ENCRYPT, s, data, out)
            reqs.append((i, data, out))
        assert b.flush() == ca.CYAES_OK
        aes = oracle.Rijndael(key)
        for i, data, out in reqs:
            want = (aes.decrypt if i % 2 else aes.encrypt)(bytearray(data))
            assert bytes(out) == bytes(want)
        total = sum(len(d) for _, d, _ in reqs)
        assert b.stats()["batches"] >= total // (1 << 20)  # no batch carries more than max_batch_bytes
    finally:
        b.close()


def test_flush_waits_for_own_requests_under_load():
    """flush() returns only after every request submitted before it completed,
    while other threads keep submitting into small batches (a global
    completion count could be reached by later requests of other shards)."""
    b = ca.Batcher(0, max_batch_bytes=64 << 10, max_delay_us=20, inflight=3)
    try:
        key = _keys(1, 11)[0]
        s = b.session_open(key)
        stop = threading.Event()

        def noise(t):
            # a relay-style window: at most 32 requests of this thread in flight
            rng = random.Random(t)
            window = threading.Semaphore(32)
            while not stop.is_set():
                if not window.acquire(timeout=0.5):
                    continue
                n = 16 * rng.randrange(1, 1024)
                b.submit(ca.OP_ENCRYPT, s, bytes(n), bytearray(n), None, lambda st, w=window: w.release())

        th = [threading.Thread(target=noise, args=(t,)) for t in range(6)]
        for t in th:
            t.start()
        try:
            for rnd in range(20):
                done = []
                for i in range(40):
                    n = 16 * (1 + (i * 37 + rnd) % 2000)
                    b.submit(ca.OP_DECRYPT, s, bytes(n), bytearray(n), None, lambda st, i=i: done.append(i))
                assert b.flush() == ca.CYAES_OK
                assert sorted(done) == list(range(40)), (rnd, len(done))
        finally:
            stop.set()
            for t in th:
                t.join()
        assert b.flush() == ca.CYAES_OK and b.stats()["pending"] == 0
    finally:
        b.close()


def test_submit_many_rejects_oversized_requests(batcher):
    s = batcher.session_open(_keys(1, 12)[0])
    with pytest.raises(ValueError):
        batcher.submit_many([(ca.OP_ENCRYPT, s, bytes(32), bytearray(16), 32, None, 0)])
    with pytest.raises(ValueError):
        batcher.submit_many([(ca.OP_DECRYPT, s, bytes(16), bytearray(64), 64, None, 0)])
    with pytest.raises(ValueError):
        batcher.submit_many([(ca.OP_RELAY_SEAL, s, bytes(100), bytearray(64), None, None, 1)])
    batcher.session_close(s)


def test_device_relay_stream_in_place():
    """A connection's byte stream of relay packets, resident in HBM: the
    payloads (packet offset 12, 4-byte aligned) are encrypted and decrypted
    where they lie by the ragged kernels."""
    import torch
    key = _keys(1, 11)[0]
    rng = random.Random(11)
    chunks = [bytes(rng.randrange(256) for _ in range(rng.choice([1, 16, 100, 1472, 0xFF00, rng.randrange(1, 9000)])))
              for _ in range(300)]
    plain = b"".join(ro.seal_forward(None, i, c, encrypt=False) for i, c in enumerate(chunks))
    sealed = b"".join(ro.seal_forward(key, i, c) for i, c in enumerate(chunks))
    parsed, used = ca.relay_parse(plain)
    assert used == len(plain)
    off, ln = ca.relay_payloads(parsed)
    assert any(o % 16 for o in off)  # genuinely misaligned payloads
    ctx = ca.GpuContext(0)
    ctx.set_keys(key)
    dev = torch.frombuffer(bytearray(plain), dtype=torch.uint8).cuda()
    d_off = torch.tensor(off, dtype=torch.int64).cuda()
    d_len = torch.tensor(ln, dtype=torch.int32).cuda()
    ctx.encrypt_ragged(dev, dev, d_off, d_len, len(off))
    assert ctx.check() == ca.CYAES_OK
    assert bytes(dev.cpu().numpy().tobytes()) == sealed
    ctx.decrypt_ragged(dev, dev, d_off, d_len, len(off))
    assert bytes(dev.cpu().numpy().tobytes()) == plain
    # the SURVEY §8(b) batch entry points (per-payload input IV, key index)
    lib = ca.load_library()
    ivs = torch.frombuffer(bytearray(bytes(range(16)) * len(off)), dtype=torch.uint8).cuda()
    kid = torch.zeros(len(off), dtype=torch.int32).cuda()
    out = torch.empty_like(dev)
    assert lib.cyaes_gpu_cbc_encrypt_batch(ctx._h, dev.data_ptr(), out.data_ptr(), d_off.data_ptr(),
                                           d_len.data_ptr(), kid.data_ptr(), ivs.data_ptr(), len(off), None) == 0
    torch.cuda.synchronize()
    got = out.cpu().numpy().tobytes()
    for o, n in zip(off, ln):
        assert got[o:o + n] == sealed[o:o + n]
    ctx.close()


def test_update_keys_partial():
    import torch
    ctx = ca.GpuContext(0)
    keys = _keys(5, 12)
    ctx.set_keys(b"".join(keys[:3]))
    new = _keys(3, 13)
    lib = ca.load_library()
    buf = (ca.ctypes.c_uint8 * 48).from_buffer_copy(b"".join(new))
    assert lib.cyaes_gpu_update_keys(ctx._h, 2, buf, 3) == 0  # replaces row 2, appends 3..4
    assert ctx.nkeys == 5
    table = [keys[0], keys[1], new[0], new[1], new[2]]
    for i, k in enumerate(table):
        assert ctx.get_key(i).words() == oracle.key_expand(k).words()
    assert lib.cyaes_gpu_update_keys(ctx._h, 6, buf, 1) == ca.CYAES_EINVAL  # first > nkeys
    data = torch.arange(5 * 256, dtype=torch.int32).to(torch.uint8).cuda()
    out = torch.empty_like(data)
    ctx.encrypt_uniform(data, out, 5, 256, payloads_per_key=1)
    torch.cuda.synchronize()
    got = out.cpu().numpy().tobytes()
    src = data.cpu().numpy().tobytes()
    for p, k in enumerate(table):
        assert got[256 * p:256 * (p + 1)] == bytes(oracle.Rijndael(k).encrypt(bytearray(src[256 * p:256 * (p + 1)])))
    ctx.close()


def test_submit_many_mixed_ops_order_and_errors(batcher):
    """cyaes_batcher_submit_many: ENCRYPT / DECRYPT / RELAY_SEAL / RELAY_OPEN in
    one call from several threads; invalid entries are rejected individually
    (status, no callback); each thread's requests complete in submission order."""
    keys = _keys(3, 7)
    slots = [batcher.session_open(k) for k in keys]
    checks, lock = [], threading.Lock()

    def worker(tid):
        rng = random.Random(500 + tid)
        order = []
        for rnd in range(20):
            reqs, recs = [], []
            for i in range(rng.randrange(1, 40)):
                k = rng.randrange(len(keys))
                kind = rng.randrange(5)
                rec = {"k": k, "kind": kind, "status": None, "seq": (rnd, i)}

                def done(status, rec=rec):
                    rec["status"] = status
                    order.append(rec["seq"])
                if kind <= 1:  # ENCRYPT / DECRYPT
                    data = bytes(rng.randrange(256) for _ in range(16 * rng.randrange(0, 100)))
                    rec.update(data=data, out=bytearray(len(data)))
                    reqs.append((kind, slots[k], data, rec["out"], None, done, 0))
                elif kind == 2:  # SEAL
                    chunk = bytes(rng.randrange(256) for _ in range(rng.randrange(0, 3000)))
                    rec.update(chunk=chunk, conn=tid * 1000 + i, out=bytearray(ca.relay_packet_bytes(len(chunk))))
                    reqs.append((ca.OP_RELAY_SEAL, slots[k], chunk, rec["out"], len(chunk), done, rec["conn"]))
                elif kind == 3:  # OPEN
                    chunk = bytes(rng.randrange(256) for _ in range(rng.randrange(0, 3000)))
                    sealed = ro.seal_forward(keys[k], 77, chunk)
                    rec.update(chunk=chunk, sealed=sealed, out=bytearray(sealed))
                    reqs.append((ca.OP_RELAY_OPEN, slots[k], None, rec["out"], len(sealed), done, 0))
                else:  # invalid: size not a multiple of 16
                    rec.update(out=bytearray(20))
                    reqs.append((ca.OP_ENCRYPT, slots[k], bytes(20), rec["out"], 20, done, 0))
                recs.append(rec)
            st = batcher.submit_many(reqs)
            for rec, s in zip(recs, st):
                rec["submit"] = s
            with lock:
                checks.extend(recs)
        with lock:
            checks.append({"order": order})

    threads = [threading.Thread(target=worker, args=(t,)) for t in range(3)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    assert batcher.flush() == ca.CYAES_OK
    for rec in checks:
        if "order" in rec:
            assert rec["order"] == sorted(rec["order"])  # per-thread FIFO
            continue
        if rec["kind"] == 4:
            assert rec["submit"] == ca.CYAES_EINVAL and rec["status"] is None
            continue
        assert rec["submit"] == ca.CYAES_OK and rec["status"] == ca.CYAES_OK
        aes = oracle.Rijndael(keys[rec["k"]])
        if rec["kind"] == 0:
            assert bytes(rec["out"]) == bytes(aes.encrypt(bytearray(rec["data"])))
        elif rec["kind"] == 1:
            assert bytes(rec["out"]) == bytes(aes.decrypt(bytearray(rec["data"])))
        elif rec["kind"] == 2:
            assert bytes(rec["out"]) == ro.seal_forward(keys[rec["k"]], rec["conn"], rec["chunk"])
        else:
            assert bytes(rec["out"]) == ro.open_forward(keys[rec["k"]], rec["sealed"])[2]
    for s in slots:
        batcher.session_close(s)


def test_device_relay_stream_config_b_default_kernels():
    """Config B's 1 M payloads as a relay packet stream in HBM (payload at packet
    offset 12, packet stride 1,484 B: 4-B aligned, relay_protocol.h:5-42), encrypted
    and decrypted in place with the runtime's default kernel choice -- one lane per
    chain from 131,072 ragged chains up (cyaes_internal.h kQuadRaggedFactor).  The
    gathered ciphertext's digest equals config B's committed OpenSSL digest
    (tests/golden/openssl_vectors.json), the packet headers stay untouched, and
    decrypt restores the plaintext."""
    import json
    import os
    import torch
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "openssl_vectors.json")))["configs"]["B"]
    n, pb, hdr, stride = g["npayloads"], g["payload_bytes"], 12, g["payload_bytes"] + 12
    ctx = ca.GpuContext(0)
    ctx.set_keys(bytes(range(16)))
    pt = torch.empty(n * pb, dtype=torch.uint8, device="cuda")
    ctx.fill_synthetic(pt, 0, n, pb, 0x5EEDC1C1)
    assert ["%016x" % v for v in ctx.digest(pt, n * pb)] == g["plain_digest"]
    buf = torch.full((n * stride + 16,), 0xA5, dtype=torch.uint8, device="cuda")
    view = buf[: n * stride].view(n, stride)
    view[:, hdr:hdr + pb] = pt.view(n, pb)
    off = (torch.arange(n, dtype=torch.int64, device="cuda") * stride + hdr).contiguous()
    nb = torch.full((n,), pb, dtype=torch.int32, device="cuda")
    ctx.encrypt_ragged(buf, buf, off, nb, n)
    assert ctx.check() == ca.CYAES_OK
    ct = view[:, hdr:hdr + pb].contiguous()
    assert ["%016x" % v for v in ctx.digest(ct, n * pb)] == g["cipher_digest"]
    assert bool((view[:, :hdr] == 0xA5).all()) and bool((buf[n * stride:] == 0xA5).all())
    ctx.decrypt_ragged(buf, buf, off, nb, n)
    assert ctx.check() == ca.CYAES_OK
    assert torch.equal(view[:, hdr:hdr + pb].reshape(-1), pt)
    ctx.close()


# ---- zero-copy packet pools (round 3) ---------------------------------------
def test_pooled_requests_zero_copy_match_oracle(batcher):
    """Requests whose buffers lie in a registered pool are gathered from and
    scattered to it by the GPU (cyaes_batch_kernels.hip): by pointer (found
    in the pool automatically) and by pool offset (submit_pooled).  ENCRYPT,
    DECRYPT, SEAL (relay_local.cpp:189-206) and OPEN (relay_server.cpp:329) at
    16-, 4- and 1-byte aligned addresses, in place and not, against the AES
    oracle and the relay restatement."""
    import numpy as np
    key = _keys(1, 21)[0]
    slot = batcher.session_open(key)
    aes = oracle.Rijndael(key)
    rng = random.Random(21)
    pool = np.zeros(8 << 20, dtype=np.uint8)
    pid = batcher.register_pool(pool)
    mv = memoryview(pool)
    pos = [64]

    def carve(n, align):
        o = (pos[0] + 63) // 64 * 64 + align
        pos[0] = o + n + 64
        return o
    checks, reqs = [], []
    for i in range(160):
        op = [ca.OP_ENCRYPT, ca.OP_DECRYPT, ca.OP_RELAY_SEAL, ca.OP_RELAY_OPEN][i % 4]
        align = [0, 4, 12, 1][(i // 4) % 4]
        if op in (ca.OP_ENCRYPT, ca.OP_DECRYPT):
            n = 16 * rng.choice([0, 1, 5, 92, 300, 4080])
            src = bytes(rng.getrandbits(8) for _ in range(n))
            io = carve(n, align)
            pool[io:io + n] = np.frombuffer(src, np.uint8)
            inplace = i % 3 == 0
            oo = io if inplace else carve(n, (align * 7) % 16)
            want = (aes.decrypt if op == ca.OP_DECRYPT else aes.encrypt)(bytearray(src))
            checks.append((oo, bytes(want)))
            reqs.append((op, io, oo, n))
        elif op == ca.OP_RELAY_SEAL:
            n = rng.choice([0, 1, 17, 1472, 4000, 0xFF00])
            chunk = bytes(rng.getrandbits(8) for _ in range(n))
            io = carve(n, align)
            pool[io:io + n] = np.frombuffer(chunk, np.uint8)
            oo = carve(ca.relay_packet_bytes(n), (align + 4) % 16)
            checks.append((oo, ro.seal_forward(key, 3000 + i, chunk)))
            reqs.append((op, io, oo, n))
        else:
            n = rng.choice([16, 1472, 9000])
            chunk = bytes(rng.getrandbits(8) for _ in range(n))
            pkt = ro.seal_forward(key, 7, chunk)
            io = carve(len(pkt), align)
            pool[io:io + len(pkt)] = np.frombuffer(pkt, np.uint8)
            checks.append((io, ro.open_forward(key, pkt)[2]))
            reqs.append((op, io, None, len(pkt)))
    status = []
    half = len(reqs) // 2
    for k, (op, io, oo, n) in enumerate(reqs[:half]):  # by pointer: found inside the pool
        if op == ca.OP_RELAY_OPEN:
            batcher.submit_open(slot, mv[io:io + n])
        elif op == ca.OP_RELAY_SEAL:
            batcher.submit_seal(slot, 3000 + k, mv[io:io + n], mv[oo:oo + ca.relay_packet_bytes(n)])
        else:
            batcher.submit(op, slot, mv[io:io + n], mv[oo:oo + n], n)
    pooled = [(op, slot, pid, io, oo or 0, n, None, 3000 + half + k)
              for k, (op, io, oo, n) in enumerate(reqs[half:])]
    status = batcher.submit_pooled(pooled)
    assert status == [0] * len(pooled)
    assert batcher.flush() == ca.CYAES_OK
    for k, (off, want) in enumerate(checks):
        assert bytes(pool[off:off + len(want)]) == want, k
    # a pooled request that runs past its pool's end is rejected
    bad = batcher.submit_pooled([(ca.OP_ENCRYPT, slot, pid, pool.size - 16, 0, 32, None, 0)])
    assert bad == [ca.CYAES_EINVAL]
    batcher.unregister_pool(pid)
    with pytest.raises(ca.CyaesError):
        batcher.unregister_pool(pid)
    batcher.session_close(slot)


def test_pool_session_rows_survive_close_and_reopen(batcher):
    """A closed slot's key row is not reused while requests submitted before
    the close are still queued: pooled requests keep the key they were
    submitted under across close/reopen churn (cyaes_batch.h, sessions)."""
    import numpy as np
    pool = np.zeros(4 << 20, dtype=np.uint8)
    pid = batcher.register_pool(pool)
    rng = random.Random(33)
    want = []
    off = 0
    for rnd in range(40):
        key = bytes(rng.getrandbits(8) for _ in range(16))
        slot = batcher.session_open(key)
        reqs = []
        for _ in range(rng.randrange(1, 8)):
            n = 16 * rng.choice([1, 92, 300])
            data = bytes(rng.getrandbits(8) for _ in range(n))
            pool[off:off + n] = np.frombuffer(data, np.uint8)
            reqs.append((ca.OP_ENCRYPT, slot, pid, off, off + n, n, None, 0))
            want.append((off + n, bytes(oracle.Rijndael(key).encrypt(bytearray(data)))))
            off += 2 * n
        assert batcher.submit_pooled(reqs) == [0] * len(reqs)
        batcher.session_close(slot)
    assert batcher.flush() == ca.CYAES_OK
    for o, w in want:
        assert bytes(pool[o:o + len(w)]) == w
    batcher.unregister_pool(pid)


def _bench_batcher_dump(tmp_path, op, extra=()):
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "build", "bench_batcher")
    if not os.path.exists(exe):
        subprocess.run(["make", "-C", root, "-s", "build/bench_batcher"], check=True)
    dump = str(tmp_path / ("dump_%s.bin" % op))
    cmd = [exe, "--op", op, "--threads", "3", "--window", "64", "--seconds", "0.3", "--dump", dump] + list(extra)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    import json
    return json.loads(line), open(dump, "rb").read()


@pytest.mark.parametrize("op,extra", [("seal", ()), ("open", ()), ("seal", ("--submit", "pooled")),
                                      ("open", ("--pool", "0"))])
def test_bench_batcher_output_matches_relay_oracle(tmp_path, op, extra):
    """tools/bench_batcher's own packets (its --dump verification round: every
    slot of every looper sealed or opened once through the zero-copy pool
    path, or the bounce path with --pool 0) against the relay restatement."""
    res, blob = _bench_batcher_dump(tmp_path, op, extra)
    assert res["errors"] == 0 and res["requests_per_s"] > 0
    opc, size, in_n, out_n = struct.unpack_from("<4I", blob, 0)
    pos, nchecked = 16, 0
    while pos < len(blob):
        key = blob[pos:pos + 16]
        nslots = struct.unpack_from("<I", blob, pos + 16)[0]
        pos += 20
        for _ in range(nslots):
            inp, out = blob[pos:pos + in_n], blob[pos + in_n:pos + in_n + out_n]
            pos += in_n + out_n
            if opc == ca.OP_RELAY_SEAL:
                assert out == ro.seal_forward(key, 7, inp)
            else:
                assert out == ro.open_forward(key, inp)[2]
            nchecked += 1
    assert nchecked == 3 * 64


def test_poll_mode_completions_in_submission_order():
    """CYAES_BATCHER_POLL: requests complete into the submitting thread's queue
    (cyaes_batcher_poll) in its submission order, instead of one callback per
    packet; SEAL and OPEN on pool memory against the relay restatement."""
    import numpy as np
    b = ca.Batcher(0, max_batch_bytes=1 << 20, max_delay_us=100, poll=True)
    try:
        key = _keys(1, 41)[0]
        slot = b.session_open(key)
        rng = random.Random(41)
        pool = np.zeros(16 << 20, dtype=np.uint8)
        pid = b.register_pool(pool)
        reqs, want, off = [], [], 0
        for i in range(3000):
            n = rng.choice([0, 16, 100, 1472, 5000])
            chunk = bytes(rng.getrandbits(8) for _ in range(n))
            pool[off:off + n] = np.frombuffer(chunk, np.uint8)
            out = off + ((n + 63) // 64) * 64
            reqs.append((ca.OP_RELAY_SEAL, slot, pid, off, out, n, i, 9))
            want.append((out, ro.seal_forward(key, 9, chunk)))
            off = out + ((ca.relay_packet_bytes(n) + 63) // 64) * 64
        assert b.submit_pooled(reqs) == [0] * len(reqs)
        got = []
        import time
        t_end = time.time() + 60
        while len(got) < len(reqs) and time.time() < t_end:
            got += b.poll()
            if len(got) < len(reqs):
                time.sleep(0.001)
        assert [t for t, _ in got] == list(range(len(reqs)))  # submission order
        assert all(st == ca.CYAES_OK for _, st in got)
        for o, w in want:
            assert bytes(pool[o:o + len(w)]) == w
        # OPEN the sealed packets in place, polled again
        opens = [(ca.OP_RELAY_OPEN, slot, pid, o, 0, len(w), ("open", k), 0) for k, (o, w) in enumerate(want)]
        assert b.submit_pooled(opens) == [0] * len(opens)
        assert b.flush() == ca.CYAES_OK  # (flush covers poll-mode requests too)
        got = b.poll()
        assert [t for t, _ in got] == [("open", k) for k in range(len(want))]
        for o, w in want:
            assert bytes(pool[o:o + len(w)]) == ro.open_forward(key, w)[2]
        assert b.poll() == []
        b.unregister_pool(pid)
    finally:
        b.close()


def test_slow_callbacks_keep_order_and_flush_semantics():
    """The completion thread hands a stage back to the builder before running
    its callbacks (r03).  With slow callbacks over many small batches, each
    submitting thread still sees its callbacks in submission order, outputs are
    the oracle's, and flush() returns only after every earlier callback has
    returned."""
    import time
    b = ca.Batcher(0, max_batch_bytes=32 << 10, max_delay_us=20, inflight=3)
    try:
        key = _keys(1, 57)[0]
        s = b.session_open(key)
        aes = oracle.Rijndael(key)
        nthreads, per = 4, 400
        seen = {t: [] for t in range(nthreads)}
        outs = {}
        errs = []

        def worker(t):
            rng = random.Random(500 + t)
            for i in range(per):
                n = 16 * rng.randrange(1, 200)
                data = bytes(rng.getrandbits(8) for _ in range(n))
                out = bytearray(n)
                outs[(t, i)] = (data, out)

                def done(st, t=t, i=i):
                    if st:
                        errs.append(st)
                    if i % 97 == 0:
                        time.sleep(0.003)  # a slow callback holds up the completion side
                    seen[t].append(i)

                b.submit(ca.OP_ENCRYPT, s, data, out, None, done)

        th = [threading.Thread(target=worker, args=(t,)) for t in range(nthreads)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert b.flush() == ca.CYAES_OK
        # flush returned: every callback of the requests above has returned
        assert all(len(seen[t]) == per for t in range(nthreads))
        assert not errs
        for t in range(nthreads):
            assert seen[t] == list(range(per)), t  # submission order per thread
        for (t, i), (data, out) in outs.items():
            assert bytes(out) == bytes(aes.encrypt(bytearray(data)))
        assert b.stats()["batches"] > 10
    finally:
        b.close()


@pytest.mark.gpu
@pytest.mark.parametrize("size,recv_copy,depth", [("1472", 1, 2), ("1472", 0, 1), ("rand:4000", 0, 3),
                                                  ("rand:65280", 1, 2)])
def test_relay_loop_both_ends(size, recv_copy, depth):
    """tools/relay_loop: the relay's whole data path through the batcher --
    SEAL chunks into per-pipe tunnel streams (packets back to back, as TCP
    carries them; relay_local.cpp:188-217), cut the received stream into
    packets (cye_packet.cpp:166-181), OPEN each in place (relay_server.cpp:329)
    -- and every forwarded payload, RelayForwardMsg field and 0xCE pad byte
    matches the client's chunk; the wire holds ciphertext.  depth: rounds in
    flight per looper (1: seal, parse, open in sequence)."""
    import json
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "build", "relay_loop")
    if not os.path.exists(exe):
        subprocess.run(["make", "-C", root, "-s", "build/relay_loop"], check=True)
    cmd = [exe, "--threads", "3", "--pipes", "4", "--chunks", "8" if size == "rand:65280" else "32",
           "--size", size, "--recv-copy", str(recv_copy), "--seconds", "0.3", "--depth", str(depth)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["error"] == 0 and out["mismatches"] == 0
    assert out["verified"] == out["packets"] > 0 and out["rounds"] > 0 and out["depth"] == depth


def test_pools_sharing_a_page(batcher):
    """Two pools on one page, the second spanning several pages (two buffers of
    one heap): the shared page stays pinned while either pool
    lives, so the second pool keeps working after the first is unregistered,
    on its shared page and on the pages past it."""
    import numpy as np
    key = _keys(1, 41)[0]
    slot = batcher.session_open(key)
    aes = oracle.Rijndael(key)
    rng = random.Random(41)
    buf = np.zeros(8 * 4096, dtype=np.uint8)
    p0 = (-buf.ctypes.data) % 4096  # first page boundary inside buf
    a_lo, a_n = p0 + 96, 1024                # pool A: inside page 0
    b_lo, b_n = p0 + 2048, 3 * 4096 + 512    # pool B: from page 0 into page 3
    pa = batcher.register_pool(buf[a_lo:a_lo + a_n])
    pb = batcher.register_pool(buf[b_lo:b_lo + b_n])

    def run(pool, base, spans):
        want = []
        reqs = []
        for off, n in spans:
            data = bytes(rng.getrandbits(8) for _ in range(n))
            buf[base + off:base + off + n] = np.frombuffer(data, np.uint8)
            reqs.append((ca.OP_ENCRYPT, slot, pool, off, off, n, None, 0))
            want.append((base + off, bytes(aes.encrypt(bytearray(data)))))
        assert batcher.submit_pooled(reqs) == [0] * len(reqs)
        assert batcher.flush() == ca.CYAES_OK
        for o, w in want:
            assert bytes(buf[o:o + len(w)]) == w
    run(pa, a_lo, [(0, 512), (512, 512)])
    run(pb, b_lo, [(0, 1024), (4096, 4096), (b_n - 512, 512)])
    batcher.unregister_pool(pa)
    # B's first page is the one A shared; its last bytes are three pages on
    run(pb, b_lo, [(0, 1008), (b_n - 1024, 1024), (1024, 8192)])
    # a new pool on the freed part of the shared page shares it again
    pc = batcher.register_pool(buf[p0:p0 + 2048])
    run(pc, p0, [(0, 2048)])
    batcher.unregister_pool(pb)
    run(pc, p0, [(16, 1024)])
    batcher.unregister_pool(pc)
    batcher.session_close(slot)


def test_pool_in_foreign_registration(batcher):
    """Memory someone else pinned is used as it is only when that one
    registration holds the whole pool: a pool inside it works, one starting in
    it and reaching past it is refused (CYAES_EINVAL) instead of handing the
    GPU unmapped pages, and one that starts on unpinned pages and
    runs into it is refused as well."""
    import numpy as np
    import hiprt
    key = _keys(1, 43)[0]
    slot = batcher.session_open(key)
    buf = np.zeros(8 * 4096, dtype=np.uint8)
    p0 = (-buf.ctypes.data) % 4096
    lo = buf.ctypes.data + p0 + 4096  # pages 1..4 of buf's page-aligned part, registered by "someone else"
    assert hiprt.host_register(lo, 4 * 4096) == 0
    key_aes = oracle.Rijndael(key)

    def encrypt_in(pid, base, n, seed):
        data = bytes(random.Random(seed).getrandbits(8) for _ in range(n))
        buf[base:base + n] = np.frombuffer(data, np.uint8)
        assert batcher.submit_pooled([(ca.OP_ENCRYPT, slot, pid, 0, 0, n, None, 0)]) == [0]
        assert batcher.flush() == ca.CYAES_OK
        assert bytes(buf[base:base + n]) == bytes(key_aes.encrypt(bytearray(data)))
    try:
        # starts inside the foreign registration and runs past it: refused
        with pytest.raises(ca.CyaesError):
            batcher.register_pool(buf[p0 + 4096:p0 + 6 * 4096])
        # starts on a page nobody pinned and runs into the registration: refused too
        # (registering over part of another owner's registration corrupts its record)
        with pytest.raises(ca.CyaesError):
            batcher.register_pool(buf[p0 + 100:p0 + 3 * 4096])
        # pages nobody pinned, next to the registration: the batcher pins them itself
        pid = batcher.register_pool(buf[p0 + 5 * 4096 + 16:p0 + 7 * 4096])
        encrypt_in(pid, p0 + 5 * 4096 + 16, 4096, 42)
        batcher.unregister_pool(pid)
        # inside the foreign registration: used as it is
        pid = batcher.register_pool(buf[p0 + 4096 + 64:p0 + 5 * 4096 - 64])
        encrypt_in(pid, p0 + 4096 + 64, 4096, 43)
        batcher.unregister_pool(pid)  # leaves the foreign registration alone
    finally:
        assert hiprt.host_unregister(lo) == 0
    batcher.session_close(slot)


def test_pool_at_the_tail_of_a_foreign_allocation(batcher):
    """A pool whose last byte is the last byte of another owner's pinned
    allocation, whose size is not a page multiple (hipHostMalloc of 3 pages +
    100 B): it lies inside that registration and is used as it is, nothing
    registered (the registry tests the pool's exact bytes, not its
    page span, which reaches past the allocation).  Bit-exact."""
    import ctypes
    import numpy as np
    import hiprt
    key = _keys(1, 47)[0]
    slot = batcher.session_open(key)
    aes = oracle.Rijndael(key)
    size = 3 * 4096 + 100
    p = hiprt.host_malloc(size)
    try:
        buf = np.ctypeslib.as_array((ctypes.c_uint8 * size).from_address(p))
        tail = buf[size - 1000:]
        before = ca.debug_pins()
        pid = batcher.register_pool(tail)
        after = ca.debug_pins()
        assert after["registered"] == before["registered"] and after["conflicts"] == before["conflicts"]
        data = bytes(random.Random(47).getrandbits(8) for _ in range(992))
        tail[8:1000] = np.frombuffer(data, np.uint8)
        assert batcher.submit_pooled([(ca.OP_ENCRYPT, slot, pid, 8, 8, 992, None, 0)]) == [0]
        assert batcher.flush() == ca.CYAES_OK
        assert bytes(tail[8:1000]) == bytes(aes.encrypt(bytearray(data)))
        batcher.unregister_pool(pid)
        assert ca.debug_pins()["live"] == 0
    finally:
        hiprt.host_free(p)
    batcher.session_close(slot)


def test_pooled_open_range_and_unregister_flush(batcher):
    """A pooled OPEN whose packet would run past its pool is refused before
    its header is read, and unregister_pool, which drains the
    requests before it, leaves flush's error hand-off to flush."""
    import numpy as np
    assert batcher.flush() == ca.CYAES_OK
    key = _keys(1, 45)[0]
    slot = batcher.session_open(key)
    pool = np.zeros(1 << 16, dtype=np.uint8)
    pid = batcher.register_pool(pool)
    # an OPEN whose packet is not a RELAY_FORWARD packet is refused at submit (no batch error) ...
    assert batcher.submit_pooled([(ca.OP_RELAY_OPEN, slot, pid, 0, 0, 64, None, 0)]) == [ca.CYAES_EINVAL]
    # ... and one that would read its header past the pool's end is refused before it reads
    assert batcher.submit_pooled([(ca.OP_RELAY_OPEN, slot, pid, pool.size - 2, 0, 64, None, 0)]) == \
        [ca.CYAES_EINVAL]
    batcher.unregister_pool(pid)
    assert batcher.flush() == ca.CYAES_OK
    batcher.session_close(slot)


@pytest.mark.parametrize("chunk", [1456, 1024 - 8, 65272, 488])  # payloads of 92, 64, 4080 and 31 blocks
@pytest.mark.parametrize("mode", ["default", "dyn1", "lists"])
def test_device_relay_stream_strided(chunk, mode):
    """A received stream of equal relay packets resident in HBM (the server's
    tunnel buffer under bulk transfer): cyaes_relay_stride recognises the
    payloads as equally strided (packet offset 12, stride = packet size) and
    cyaes_gpu_{en,de}crypt_strided process them where they lie, in place and
    out of place, headers untouched -- the flat kernel's strided addressing
    for payloads of >= 64 blocks, the ragged kernels otherwise ("lists" forces
    those), bit-exact against the relay restatement (relay_local.cpp:189-206,
    relay_server.cpp:329)."""
    import numpy as np
    import torch
    env = {"default": {}, "dyn1": {"CYAES_DEC_GRID": "3", "CYAES_DEC_RANGE_STEPS": "1", "CYAES_DEC_DYN": "1"},
           "lists": {"CYAES_STRIDED_LISTS": "1"}}[mode]
    key = _keys(1, 51)[0]
    rng = random.Random(51)
    n = 700 if chunk < 60000 else 40
    chunks = [bytes(rng.randrange(256) for _ in range(chunk)) for _ in range(n)]
    plain = b"".join(ro.seal_forward(None, i, c, encrypt=False) for i, c in enumerate(chunks))
    sealed = b"".join(ro.seal_forward(key, i, c) for i, c in enumerate(chunks))
    parsed, used = ca.relay_parse(plain)
    assert used == len(plain)
    off, ln = ca.relay_payloads(parsed)
    first, stride, pb = ca.relay_stride(off, ln)
    assert (first, stride, pb) == (12, ca.relay_packet_bytes(chunk), ln[0])
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    ctx = ca.GpuContext(0)
    for k, v in old.items():
        os.environ.pop(k) if v is None else os.environ.__setitem__(k, v)
    ctx.set_keys(key)
    dev = torch.frombuffer(bytearray(plain), dtype=torch.uint8).cuda()
    ctx.encrypt_strided(dev, dev, first, stride, n, pb)
    assert bytes(dev.cpu().numpy().tobytes()) == sealed
    ctx.decrypt_strided(dev, dev, first, stride, n, pb)
    assert bytes(dev.cpu().numpy().tobytes()) == plain
    # out of place: the bytes between payloads of the output stream are left alone
    src = torch.frombuffer(bytearray(sealed), dtype=torch.uint8).cuda()
    out = torch.full_like(src, 0x5A)
    ctx.decrypt_strided(src, out, first, stride, n, pb)
    got = out.cpu().numpy().tobytes()
    want = bytearray(b"\x5a" * len(sealed))
    for o in off:
        want[o:o + pb] = plain[o:o + pb]
    assert got == bytes(want)
    assert ctx.check() == ca.CYAES_OK
    # an irregular stream is not strided
    assert ca.relay_stride(off[:-1] + [off[-1] + 4], ln) is None
    with pytest.raises(ca.CyaesError):  # stride shorter than the payload
        ctx.decrypt_strided(dev, dev, first, pb - 16, n, pb)
    ctx.close()


@pytest.mark.parametrize("pb,stride,first,inplace", [
    (1472, 1484, 12, True), (1472, 1484, 12, False),  # relay packets: 4 line phases (12 + 12 p mod 64)
    (1472, 1476, 60, True),                           # phases 60 + 4 p: all 16
    (4080, 4092, 12, False), (64, 76, 4, True),       # 255 and 4 blocks
    (16, 20, 8, False),                               # one block per payload
    (1456, 1520, 16, True), (1472, 1536, 0, True),    # 16-B phases (no dword shift), line-aligned
])
def test_strided_encrypt_by_lines(pb, stride, first, inplace):
    """Strided encrypts read by 64-B lines (k_encrypt_lines, cyaes_lines_body.h):
    whole 1,024-payload groups by lines, the rest by the ragged lane / quad
    kernels; every payload a chain from DefaultIV (relay_local.cpp:206), at
    payload phases 0-60 B in the line, in place and out of place.  Bit-exact
    against the oracle and against a context without the lines kernel
    (CYAES_ENC_LINES=0); a 3-workgroup grid walks several items per wave (each
    item's first chunk loaded during the previous one's last); the bytes around
    the payloads are untouched; the stream decrypts back (relay_server.cpp:329)."""
    import numpy as np
    import torch
    n = 2 * 1024 + 437
    key = _keys(1, 83)[0]
    rng = np.random.default_rng(83)
    plain = rng.integers(0, 256, n * pb, dtype=np.uint8)
    want = oracle.batch(False, [key], 0, plain, pb)
    size = first + (n - 1) * stride + pb + 3
    ctxs = []
    for env in ({"CYAES_QUAD_MAX_CHAINS": "1024"}, {"CYAES_QUAD_MAX_CHAINS": "1024", "CYAES_LINES_GRID": "3"},
                {"CYAES_QUAD_MAX_CHAINS": "1024", "CYAES_ENC_LINES": "0"}):
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        ctxs.append(ca.GpuContext(0))
        for k, v in old.items():
            os.environ.pop(k) if v is None else os.environ.__setitem__(k, v)
    outs = []
    for ctx in ctxs:
        ctx.set_keys(key)
        src = torch.full((size,), 0xA7, dtype=torch.uint8, device="cuda")
        view = src[first: first + n * stride - (stride - pb)].as_strided((n, pb), (stride, 1))
        view.copy_(torch.from_numpy(plain.reshape(n, pb)).cuda())
        before = src.clone()
        dst = src if inplace else torch.full_like(src, 0x3C)
        ctx.encrypt_strided(src, dst, first, stride, n, pb)
        torch.cuda.synchronize()
        got = dst[first: first + n * stride - (stride - pb)].as_strided((n, pb), (stride, 1)).cpu().numpy()
        assert np.array_equal(got.reshape(-1), want), "payloads differ from the oracle"
        mask = torch.ones(size, dtype=torch.bool, device="cuda")
        mask[first: first + n * stride - (stride - pb)].as_strided((n, pb), (stride, 1)).fill_(False)
        around = dst[mask]
        assert bool((around == (before[mask] if inplace else 0x3C)).all()), "bytes outside the payloads changed"
        if not inplace:
            assert torch.equal(src, before), "input stream changed"
        outs.append(dst.cpu())
        # and back: the ciphertext stream decrypted (in place, or into a fresh output stream)
        back = dst if inplace else torch.full_like(dst, 0x5D)
        ctx.decrypt_strided(dst, back, first, stride, n, pb)
        torch.cuda.synchronize()
        got = back[first: first + n * stride - (stride - pb)].as_strided((n, pb), (stride, 1)).cpu().numpy()
        assert np.array_equal(got.reshape(-1), plain), "decrypt differs from the plaintext"
        around = back[mask]
        assert bool((around == (before[mask] if inplace else 0x5D)).all()), "bytes outside the payloads changed"
        assert ctx.check() == ca.CYAES_OK
        ctx.close()
    assert torch.equal(outs[0], outs[2]) and torch.equal(outs[1], outs[2])


def test_strided_stream_beyond_4gib():
    """A strided stream spanning more than 4 GiB (three 2,048-B payloads 2 GiB
    + 16 B apart): the flat decrypt's strided rows use 32-bit offsets, so the
    runtime sends such a stream through the list path; encrypt and decrypt in
    place stay bit-exact and the bytes between payloads are untouched."""
    import numpy as np
    import torch
    n, pb, stride, first = 3, 2048, (1 << 31) + 16, 12
    key = _keys(1, 71)[0]
    rng = np.random.default_rng(71)
    plain = [rng.integers(0, 256, pb, dtype=np.uint8) for _ in range(n)]
    ct = [np.frombuffer(bytes(oracle.Rijndael(key).encrypt(bytearray(x.tobytes()))), np.uint8) for x in plain]
    size = first + (n - 1) * stride + pb + 64
    buf = torch.full((size,), 0xA5, dtype=torch.uint8, device="cuda")
    offs = [first + p * stride for p in range(n)]
    for o, x in zip(offs, plain):
        buf[o:o + pb] = torch.from_numpy(x).cuda()
    ctx = ca.GpuContext(0)
    ctx.set_keys(key)
    ctx.encrypt_strided(buf, buf, first, stride, n, pb)
    for o, x in zip(offs, ct):
        assert np.array_equal(buf[o:o + pb].cpu().numpy(), x)
    ctx.decrypt_strided(buf, buf, first, stride, n, pb)
    for o, x in zip(offs, plain):
        assert np.array_equal(buf[o:o + pb].cpu().numpy(), x)
        assert int((buf[o - 12:o] != 0xA5).sum()) == 0 and int((buf[o + pb:o + pb + 12] != 0xA5).sum()) == 0
    assert ctx.check() == ca.CYAES_OK
    ctx.close()
    del buf
    torch.cuda.empty_cache()


@pytest.mark.parametrize("first", [0, 16, 12])
def test_strided_contiguous_stream(first):
    """A strided stream whose payloads lie back to back (stride = payload
    bytes): at a 16-B aligned start it runs as a contiguous uniform batch,
    per-session keys included; at a 4-B aligned one through the strided path.
    Bit-exact against the oracle either way, bytes around the stream untouched."""
    import numpy as np
    import torch
    n, pb, ppk = 257, 1472, 16
    keys = _keys((n - 1) // ppk + 1, 81)
    rng = np.random.default_rng(81)
    plain = rng.integers(0, 256, n * pb, dtype=np.uint8)
    ct = np.concatenate([np.frombuffer(bytes(oracle.Rijndael(keys[p // ppk]).encrypt(
        bytearray(plain[p * pb:(p + 1) * pb].tobytes()))), np.uint8) for p in range(n)])
    ctx = ca.GpuContext(0)
    ctx.set_keys(b"".join(keys))
    buf = torch.full((first + n * pb + 32,), 0xA5, dtype=torch.uint8, device="cuda")
    buf[first:first + n * pb] = torch.from_numpy(plain).cuda()
    ctx.encrypt_strided(buf, buf, first, pb, n, pb, payloads_per_key=ppk)
    got = buf.cpu().numpy()
    assert np.array_equal(got[first:first + n * pb], ct)
    assert (got[:first] == 0xA5).all() and (got[first + n * pb:] == 0xA5).all()
    ctx.decrypt_strided(buf, buf, first, pb, n, pb, payloads_per_key=ppk)
    assert np.array_equal(buf[first:first + n * pb].cpu().numpy(), plain)
    assert ctx.check() == ca.CYAES_OK
    ctx.close()


def test_strided_batch_session_keys():
    """Strided batches with per-session keys (payloads_per_key and a key index
    array) run as ragged batches with lists written on the device; the bytes
    between payloads are untouched and every payload matches the oracle under
    its own key (relay_server.cpp:218-240 gives each connection its key)."""
    import numpy as np
    import torch
    rng = np.random.default_rng(61)
    n, pb, stride, first, ppk = 300, 1472, 1500, 20, 7
    nk = (n + ppk - 1) // ppk
    keys = [oracle.session_key(s) for s in range(nk)]
    ctx = ca.GpuContext(0)
    ctx.set_keys(b"".join(keys))
    buf = rng.integers(0, 256, first + n * stride + 64, dtype=np.uint8)
    pt = np.stack([buf[first + p * stride: first + p * stride + pb] for p in range(n)]).reshape(-1)
    want = oracle.batch(False, keys, ppk, pt, pb, nthreads=8)
    d = torch.from_numpy(buf.copy()).cuda()
    ctx.encrypt_strided(d, d, first, stride, n, pb, payloads_per_key=ppk)
    got = d.cpu().numpy()
    for p in range(n):
        o = first + p * stride
        assert np.array_equal(got[o:o + pb], want[p * pb:(p + 1) * pb]), p
        assert np.array_equal(got[o + pb:o + stride], buf[o + pb:o + stride])
    kidx = torch.from_numpy((np.arange(n) // ppk).astype(np.uint32)).cuda()
    ctx.decrypt_strided(d, d, first, stride, n, pb, key_idx=kidx)
    assert np.array_equal(d.cpu().numpy(), buf)
    assert ctx.check() == ca.CYAES_OK
    ctx.close()
