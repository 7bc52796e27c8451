"""Pins the oracle (oracle/aes_oracle.c) to the reference before it is trusted.

Reference: thejinchao/cyclone test/unit/cyt_unit_crypt.cpp:173-248 (the
Rijndael TEST_CASE) and source/cyCrypt/crypt/cyr_rijndael.cpp.  Fixtures:
tests/golden/ref_kat.json + ref_tables.json (from the reference text by
gen_ref_fixtures.py) and openssl_vectors.json (gen_openssl_vectors.c).
"""
import hashlib
import random
import struct

import numpy as np
import pytest

import oracle


def test_tables_match_reference_digests(golden):
    """Regenerated S/Si/T1..T8/U1..U4/rcon == cyr_rijndael.cpp:25-501."""
    ref = golden["tables"]
    for name in oracle.TABLE_NAMES:
        got = oracle.table_bytes(name)
        assert len(got) == ref[name]["bytes"], name
        assert hashlib.sha256(got).hexdigest() == ref[name]["sha256"], name
    assert oracle.default_iv().hex() == ref["DefaultIV"]


def test_reference_kat(golden):
    """cyt_unit_crypt.cpp:190-200: one-shot encrypt / decrypt, iv=nullptr."""
    k = golden["kat"]
    aes = oracle.Rijndael(bytes.fromhex(k["key"]))
    plain, cipher = bytes.fromhex(k["plaintext"]), bytes.fromhex(k["ciphertext"])
    assert len(plain) % aes.BLOCK_SIZE == 0
    assert bytes(aes.encrypt(plain)) == cipher
    assert bytes(aes.decrypt(cipher)) == plain


def test_reference_iv_streaming(golden):
    """cyt_unit_crypt.cpp:203-219: 16-byte calls carrying iv reproduce the chain."""
    k = golden["kat"]
    aes = oracle.Rijndael(bytes.fromhex(k["key"]))
    plain, cipher = bytes.fromhex(k["plaintext"]), bytes.fromhex(k["ciphertext"])
    iv = bytearray(aes.DefaultIV)
    out = bytearray()
    for i in range(0, len(plain), 16):
        out += aes.encrypt(plain[i:i + 16], None, 16, iv)
    assert bytes(out) == cipher and bytes(iv) == bytes.fromhex(k["iv_check"])
    iv = bytearray(aes.DefaultIV)
    out = bytearray()
    for i in range(0, len(cipher), 16):
        out += aes.decrypt(cipher[i:i + 16], None, 16, iv)
    assert bytes(out) == plain and bytes(iv) == bytes.fromhex(k["iv_check"])


def test_reference_in_place(golden):
    """cyt_unit_crypt.cpp:221-231: encrypt(buf, buf) / decrypt(buf, buf)."""
    k = golden["kat"]
    aes = oracle.Rijndael(bytes.fromhex(k["key"]))
    buf = bytearray.fromhex(k["plaintext"])
    aes.encrypt(buf, buf)
    assert buf.hex() == k["ciphertext"]
    aes.decrypt(buf, buf)
    assert buf.hex() == k["plaintext"]


def test_reference_random_roundtrips():
    """cyt_unit_crypt.cpp:234-247: 20 random keys, 128-byte round trips."""
    rng = random.Random(1)
    for _ in range(20):
        aes = oracle.Rijndael(bytes(rng.randrange(256) for _ in range(16)))
        buf = bytes(rng.randrange(256) for _ in range(128))
        assert bytes(aes.decrypt(aes.encrypt(buf))) == buf


def test_size_zero_is_noop_and_bad_size_rejected():
    aes = oracle.Rijndael(oracle.KEY_00_0F)
    iv = bytearray(b"\x55" * 16)
    aes.encrypt(b"", bytearray(16), 0, iv)
    assert bytes(iv) == b"\x55" * 16
    with pytest.raises(ValueError):
        aes.encrypt(b"\0" * 17, bytearray(17), 17)


def test_fips197_and_sp800_38a(golden):
    ov = golden["openssl"]
    c1 = ov["fips197_c1"]
    aes = oracle.Rijndael(bytes.fromhex(c1["key"]))
    assert bytes(aes.encrypt(bytes.fromhex(c1["plaintext"]), None, 16, bytearray(16))).hex() == c1["ciphertext"]
    f = ov["sp800_38a_f21"]
    aes = oracle.Rijndael(bytes.fromhex(f["key"]))
    assert f["iv"] == aes.DefaultIV.hex()  # SP 800-38A's IV is the reference DefaultIV
    assert bytes(aes.encrypt(bytes.fromhex(f["plaintext"]))).hex() == f["ciphertext"]
    assert bytes(aes.decrypt(bytes.fromhex(f["ciphertext"]))).hex() == f["plaintext"]  # F.2.2


def test_key_schedules_match_openssl(golden):
    """m_Ke / m_Kd (cyr_rijndael.h:50,52) == OpenSSL rd_key (FIPS-197 A.1 incl.)."""
    for s in golden["openssl"]["schedules"]:
        ke, kd = oracle.key_expand(bytes.fromhex(s["key"])).words()
        assert ke == s["ke"] and kd == s["kd"]


def test_synthetic_sizes_match_openssl(golden):
    """Generator + oracle vs OpenSSL at every configured payload size."""
    for v in golden["openssl"]["sizes"]:
        pb, p = v["payload_bytes"], v["p"]
        pt = oracle.synthetic(p, 1, pb)
        ct = oracle.batch(False, [oracle.KEY_00_0F], 0, pt, pb)
        assert hashlib.sha256(ct.tobytes()).hexdigest() == v["cipher_sha256"], (pb, p)
        assert ct[-16:].tobytes().hex() == v["last_block"]
        if "ciphertext" in v:
            assert ct.tobytes().hex() == v["ciphertext"]
        assert np.array_equal(oracle.batch(True, [oracle.KEY_00_0F], 0, ct, pb), pt)


def test_session_keys_match(golden):
    assert [oracle.session_key(s).hex() for s in range(3)] == golden["openssl"]["session_keys"]


def test_config_a_full_digest(golden):
    """Config A (4096 x 1024 B, the reference's CPU case) end to end on the oracle."""
    cfg = golden["openssl"]["configs"]["A"]
    pt = oracle.synthetic(0, cfg["npayloads"], cfg["payload_bytes"])
    assert "%016x" % oracle.digest(pt)[0] == cfg["plain_digest"][0]
    ct = oracle.batch(False, [oracle.KEY_00_0F], 0, pt, cfg["payload_bytes"], nthreads=8)
    x, s = oracle.digest(ct)
    assert ["%016x" % x, "%016x" % s] == cfg["cipher_digest"]
    assert np.array_equal(oracle.batch(True, [oracle.KEY_00_0F], 0, ct, cfg["payload_bytes"], nthreads=8), pt)


def test_config_d_keyed_prefix(golden):
    """Config D's per-session keys: first 3 sessions x 256 payloads vs per-payload oracle."""
    pb, ppk = 1472, 256
    n = 3 * ppk
    pt = oracle.synthetic(0, n, pb)
    keys = [oracle.session_key(s) for s in range(3)]
    ct = oracle.batch(False, keys, ppk, pt, pb, nthreads=8)
    for p in (0, 255, 256, 700):
        one = oracle.Rijndael(keys[p // ppk]).encrypt(pt[p * pb:(p + 1) * pb].tobytes())
        assert bytes(one) == ct[p * pb:(p + 1) * pb].tobytes()


def test_digest_definition():
    w = np.array([1, 2, 3], dtype="<u8")
    x, s = oracle.digest(w.view(np.uint8))
    hs = [int(oracle._splitmix64(np.uint64(v) ^ oracle._splitmix64(np.uint64(i)))) for i, v in enumerate([1, 2, 3])]
    assert x == hs[0] ^ hs[1] ^ hs[2] and s == sum(hs) % (1 << 64)
    assert struct.calcsize("<Q") == 8


# ---- Adler-32 (cyr_adler32.cpp:66-133) -------------------------------------
def test_adler32_oracle_reference_kat(golden):
    """The reference's own known answers, test/unit/cyt_unit_crypt.cpp:18-50."""
    k = golden["kat"]["adler32"]
    assert oracle.adler32(0, None) == k["null_or_empty"] == 1
    assert oracle.adler32(0xFFFFFFFF, None) == 1
    for s in k["strings"]:
        assert oracle.adler32(1, s["text"].encode()) == s["adler"]
    data = bytes.fromhex(k["data_buf"])
    assert oracle.adler32(1, data) == k["data_adler"]
    first = k["split"]
    assert oracle.adler32(oracle.adler32(1, data[:first]), data[first:]) == k["data_adler"]


def ringbuf_checksum(ring, read, size, off, count):
    """RingBuf::checksum (cyc_ring_buf.cpp:365-387) over a ring of len(ring)
    bytes holding `size` bytes from index `read`: Adler-32 chained over the
    (at most two) contiguous pieces; an empty or out-of-range request returns
    INITIAL_ADLER."""
    adler = 1
    if off > size or off + count > size or count == 0:
        return adler
    pos, done = (read + off) % len(ring), 0
    while done != count:
        n = min(len(ring) - pos, count - done)
        adler = oracle.adler32(adler, bytes(ring[pos:pos + n]))
        pos, done = (pos + n) % len(ring), done + n
    return adler


def test_ringbuf_checksum_reference_kat(golden):
    """RingBuf::checksum answers of the reference's own test
    (test/unit/cyt_unit_ring_buf.cpp:370-401) on the oracle's Adler-32."""
    k = golden["kat"]["ringbuf_checksum"]
    text = k["text"].encode()
    ring = bytearray(k["capacity"] + 1)  # m_end = capacity + 1 (cyc_ring_buf.cpp:20)
    ring[:len(text)] = text
    n = len(text)
    assert ringbuf_checksum(ring, 0, n, 0, n) == k["full"]
    for c in k["ranges"]:
        assert ringbuf_checksum(ring, 0, n, c["off"], c["count"]) == c["adler"]
    for off, count in [(n, 0), (n, 1), (0, n + 1), (0, 0)]:  # :375-378
        assert ringbuf_checksum(ring, 0, n, off, count) == 1
    # wrap (:387-401): the buffer's bytes [read, end) then [0, ...) chain as one stream
    rng = random.Random(7)
    w = k["wrap_size"]
    ring = bytearray(rng.getrandbits(8) for _ in range(k["capacity"] + 1))
    read = len(ring) - w
    size = 4 * w
    stream = bytes(ring[read:]) + bytes(ring[:size - w])
    for off, count in [(0, w), (0, 3 * w), (2 * w, w), (3 * w, w)]:
        assert ringbuf_checksum(ring, read, size, off, count) == oracle.adler32(1, stream[off:off + count])


def test_adler32_oracle_random_split_and_zlib():
    """cyt_unit_crypt.cpp:54-78 (random split property) and, independently,
    zlib's adler32 (same algorithm) for every length class of the reference's
    code paths (1, <16, NMAX blocks)."""
    import zlib
    rng = random.Random(31)
    for _ in range(100):
        size = 257 - rng.randrange(32)
        buf = bytes(rng.randrange(256) for _ in range(size))
        cut = rng.randrange(size - 1) + 1
        assert oracle.adler32(oracle.adler32(1, buf[:cut]), buf[cut:]) == oracle.adler32(1, buf)
    for n in [1, 2, 15, 16, 17, 5551, 5552, 5553, 11104, 20000]:
        buf = bytes(rng.randrange(256) for _ in range(n))
        start = zlib.adler32(bytes(rng.randrange(256) for _ in range(7)))
        assert oracle.adler32(1, buf) == zlib.adler32(buf)
        assert oracle.adler32(start, buf) == zlib.adler32(buf, start)
    # the reference's own rule differs from zlib for len == 0
    assert oracle.adler32(0xdeadbeef, b"") == 1 and zlib.adler32(b"", 0xdeadbeef) == 0xdeadbeef


def test_ragged_relay_batch_matches_per_packet_calls():
    """cyo_batch_ragged (the relay stream restatement): each payload of a
    ragged in-place stream equals one Rijndael::encrypt(buf, buf, size) call
    from DefaultIV (relay_local.cpp:206), payloads at 4-B phases, sizes 0 to
    0xFF00; decrypt restores the stream; bytes between payloads untouched."""
    rng = np.random.default_rng(11)
    key = bytes(rng.integers(0, 256, 16, dtype=np.uint8))
    sizes = np.array([0, 16, 0xFF00, 1472, 32, 4080, 65264, 16 * 7], dtype=np.uint32)
    pkt = sizes.astype(np.uint64) + 12
    offsets = (np.cumsum(pkt) - pkt + 12).astype(np.uint64)
    buf = rng.integers(0, 256, int(pkt.sum()) + 16, dtype=np.uint8)
    ref = buf.copy()
    oracle.batch_ragged(False, key, buf, offsets, sizes, nthreads=3)
    aes = oracle.Rijndael(key)
    mask = np.ones(buf.size, dtype=bool)
    for o, n in zip(offsets.tolist(), sizes.tolist()):
        want = bytes(aes.encrypt(ref[o:o + n].tobytes(), None, n, None)) if n else b""
        assert bytes(buf[o:o + n]) == want
        mask[o:o + n] = False
    assert np.array_equal(buf[mask], ref[mask])
    oracle.batch_ragged(True, key, buf, offsets, sizes, nthreads=2)
    assert np.array_equal(buf, ref)


def test_mixed_relay_stream_layout_is_the_golden_one():
    """bench.py's relay_stream.mixed regenerates the layout its golden digests
    (tests/golden/relay_mixed.json) were computed on: same packets, payload
    bytes, stream size and offset / size lists (hash)."""
    import json
    import os
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    g = json.load(open(os.path.join(root, "tests", "golden", "relay_mixed.json")))
    offsets, nbytes, alloc = bench.mixed_stream_layout(g["chunk_bytes"])
    assert (int(offsets.size), int(nbytes.sum()), alloc) == (g["packets"], g["payload_bytes"], g["stream_bytes"])
    assert hashlib.sha256(offsets.tobytes() + nbytes.tobytes()).hexdigest()[:16] == g["layout_sha256_16"]
    assert int(nbytes.max()) == bench.RELAY_MAX_CHUNK and int((nbytes % 16).max()) == 0
    assert int(offsets[0]) == 12 and np.all(offsets[1:] == offsets[:-1] + nbytes[:-1].astype(np.uint64) + 12)
