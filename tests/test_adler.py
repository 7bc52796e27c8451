"""Adler-32 on the MI355X (include/cyaes_adler32.h) vs the oracle restatement
of cyr_adler32.cpp:66-133 (pinned by the reference's KATs in test_oracle.py)."""
import ctypes
import random

import numpy as np
import pytest

import cyclone_amd as ca
import oracle

pytestmark = pytest.mark.gpu


def _lib():
    return ca.load_library()


def test_batch_matches_oracle_any_offsets_lengths():
    import torch
    rng = random.Random(41)
    lens = [0, 1, 2, 3, 15, 16, 17, 31, 33, 64, 255, 1023, 5551, 5552, 5553, 65280, 65536, 200001]
    lens += [rng.randrange(0, 70000) for _ in range(300)]
    offs, pos = [], 0
    for n in lens:
        pos += rng.randrange(0, 20)  # arbitrary byte offsets
        offs.append(pos)
        pos += n
    data = np.frombuffer(bytes(rng.getrandbits(8) for _ in range(pos + 16)), dtype=np.uint8).copy()
    adl = [rng.choice([1, rng.getrandbits(32) & 0xFFF0FFF0, (65520 << 16) | 65520]) for _ in lens]
    adl[1] = 0xFFFFFFFF  # len 1 with an out-of-range running value: the reference's subtraction rule
    d = torch.from_numpy(data).cuda()
    d_off = torch.tensor(offs, dtype=torch.int64).cuda()
    d_len = torch.tensor(lens, dtype=torch.int64).cuda()
    d_in = torch.tensor(np.array(adl, dtype=np.uint32).view(np.int32)).cuda()
    d_out = torch.empty(len(lens), dtype=torch.int32).cuda()
    lib = _lib()
    assert lib.cyaes_gpu_adler32_batch(d.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), d_in.data_ptr(),
                                       d_out.data_ptr(), len(lens), None) == 0
    got = d_out.cpu().numpy().view(np.uint32)
    for k, (o, n) in enumerate(zip(offs, lens)):
        assert int(got[k]) == oracle.adler32(adl[k], data[o:o + n].tobytes()), (k, o, n, hex(adl[k]))
    # NULL adler_in => INITIAL_ADLER
    assert lib.cyaes_gpu_adler32_batch(d.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), None,
                                       d_out.data_ptr(), len(lens), None) == 0
    got = d_out.cpu().numpy().view(np.uint32)
    for k, (o, n) in enumerate(zip(offs, lens)):
        assert int(got[k]) == oracle.adler32(1, data[o:o + n].tobytes())


def test_large_buffer_and_split_property():
    import torch
    lib = _lib()
    n = (1 << 30) + 12345
    d = torch.empty(n + 3, dtype=torch.uint8, device="cuda")
    ctx = ca.GpuContext(0)
    ctx.fill_synthetic(d, 0, 1, (n + 3) // 8 * 8, 77)  # seeded bytes
    torch.cuda.synchronize()
    host = d.cpu().numpy()
    out = ctypes.c_uint32()
    assert lib.cyaes_gpu_adler32(d.data_ptr() + 3, n, 1, ctypes.byref(out), None) == 0  # unaligned start
    want = oracle.adler32(1, host[3:3 + n])
    assert out.value == want
    # chaining (RingBuf::checksum over a wrap, cyc_ring_buf.cpp:365-387)
    cut = 777777777
    a = ctypes.c_uint32()
    b = ctypes.c_uint32()
    assert lib.cyaes_gpu_adler32(d.data_ptr() + 3, cut, 1, ctypes.byref(a), None) == 0
    assert lib.cyaes_gpu_adler32(d.data_ptr() + 3 + cut, n - cut, a.value, ctypes.byref(b), None) == 0
    assert b.value == want
    assert lib.cyaes_gpu_adler32(d.data_ptr(), 0, 0xdeadbeef, ctypes.byref(out), None) == 0 and out.value == 1
    ctx.close()


def test_ringbuf_checksum_reference_kat_on_device():
    """The RingBuf::checksum answers of the reference's own test
    (test/unit/cyt_unit_ring_buf.cpp:370-401) from the device Adler-32: byte
    ranges of "Hello,World!" in one batch, and a wrapped ring buffer as two
    chained calls (the running value of the first piece seeds the second,
    cyc_ring_buf.cpp:375-384)."""
    import json
    import os
    import torch
    k = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "ref_kat.json")))["ringbuf_checksum"]
    lib = _lib()
    text = np.frombuffer(k["text"].encode(), dtype=np.uint8).copy()
    d = torch.from_numpy(text).cuda()
    cases = [(0, len(text), k["full"])] + [(c["off"], c["count"], c["adler"]) for c in k["ranges"]]
    d_off = torch.tensor([c[0] for c in cases], dtype=torch.int64).cuda()
    d_len = torch.tensor([c[1] for c in cases], dtype=torch.int64).cuda()
    d_out = torch.empty(len(cases), dtype=torch.int32).cuda()
    assert lib.cyaes_gpu_adler32_batch(d.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), None, d_out.data_ptr(),
                                       len(cases), None) == 0
    got = d_out.cpu().numpy().view(np.uint32)
    assert [int(x) for x in got] == [c[2] for c in cases]
    # wrap: ring of capacity + 1 bytes (cyc_ring_buf.cpp:20), data from read = end - w, 4w bytes
    rng = random.Random(7)
    w = k["wrap_size"]
    ring = np.frombuffer(bytes(rng.getrandbits(8) for _ in range(k["capacity"] + 1)), dtype=np.uint8).copy()
    dr = torch.from_numpy(ring).cuda()
    read = len(ring) - w
    stream = np.concatenate([ring[read:], ring[:3 * w]])
    a = ctypes.c_uint32()
    b = ctypes.c_uint32()
    assert lib.cyaes_gpu_adler32(dr.data_ptr() + read, w, 1, ctypes.byref(a), None) == 0
    assert lib.cyaes_gpu_adler32(dr.data_ptr(), 2 * w, a.value, ctypes.byref(b), None) == 0
    assert b.value == oracle.adler32(1, stream[:3 * w].tobytes())

