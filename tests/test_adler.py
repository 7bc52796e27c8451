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
