"""Randomized parity sweep over the batch API (GPU): every kernel choice the
runtime can make for encrypt and decrypt, against the oracle, bit-exact.

Each case draws a batch shape, key mode, IV mode and layout from a seeded
generator and forces the kernel choice through the runtime's A/B knobs:
  encrypt  CYAES_QUAD_MAX_CHAINS   lane per chain / four lanes per chain
  decrypt  CYAES_RAGGED_GROUP      payloads per wave group of the ragged kernel
           CYAES_DEC_GRID / CYAES_DEC_RANGE_STEPS / CYAES_DEC_DYN   work ranges from the
           ticket counter on a small grid, or the static per-wave split
Layouts: uniform (flat decrypt, incl. the session-aligned keyed path),
ragged relay-packet streams (payload at packet offset 12, gaps, empties) and
strided streams of equal payloads (cyaes_gpu_{en,de}crypt_strided: any 4-B
phase and gap; k_encrypt_lines for whole 1,024-payload groups, also on a
capped grid, CYAES_LINES_GRID; no IV arrays in that API).
Semantics: Rijndael::encrypt/decrypt per payload (cyr_rijndael.cpp:588-635),
IV in/out per payload, in place allowed."""
import os

import numpy as np
import pytest

import cyclone_amd as ca
import oracle

pytestmark = pytest.mark.gpu
NCASES = int(os.environ.get("CYAES_SWEEP_CASES", "160"))  # soak runs raise it


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "gpu tests need a ROCm device"
    return t


def dev(torch, arr):
    a = np.ascontiguousarray(arr)
    return torch.from_numpy(a.view(np.uint8).reshape(-1).copy()).to("cuda")


def host(t):
    import torch as _t
    _t.cuda.synchronize()
    return t.cpu().numpy()


def context(env):
    old = {k: os.environ.get(k) for k in env}
    try:
        for k, v in env.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        return ca.GpuContext(0)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def draw_case(seed):
    rng = np.random.default_rng(1000 + seed)
    layout = rng.choice(["uniform", "ragged", "strided"])
    n = int(rng.choice([1, 7, 63, 64, 65, 300, 1000, 2500]))
    if layout == "strided":
        n = int(rng.choice([1, 63, 1024, 2100, 3072]))
    if layout == "uniform":
        blocks = np.full(n, int(rng.choice([1, 3, 8, 9, 15, 16, 23, 92, 256, 300])), dtype=np.uint32)
    elif layout == "strided":
        blocks = np.full(n, int(rng.choice([1, 4, 8, 9, 23, 92, 100])), dtype=np.uint32)
    else:
        blocks = rng.choice([0, 1, 2, 5, 7, 8, 9, 16, 63, 64, 65, 92, 257], n).astype(np.uint32)
        blocks[rng.integers(0, n, max(1, n // 200))] = int(rng.choice([600, 4080]))
    keying = rng.choice(["one", "index", "ppk"])
    ppk = int(rng.choice([1, 2, 7, 16, 64])) if keying == "ppk" else 0
    return dict(
        rng=rng, layout=layout, n=n, blocks=blocks, keying=keying, ppk=ppk,
        iv_in=bool(rng.integers(0, 2)) and layout != "strided", iv_out=bool(rng.integers(0, 2)) and layout != "strided",
        inplace=bool(rng.integers(0, 2)), first=4 * int(rng.integers(0, 17)), gap=4 * int(rng.integers(0, 21)),
        env={"CYAES_QUAD_MAX_CHAINS": str(rng.choice(["0", str(1 << 40)])) if rng.integers(0, 3) else None,
             "CYAES_LINES_GRID": str(rng.choice([1, 3, 7])) if rng.integers(0, 3) == 0 else None,
             "CYAES_RAGGED_GROUP": str(rng.choice([1, 2, 5, 64])) if rng.integers(0, 3) else None,
             # decrypt work distribution: a small grid with 1- or 3-step ticket ranges, or the static split
             "CYAES_DEC_GRID": str(rng.choice([1, 2, 5])) if rng.integers(0, 2) else None,
             "CYAES_DEC_RANGE_STEPS": str(rng.choice([1, 3])) if rng.integers(0, 2) else None,
             "CYAES_DEC_DYN": str(rng.integers(0, 2)) if rng.integers(0, 3) else None})


@pytest.mark.parametrize("seed", range(NCASES))
def test_batch_sweep(torch, seed):
    k = draw_case(seed)
    rng, n, blocks, ppk = k["rng"], k["n"], k["blocks"], k["ppk"]
    sizes = blocks * 16
    nk = (n - 1) // ppk + 1 if ppk else 11
    keys = [bytes(rng.integers(0, 256, 16, dtype=np.uint8)) for _ in range(nk)]
    kidx = rng.integers(0, nk, n, dtype=np.uint32) if k["keying"] == "index" else None

    def key_of(p):
        if k["keying"] == "index":
            return keys[kidx[p]]
        return keys[p // ppk] if ppk else keys[0]

    if k["layout"] == "uniform":
        offsets = np.arange(n, dtype=np.uint64) * int(sizes[0])
        total = int(n * int(sizes[0]))
    elif k["layout"] == "strided":
        stride = int(sizes[0]) + k["gap"]
        offsets = k["first"] + np.arange(n, dtype=np.uint64) * stride
        total = k["first"] + (n - 1) * stride + int(sizes[0])
    else:
        offsets = np.zeros(n, dtype=np.uint64)
        pos = 0
        gaps = rng.integers(0, 3, n) * 4
        for p in range(n):
            pos += 12 + int(gaps[p])
            offsets[p] = pos
            pos += int(sizes[p])
        total = pos
    ivs = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    plain = rng.integers(0, 256, max(total, 16), dtype=np.uint8)
    ct, want_iv = plain.copy(), np.empty_like(ivs)
    for p in range(n):
        o, s = int(offsets[p]), int(sizes[p])
        iv = bytearray(ivs[p].tobytes() if k["iv_in"] else oracle.default_iv())
        ct[o:o + s] = np.frombuffer(bytes(oracle.Rijndael(key_of(p)).encrypt(plain[o:o + s].tobytes(), None, s, iv)),
                                    np.uint8)
        want_iv[p] = np.frombuffer(bytes(iv), np.uint8)  # final chain (unchanged for an empty payload)

    c = context(k["env"])
    try:
        c.set_keys(b"".join(keys))
        kw = dict(key_idx=dev(torch, kidx) if kidx is not None else None, payloads_per_key=ppk)
        d_ivi = dev(torch, ivs) if k["iv_in"] else None
        d_ivo = torch.zeros(n * 16, dtype=torch.uint8, device="cuda") if k["iv_out"] else None
        d_pt = dev(torch, plain)
        d_ct = d_pt if k["inplace"] else dev(torch, plain)  # out starts as a copy: gaps keep their bytes
        if k["layout"] == "uniform":
            c.encrypt_uniform(d_pt, d_ct, n, int(sizes[0]), iv_in=d_ivi, iv_out=d_ivo, **kw)
        elif k["layout"] == "strided":
            c.encrypt_strided(d_pt, d_ct, k["first"], int(sizes[0]) + k["gap"], n, int(sizes[0]), **kw)
        else:
            d_off, d_nb = dev(torch, offsets), dev(torch, sizes)
            c.encrypt_ragged(d_pt, d_ct, d_off, d_nb, n, iv_in=d_ivi, iv_out=d_ivo, **kw)
        got = host(d_ct)
        assert np.array_equal(got[:total], ct[:total]), k
        if k["iv_out"]:
            assert np.array_equal(host(d_ivo).reshape(n, 16), want_iv), k
        # decrypt the ciphertext back; the IV out of a decrypt is the last ciphertext block
        d_src = dev(torch, ct)
        d_back = d_src if k["inplace"] else dev(torch, ct)
        d_ivo2 = torch.zeros(n * 16, dtype=torch.uint8, device="cuda") if k["iv_out"] else None
        if k["layout"] == "uniform":
            c.decrypt_uniform(d_src, d_back, n, int(sizes[0]), iv_in=d_ivi, iv_out=d_ivo2, **kw)
        elif k["layout"] == "strided":
            c.decrypt_strided(d_src, d_back, k["first"], int(sizes[0]) + k["gap"], n, int(sizes[0]), **kw)
        else:
            c.decrypt_ragged(d_src, d_back, d_off, d_nb, n, iv_in=d_ivi, iv_out=d_ivo2, **kw)
        assert np.array_equal(host(d_back)[:total], plain[:total]), k
        if k["iv_out"]:
            exp = np.array([ct[int(offsets[p]) + int(sizes[p]) - 16:int(offsets[p]) + int(sizes[p])]
                            if sizes[p] else (ivs[p] if k["iv_in"] else np.frombuffer(oracle.default_iv(), np.uint8))
                            for p in range(n)])
            assert np.array_equal(host(d_ivo2).reshape(n, 16), exp), k
        assert c.check() == ca.CYAES_OK
    finally:
        c.close()


@pytest.mark.parametrize("layout", ["uniform", "strided"])
@pytest.mark.parametrize("grid", [None, "1", "2", "5"])
@pytest.mark.parametrize("handoff", [None, "0"])
def test_inplace_decrypt_range_handoff(torch, layout, grid, handoff):
    """In-place flat decrypts whose static ranges start inside payloads: the
    carries handed over in the kernel (DecArgs.handoff, the default) or
    snapshot by the prepass (CYAES_DEC_HANDOFF=0), on full and small grids,
    against the oracle (cyr_rijndael.cpp:612-635 per payload)."""
    rng = np.random.default_rng(77 + (grid is not None) * int(grid or 0) + (layout == "strided") * 10)
    n, bpp = 301, 92  # 27,692 blocks: ranges end inside payloads on every grid here
    pb = 16 * bpp
    key = bytes(rng.integers(0, 256, 16, dtype=np.uint8))
    stride, first = (pb + 12, 12) if layout == "strided" else (pb, 0)
    plain = rng.integers(0, 256, first + n * stride + 64, dtype=np.uint8)
    ct = plain.copy()
    r = oracle.Rijndael(key)
    for p in range(n):
        o = first + p * stride
        ct[o:o + pb] = np.frombuffer(bytes(r.encrypt(plain[o:o + pb].tobytes(), None, pb,
                                                     bytearray(oracle.default_iv()))), np.uint8)
    c = context({"CYAES_DEC_GRID": grid, "CYAES_DEC_DYN": "0", "CYAES_DEC_HANDOFF": handoff})
    try:
        c.set_keys(key)
        d = dev(torch, ct)
        for _ in range(3):  # repeated launches: every one tags its records with a new epoch
            d.copy_(dev(torch, ct))
            if layout == "strided":
                c.decrypt_strided(d, d, first, stride, n, pb)
            else:
                c.decrypt_uniform(d, d, n, pb)
            assert np.array_equal(host(d), plain)
        assert c.check() == ca.CYAES_OK
    finally:
        c.close()


@pytest.mark.parametrize("pb", [1040, 1472, 4096])
@pytest.mark.parametrize("inplace", [False, True])
def test_strided_kernels_on_contiguous_payloads(torch, pb, inplace):
    """CYAES_STRIDED_FORCE=1 keeps the strided kernels (k_encrypt_lines / the
    flat decrypt's STRIDED rows) on payloads that are back to back, which the
    runtime otherwise hands to the uniform kernels: the A/B that located the
    strided decrypt's cost in its code, not its layout.
    Against the oracle, both directions."""
    rng = np.random.default_rng(pb + inplace)
    n, first = 2048 + 37, 64
    key = bytes(rng.integers(0, 256, 16, dtype=np.uint8))
    plain = rng.integers(0, 256, first + n * pb + 64, dtype=np.uint8)
    ct = plain.copy()
    r = oracle.Rijndael(key)
    for p in range(n):
        o = first + p * pb
        ct[o:o + pb] = np.frombuffer(bytes(r.encrypt(plain[o:o + pb].tobytes(), None, pb,
                                                     bytearray(oracle.default_iv()))), np.uint8)
    c = context({"CYAES_STRIDED_FORCE": "1"})
    try:
        c.set_keys(key)
        src = dev(torch, plain)
        dst = src if inplace else dev(torch, plain)
        c.encrypt_strided(src, dst, first, pb, n, pb)
        assert np.array_equal(host(dst), ct)
        src = dev(torch, ct)
        dst = src if inplace else dev(torch, ct)
        c.decrypt_strided(src, dst, first, pb, n, pb)
        assert np.array_equal(host(dst), plain)
        assert c.check() == ca.CYAES_OK
    finally:
        c.close()
