"""oracle.py -- TEST INFRASTRUCTURE ONLY: ctypes wrapper of oracle/liboracle.so.

liboracle.so is the plain-C restatement of the reference's cyCrypt AES path
(oracle/aes_oracle.c; cites thejinchao/cyclone cyr_rijndael.cpp line by
line).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
may import this module, and only as the checker / CPU baseline -- the
product (cyclone_amd) never does.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
PLAINTEXT_SEED = 0x5EEDC1C1
SESSION_KEY_SEED = 0xC1C10E55D0000000  # config D session keys
KEY_00_0F = bytes(range(16))

_u8p = ctypes.c_void_p


class OracleKey(ctypes.Structure):
    _fields_ = [("Ke", (ctypes.c_uint32 * 4) * 11), ("Kd", (ctypes.c_uint32 * 4) * 11)]

    def words(self):
        return ([self.Ke[r][c] for r in range(11) for c in range(4)],
                [self.Kd[r][c] for r in range(11) for c in range(4)])


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError("oracle not built: %s (run `make oracle`)" % LIB_PATH)
        L = ctypes.CDLL(LIB_PATH)
        L.cyo_table.restype = ctypes.c_void_p
        L.cyo_table.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_size_t)]
        L.cyo_default_iv.restype = ctypes.c_void_p
        L.cyo_key_size.restype = ctypes.c_size_t
        L.cyo_key_expand.argtypes = [_u8p, ctypes.POINTER(OracleKey)]
        L.cyo_encrypt.argtypes = [ctypes.POINTER(OracleKey), _u8p, _u8p, ctypes.c_size_t, _u8p]
        L.cyo_decrypt.argtypes = [ctypes.POINTER(OracleKey), _u8p, _u8p, ctypes.c_size_t, _u8p]
        L.cyo_fill_synthetic.argtypes = [_u8p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64]
        L.cyo_session_key.argtypes = [ctypes.c_uint64, ctypes.c_uint64, _u8p]
        L.cyo_batch.argtypes = [ctypes.c_int, ctypes.POINTER(OracleKey), ctypes.c_uint32, _u8p, _u8p,
                                ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int]
        L.cyo_batch_ragged.argtypes = [ctypes.c_int, ctypes.POINTER(OracleKey), ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int]
        _lib = L
    return _lib


TABLE_NAMES = ["sm_S", "sm_Si", "sm_T1", "sm_T2", "sm_T3", "sm_T4", "sm_T5", "sm_T6", "sm_T7", "sm_T8",
               "sm_U1", "sm_U2", "sm_U3", "sm_U4", "sm_rcon"]


def table_bytes(name):
    n = ctypes.c_size_t()
    p = lib().cyo_table(TABLE_NAMES.index(name), ctypes.byref(n))
    return ctypes.string_at(p, n.value)


def default_iv():
    return ctypes.string_at(lib().cyo_default_iv(), 16)


def key_expand(key):
    k = OracleKey()
    kb = (ctypes.c_uint8 * 16).from_buffer_copy(bytes(key))
    lib().cyo_key_expand(ctypes.addressof(kb), ctypes.byref(k))
    return k


_EMPTY = (ctypes.c_uint8 * 16)()


def _addr(buf):
    if len(buf) == 0:
        return ctypes.addressof(_EMPTY)  # reference asserts non-NULL even for size 0
    return ctypes.addressof((ctypes.c_uint8 * len(buf)).from_buffer(buf))


class Rijndael:
    """Oracle twin of cyclone::Rijndael (cyr_rijndael.h:11-53)."""

    BLOCK_SIZE = 16
    DefaultIV = bytes(range(16))

    def __init__(self, key):
        self.key = key_expand(key)

    def _run(self, fn, inp, out, size, iv):
        src = inp if isinstance(inp, bytearray) else bytearray(inp)
        if out is None:
            out = bytearray(len(src) if size is None else size)
        dst = src if out is inp else out
        size = len(src) if size is None else size
        ivp = _addr(iv) if iv is not None else None
        rc = fn(ctypes.byref(self.key), _addr(src), _addr(dst), size, ivp)
        if rc != 0:
            raise ValueError("oracle rejected arguments (reference would assert)")
        return out

    def encrypt(self, inp, out=None, size=None, iv=None):
        return self._run(lib().cyo_encrypt, inp, out, size, iv)

    def decrypt(self, inp, out=None, size=None, iv=None):
        return self._run(lib().cyo_decrypt, inp, out, size, iv)


def synthetic(p0, npayloads, payload_bytes, seed=PLAINTEXT_SEED):
    buf = np.empty(npayloads * payload_bytes, dtype=np.uint8)
    lib().cyo_fill_synthetic(buf.ctypes.data, p0, npayloads, payload_bytes, seed)
    return buf


def session_key(s, seed=SESSION_KEY_SEED):
    k = (ctypes.c_uint8 * 16)()
    lib().cyo_session_key(seed, s, ctypes.addressof(k))
    return bytes(k)


def batch(decrypt, keys, payloads_per_key, data, payload_bytes, nthreads=1):
    """Relay semantics: every payload an independent chain from DefaultIV.
    keys: list of 16-byte keys; data: uint8 numpy array (contiguous)."""
    ks = (OracleKey * len(keys))()
    for i, k in enumerate(keys):
        ks[i] = key_expand(k)
    data = np.ascontiguousarray(data, dtype=np.uint8)
    out = np.empty_like(data)
    n = data.size // payload_bytes
    rc = lib().cyo_batch(1 if decrypt else 0, ks, payloads_per_key, data.ctypes.data, out.ctypes.data, n,
                         payload_bytes, nthreads)
    if rc != 0:
        raise ValueError("oracle batch rejected arguments")
    return out


def batch_ragged(decrypt, key, buf, offsets, nbytes, nthreads=1):
    """Relay stream in place: payload p = buf[offsets[p] : offsets[p] + nbytes[p]],
    each an independent chain from DefaultIV under one key (cyo_batch_ragged).
    buf: writable contiguous uint8 numpy array, modified in place."""
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    nbytes = np.ascontiguousarray(nbytes, dtype=np.uint32)
    if offsets.size != nbytes.size or (offsets.size and int((offsets + nbytes).max()) > buf.size):
        raise ValueError("payload outside the buffer")
    k = key_expand(key)
    rc = lib().cyo_batch_ragged(1 if decrypt else 0, ctypes.byref(k), buf.ctypes.data, offsets.ctypes.data,
                                nbytes.ctypes.data, offsets.size, nthreads)
    if rc != 0:
        raise ValueError("oracle ragged batch rejected arguments")
    return buf


def _splitmix64(x):
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def digest(buf):
    """Digest of include/cyaes.h cyaes_gpu_digest: (XOR h_i, SUM h_i mod 2^64),
    h_i = splitmix64(word_i ^ splitmix64(i))."""
    w = np.frombuffer(np.ascontiguousarray(buf).tobytes() if not isinstance(buf, np.ndarray) else
                      np.ascontiguousarray(buf).view(np.uint8), dtype="<u8")
    i = np.arange(w.size, dtype=np.uint64)
    h = _splitmix64(w ^ _splitmix64(i))
    x = np.bitwise_xor.reduce(h) if h.size else np.uint64(0)
    with np.errstate(over="ignore"):
        s = np.add.reduce(h, dtype=np.uint64) if h.size else np.uint64(0)
    return int(x), int(s)


def adler32(adler, data):
    """cyclone::adler32 (cyr_adler32.cpp:66-133); data None => the NULL-buffer rule."""
    f = lib().cyo_adler32
    f.restype = ctypes.c_uint32
    f.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t]
    if data is None:
        return f(adler, None, 0)
    arr = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    return f(adler, arr.ctypes.data if arr.size else None, arr.size)
