"""cyclone_amd -- MI355X-native cyCrypt AES-128-CBC (cyclone::Rijndael drop-in).

Python binding over the C-ABI declared in include/cyaes.h (ctypes; the ABI
carries plain pointers and sizes, no torch types).  The product path is the
gfx950 HIP code in libcyaes.so: importing this package without the built
library raises -- there is no CPU fallback.

Mirrors the reference interface thejinchao/cyclone
source/cyCrypt/crypt/cyr_rijndael.h:11-53:

    aes = Rijndael(key)                      # Rijndael::Rijndael  (:21)
    aes.encrypt(inp, out, size, iv=None)     # Rijndael::encrypt   (:29)
    aes.decrypt(inp, out, size, iv=None)     # Rijndael::decrypt   (:33)
    Rijndael.BLOCK_SIZE, Rijndael.DefaultIV  # (:14-18)

and exposes the batched device API (GpuContext) used by bench.py.
"""
import ctypes
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libcyaes.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "cyaes.h")

CYAES_OK, CYAES_EINVAL, CYAES_EDEVICE, CYAES_ENOMEM, CYAES_ERANGE, CYAES_ENODEV = 0, -1, -2, -3, -4, -5
BLOCK_SIZE = 16
DEFAULT_IV = bytes(range(16))

_u8p = ctypes.POINTER(ctypes.c_uint8)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_vp = ctypes.c_void_p


class CyaesKey(ctypes.Structure):
    """struct cyaes_key == Rijndael::m_Ke / m_Kd (cyr_rijndael.h:48-52)."""

    _fields_ = [("ke", (ctypes.c_uint32 * 4) * 11), ("kd", (ctypes.c_uint32 * 4) * 11)]

    def words(self):
        ke = [self.ke[r][c] for r in range(11) for c in range(4)]
        kd = [self.kd[r][c] for r in range(11) for c in range(4)]
        return ke, kd


class CyaesError(RuntimeError):
    def __init__(self, status, what=""):
        self.status = status
        super().__init__("%s: %s (status %d)" % (what or "cyaes", strerror(status), status))


# name -> (restype, argtypes); every function declared in include/cyaes.h
_SIGS = {
    "cyaes_default_iv": (_u8p, []),
    "cyaes_strerror": (ctypes.c_char_p, [ctypes.c_int]),
    "cyaes_version": (ctypes.c_char_p, []),
    "cyaes_key_expand": (ctypes.c_int, [_u8p, ctypes.POINTER(CyaesKey)]),
    "cyaes_cbc_encrypt": (ctypes.c_int, [ctypes.POINTER(CyaesKey), _vp, _vp, ctypes.c_size_t, _vp]),
    "cyaes_cbc_decrypt": (ctypes.c_int, [ctypes.POINTER(CyaesKey), _vp, _vp, ctypes.c_size_t, _vp]),
    "cyaes_gpu_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(_vp)]),
    "cyaes_gpu_destroy": (None, [_vp]),
    "cyaes_gpu_device": (ctypes.c_int, [_vp]),
    "cyaes_gpu_num_cus": (ctypes.c_int, [_vp]),
    "cyaes_gpu_set_keys": (ctypes.c_int, [_vp, _vp, ctypes.c_uint32]),
    "cyaes_gpu_set_keys_device": (ctypes.c_int, [_vp, _vp, ctypes.c_uint32, _vp]),
    "cyaes_gpu_nkeys": (ctypes.c_uint32, [_vp]),
    "cyaes_gpu_get_key": (ctypes.c_int, [_vp, ctypes.c_uint32, ctypes.POINTER(CyaesKey)]),
    "cyaes_gpu_encrypt_uniform": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_uint64, ctypes.c_uint32, _vp,
                                                 ctypes.c_uint32, _vp, _vp, _vp]),
    "cyaes_gpu_decrypt_uniform": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_uint64, ctypes.c_uint32, _vp,
                                                 ctypes.c_uint32, _vp, _vp, _vp]),
    "cyaes_gpu_encrypt_ragged": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, ctypes.c_uint64, _vp, ctypes.c_uint32,
                                                _vp, _vp, _vp]),
    "cyaes_gpu_decrypt_ragged": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, ctypes.c_uint64, _vp, ctypes.c_uint32,
                                                _vp, _vp, _vp]),
    "cyaes_gpu_check": (ctypes.c_int, [_vp]),
    "cyaes_gpu_fill_synthetic": (ctypes.c_int, [_vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                                                ctypes.c_uint64, _vp]),
    "cyaes_gpu_digest": (ctypes.c_int, [_vp, ctypes.c_uint64, _u64p, _vp]),
}

_lib = None


def header_functions(path=HEADER_PATH):
    """Names of the functions include/cyaes.h declares."""
    text = open(path).read()
    return sorted(set(re.findall(r"\b(cyaes_[a-z0-9_]+)\s*\(", text)))


def load_library(path=LIB_PATH):
    """Loads libcyaes.so (fails loudly; there is no fallback path)."""
    global _lib
    if _lib is not None and path == LIB_PATH:
        return _lib
    if not os.path.exists(path):
        raise ImportError("cyclone_amd: %s is not built (run `make` or __graft_entry__.build())" % path)
    lib = ctypes.CDLL(path)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path == LIB_PATH:
        _lib = lib
    return lib


def strerror(status):
    return load_library().cyaes_strerror(status).decode()


def version():
    return load_library().cyaes_version().decode()


def _check(status, what):
    if status != CYAES_OK:
        raise CyaesError(status, what)


def key_expand(key):
    """Host key schedule in reference layout (cyr_rijndael.cpp:507-572)."""
    key = bytes(key)
    if len(key) != 16:
        raise ValueError("AES-128 key must be 16 bytes")
    k = CyaesKey()
    _check(load_library().cyaes_key_expand((ctypes.c_uint8 * 16).from_buffer_copy(key), ctypes.byref(k)),
           "cyaes_key_expand")
    return k


class _Buf:
    """Pins a writable view (bytearray/memoryview) or a private copy of bytes."""

    def __init__(self, obj, writable):
        if isinstance(obj, (bytearray, memoryview)) or hasattr(obj, "__array_interface__"):
            mv = memoryview(obj).cast("B")
            if writable and mv.readonly:
                raise TypeError("output buffer is read-only")
            self.obj = obj
            self.n = mv.nbytes
            self.arr = (ctypes.c_uint8 * max(self.n, 1)).from_buffer(mv) if not mv.readonly else \
                (ctypes.c_uint8 * max(self.n, 1)).from_buffer_copy(mv.tobytes() or b"\0")
        else:
            if writable:
                raise TypeError("output must be a writable buffer (bytearray)")
            data = bytes(obj)
            self.obj = data
            self.n = len(data)
            self.arr = (ctypes.c_uint8 * max(self.n, 1)).from_buffer_copy(data or b"\0")

    @property
    def ptr(self):
        return ctypes.addressof(self.arr)


class Rijndael:
    """cyclone::Rijndael (cyr_rijndael.h:11-53), executed on the MI355X."""

    BLOCK_SIZE = BLOCK_SIZE
    DefaultIV = DEFAULT_IV

    def __init__(self, key):
        self._key = key_expand(key)

    def schedule(self):
        """(m_Ke words, m_Kd words), reference layout."""
        return self._key.words()

    def _run(self, fn, what, inp, out, size, iv):
        lib = load_library()
        src = _Buf(inp, False)
        if out is None:
            out = bytearray(size if size is not None else src.n)
        same = out is inp
        dst = src if same else _Buf(out, True)
        if size is None:
            size = src.n
        if size > src.n or size > dst.n:
            raise ValueError("size exceeds buffer")
        ivb = None
        if iv is not None:
            if not isinstance(iv, (bytearray, memoryview)) or len(iv) != 16:
                raise TypeError("iv must be a writable 16-byte buffer (it is updated in place)")
            ivb = (ctypes.c_uint8 * 16).from_buffer(iv)
        st = getattr(lib, fn)(ctypes.byref(self._key), src.ptr, dst.ptr, size, ctypes.addressof(ivb) if ivb else None)
        _check(st, what)
        return out

    def encrypt(self, input, output=None, size=None, iv=None):
        """CBC encrypt (cyr_rijndael.cpp:588-609); returns `output`."""
        return self._run("cyaes_cbc_encrypt", "Rijndael.encrypt", input, output, size, iv)

    def decrypt(self, input, output=None, size=None, iv=None):
        """CBC decrypt (cyr_rijndael.cpp:612-635); returns `output`."""
        return self._run("cyaes_cbc_decrypt", "Rijndael.decrypt", input, output, size, iv)


def _p(x):
    """Device pointer argument: int address, torch tensor, or None."""
    if x is None:
        return None
    if hasattr(x, "data_ptr"):
        return x.data_ptr()
    return int(x) or None


class GpuContext:
    """Device context (cyaes_gpu_*): key table + batched kernels.

    Buffer arguments are device pointers (ints) or torch tensors on the
    context's device; `stream` is a hipStream_t handle (int) or None."""

    def __init__(self, device=0, lib=None):
        self._lib = lib if lib is not None else load_library()
        h = _vp()
        _check(self._lib.cyaes_gpu_create(device, ctypes.byref(h)), "cyaes_gpu_create(%d)" % device)
        self._h = h
        self.device = device

    def close(self):
        if getattr(self, "_h", None):
            self._lib.cyaes_gpu_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def num_cus(self):
        return self._lib.cyaes_gpu_num_cus(self._h)

    @property
    def nkeys(self):
        return self._lib.cyaes_gpu_nkeys(self._h)

    def set_keys(self, keys):
        keys = bytes(keys)
        if not keys or len(keys) % 16:
            raise ValueError("keys must be a non-empty multiple of 16 bytes")
        buf = (ctypes.c_uint8 * len(keys)).from_buffer_copy(keys)
        _check(self._lib.cyaes_gpu_set_keys(self._h, ctypes.addressof(buf), len(keys) // 16), "set_keys")

    def set_keys_device(self, d_keys, nkeys, stream=None):
        _check(self._lib.cyaes_gpu_set_keys_device(self._h, _p(d_keys), nkeys, _p(stream)), "set_keys_device")

    def get_key(self, index):
        k = CyaesKey()
        _check(self._lib.cyaes_gpu_get_key(self._h, index, ctypes.byref(k)), "get_key")
        return k

    def encrypt_uniform(self, d_in, d_out, npayloads, payload_bytes, key_idx=None, payloads_per_key=0,
                        iv_in=None, iv_out=None, stream=None):
        _check(self._lib.cyaes_gpu_encrypt_uniform(self._h, _p(d_in), _p(d_out), npayloads, payload_bytes,
                                                   _p(key_idx), payloads_per_key, _p(iv_in), _p(iv_out),
                                                   _p(stream)), "encrypt_uniform")

    def decrypt_uniform(self, d_in, d_out, npayloads, payload_bytes, key_idx=None, payloads_per_key=0,
                        iv_in=None, iv_out=None, stream=None):
        _check(self._lib.cyaes_gpu_decrypt_uniform(self._h, _p(d_in), _p(d_out), npayloads, payload_bytes,
                                                   _p(key_idx), payloads_per_key, _p(iv_in), _p(iv_out),
                                                   _p(stream)), "decrypt_uniform")

    def encrypt_ragged(self, d_in, d_out, offsets, nbytes, npayloads, key_idx=None, payloads_per_key=0,
                       iv_in=None, iv_out=None, stream=None):
        _check(self._lib.cyaes_gpu_encrypt_ragged(self._h, _p(d_in), _p(d_out), _p(offsets), _p(nbytes), npayloads,
                                                  _p(key_idx), payloads_per_key, _p(iv_in), _p(iv_out),
                                                  _p(stream)), "encrypt_ragged")

    def decrypt_ragged(self, d_in, d_out, offsets, nbytes, npayloads, key_idx=None, payloads_per_key=0,
                       iv_in=None, iv_out=None, stream=None):
        _check(self._lib.cyaes_gpu_decrypt_ragged(self._h, _p(d_in), _p(d_out), _p(offsets), _p(nbytes), npayloads,
                                                  _p(key_idx), payloads_per_key, _p(iv_in), _p(iv_out),
                                                  _p(stream)), "decrypt_ragged")

    def check(self):
        """CYAES_OK, or CYAES_ERANGE if a batch clamped a key index (no raise)."""
        st = self._lib.cyaes_gpu_check(self._h)
        if st not in (CYAES_OK, CYAES_ERANGE):
            raise CyaesError(st, "check")
        return st

    def fill_synthetic(self, d_buf, p0, npayloads, payload_bytes, seed, stream=None):
        _check(self._lib.cyaes_gpu_fill_synthetic(_p(d_buf), p0, npayloads, payload_bytes, seed, _p(stream)),
               "fill_synthetic")

    def digest(self, d_buf, nbytes, stream=None):
        out = (ctypes.c_uint64 * 2)()
        _check(self._lib.cyaes_gpu_digest(_p(d_buf), nbytes, out, _p(stream)), "digest")
        return int(out[0]), int(out[1])
