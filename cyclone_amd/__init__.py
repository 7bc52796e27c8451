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
# CYAES_LIBRARY selects a build variant of the same library for a whole process
# (the bounds-checked build, `make bounds`: tests/conftest.py reads its record).
LIB_PATH = os.environ.get("CYAES_LIBRARY") or os.path.join(_HERE, "libcyaes.so")
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
    "cyaes_gpu_destroy": (ctypes.c_int, [_vp]),
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
    "cyaes_gpu_encrypt_strided": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                                 ctypes.c_uint32, _vp, ctypes.c_uint32, _vp]),
    "cyaes_gpu_decrypt_strided": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                                 ctypes.c_uint32, _vp, ctypes.c_uint32, _vp]),
    "cyaes_gpu_check": (ctypes.c_int, [_vp]),
    "cyaes_gpu_check_stream": (ctypes.c_int, [_vp, _vp]),
    "cyaes_gpu_encrypt_host": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                              ctypes.c_uint64]),
    "cyaes_gpu_decrypt_host": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                              ctypes.c_uint64]),
    "cyaes_gpu_fill_synthetic": (ctypes.c_int, [_vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                                                ctypes.c_uint64, _vp]),
    "cyaes_gpu_digest": (ctypes.c_int, [_vp, ctypes.c_uint64, _u64p, _vp]),
    "cyaes_gpu_update_keys": (ctypes.c_int, [_vp, ctypes.c_uint32, _vp, ctypes.c_uint32]),
    "cyaes_gpu_cbc_encrypt_batch": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, ctypes.c_uint32, _vp]),
    "cyaes_gpu_cbc_decrypt_batch": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, ctypes.c_uint32, _vp]),
    "cyaes_debug_pins": (ctypes.c_int, [_u64p]),
    "cyaes_debug_ctx": (ctypes.c_int, [_vp, _u64p]),
    "cyaes_debug_pin_history": (ctypes.c_uint64, [_u64p, ctypes.c_uint64, _u64p]),
    "cyaes_gpu_duplex_uniform": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                                _vp, _vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, _vp]),
    "cyaes_gpu_duplex_strided": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                                ctypes.c_uint32, ctypes.c_uint32, _vp, _vp, ctypes.c_uint64,
                                                ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                                _vp]),
    "cyaes_gpu_duplex_ragged": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, ctypes.c_uint64, ctypes.c_uint32, _vp, _vp,
                                               _vp, _vp, ctypes.c_uint64, ctypes.c_uint32, _vp]),
    # include/cyaes_relay.h
    "cyaes_relay_round16": (ctypes.c_uint32, [ctypes.c_uint32]),
    "cyaes_relay_packet_bytes": (ctypes.c_uint32, [ctypes.c_uint32]),
    "cyaes_relay_build_forward": (ctypes.c_uint32, [_vp, ctypes.c_int32, _vp, ctypes.c_uint32]),
    "cyaes_relay_parse": (ctypes.c_uint32, [_vp, ctypes.c_size_t, _vp, _vp, _vp, ctypes.c_uint32,
                                            ctypes.POINTER(ctypes.c_size_t)]),
    "cyaes_relay_payloads": (ctypes.c_int64, [_vp, _vp, _vp, ctypes.c_uint32, ctypes.c_uint64, _vp, _vp]),
    "cyaes_relay_stride": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, _vp, _vp, _vp]),
    "cyaes_relay_forward_id": (ctypes.c_int32, [_vp]),
    "cyaes_relay_forward_size": (ctypes.c_int32, [_vp]),
    # include/cyaes_adler32.h
    "cyaes_gpu_adler32_batch": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, ctypes.c_uint64, _vp]),
    "cyaes_gpu_adler32": (ctypes.c_int, [_vp, ctypes.c_uint64, ctypes.c_uint32, _u32p, _vp]),
    # include/cyaes_batch.h
    "cyaes_batcher_create": (ctypes.c_int, [_vp, ctypes.POINTER(_vp)]),
    "cyaes_batcher_destroy": (None, [_vp]),
    "cyaes_batcher_session_open": (ctypes.c_int, [_vp, _vp, _u32p]),
    "cyaes_batcher_session_close": (ctypes.c_int, [_vp, ctypes.c_uint32]),
    "cyaes_batcher_submit": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_uint32, _vp, _vp, ctypes.c_size_t, _vp,
                                            _vp]),
    "cyaes_batcher_submit_seal": (ctypes.c_int, [_vp, ctypes.c_uint32, ctypes.c_int32, _vp, ctypes.c_uint32, _vp,
                                                 _vp, _vp]),
    "cyaes_batcher_submit_open": (ctypes.c_int, [_vp, ctypes.c_uint32, _vp, ctypes.c_uint32, _vp, _vp]),
    "cyaes_batcher_submit_many": (ctypes.c_int, [_vp, _vp, ctypes.c_uint32, _vp]),
    "cyaes_batcher_flush": (ctypes.c_int, [_vp]),
    "cyaes_batcher_register_pool": (ctypes.c_int, [_vp, _vp, ctypes.c_size_t, _u32p]),
    "cyaes_batcher_unregister_pool": (ctypes.c_int, [_vp, ctypes.c_uint32]),
    "cyaes_batcher_submit_pooled": (ctypes.c_int, [_vp, _vp, ctypes.c_uint32, _vp]),
    "cyaes_batcher_poll": (ctypes.c_uint32, [_vp, _vp, _vp, ctypes.c_uint32]),
    "cyaes_batcher_stats": (ctypes.c_int, [_vp, _u64p]),
}

_lib = None


HEADERS = [os.path.join(os.path.dirname(_HERE), "include", h)
           for h in ("cyaes.h", "cyaes_relay.h", "cyaes_batch.h", "cyaes_adler32.h")]
MGPU_HEADER = os.path.join(os.path.dirname(_HERE), "include", "cyaes_mgpu.h")
MGPU_LIB_PATH = os.path.join(_HERE, "libcyaes_mgpu.so")


def header_functions(paths=None):
    """Names of the functions the C-ABI headers (include/cyaes*.h) declare."""
    names = set()
    for path in paths or HEADERS:
        text = re.sub(r"/\*.*?\*/", "", open(path).read(), flags=re.S)  # drop comments
        names |= set(re.findall(r"\b(cyaes_[a-z0-9_]+)\s*\(", text))
    return sorted(names)


def load_library(path=LIB_PATH):
    """Loads libcyaes.so (fails loudly; there is no fallback path)."""
    global _lib
    if _lib is not None and path == LIB_PATH:
        return _lib
    if not os.path.exists(path):
        raise ImportError("cyclone_amd: %s is not built (run `make` or __graft_entry__.build())" % path)
    # PyTorch-ROCm bundles its own libamdhip64 (soname libamdhip64.so.7, like
    # /opt/rocm's).  Loaded first, it satisfies libcyaes.so's dependency and the
    # process has one HIP runtime; loaded after ours, torch would map a second
    # runtime and find no GPU.  So let torch (if present) load first.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
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


PIN_FIELDS = ("live", "live_bytes", "registered", "unregistered", "failed_unregisters", "stale", "conflicts",
              "refs")


def debug_pins():
    """The library's host-memory registrations (cyaes_debug_pins, include/cyaes.h)."""
    out = (ctypes.c_uint64 * 8)()
    _check(load_library().cyaes_debug_pins(out), "cyaes_debug_pins")
    return dict(zip(PIN_FIELDS, (int(v) for v in out)))


def debug_pin_history(cap=1024):
    """(ranges, outlived): the [lo, hi) host ranges the library unregistered,
    most recent first, and how many unregisters found their memory already
    unmapped (cyaes_debug_pin_history, include/cyaes.h)."""
    out = (ctypes.c_uint64 * (2 * cap))()
    outlived = ctypes.c_uint64(0)
    n = load_library().cyaes_debug_pin_history(out, cap, ctypes.byref(outlived))
    return [(int(out[2 * i]), int(out[2 * i + 1])) for i in range(n)], int(outlived.value)


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
            if self.n == 0:
                self.arr = (ctypes.c_uint8 * 1)()  # never dereferenced for size 0
            elif mv.readonly:
                self.arr = (ctypes.c_uint8 * self.n).from_buffer_copy(mv.tobytes())
            else:
                self.arr = (ctypes.c_uint8 * self.n).from_buffer(mv)
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
        """Frees the context; raises CyaesError if the device reports a pending
        asynchronous fault (cyaes_gpu_destroy's synchronisation status)."""
        if getattr(self, "_h", None):
            h, self._h = self._h, None
            _check(self._lib.cyaes_gpu_destroy(h), "cyaes_gpu_destroy")

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

    def update_keys(self, first, keys):
        """Replaces / appends rows [first, first + len(keys) / 16) (cyaes_gpu_update_keys)."""
        keys = bytes(keys)
        if not keys or len(keys) % 16:
            raise ValueError("keys must be a non-empty multiple of 16 bytes")
        buf = (ctypes.c_uint8 * len(keys)).from_buffer_copy(keys)
        _check(self._lib.cyaes_gpu_update_keys(self._h, first, ctypes.addressof(buf), len(keys) // 16), "update_keys")

    def debug_state(self):
        """cyaes_debug_ctx: key-table readers in flight, scratch blocks / bytes, outgrown tables."""
        out = (ctypes.c_uint64 * 4)()
        _check(self._lib.cyaes_debug_ctx(self._h, out), "cyaes_debug_ctx")
        return dict(zip(("key_uses", "scratch_blocks", "scratch_bytes", "retired_tables"), (int(v) for v in out)))

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

    def duplex_uniform(self, enc_in, enc_out, enc_npayloads, enc_payload_bytes, dec_in, dec_out, dec_npayloads,
                       dec_payload_bytes, enc_key=0, dec_key=0, stream=None):
        """Encrypt one uniform batch and decrypt another in one launch (cyaes_gpu_duplex_uniform)."""
        _check(self._lib.cyaes_gpu_duplex_uniform(self._h, _p(enc_in), _p(enc_out), enc_npayloads, enc_payload_bytes,
                                                  enc_key, _p(dec_in), _p(dec_out), dec_npayloads, dec_payload_bytes,
                                                  dec_key, _p(stream)), "duplex_uniform")

    def duplex_ragged(self, enc_in, enc_out, enc_offsets, enc_nbytes, enc_npayloads, dec_in, dec_out, dec_offsets,
                      dec_nbytes, dec_npayloads, enc_key=0, dec_key=0, stream=None):
        """Encrypt one ragged relay stream and decrypt another (cyaes_gpu_duplex_ragged)."""
        _check(self._lib.cyaes_gpu_duplex_ragged(self._h, _p(enc_in), _p(enc_out), _p(enc_offsets), _p(enc_nbytes),
                                                 enc_npayloads, enc_key, _p(dec_in), _p(dec_out), _p(dec_offsets),
                                                 _p(dec_nbytes), dec_npayloads, dec_key, _p(stream)), "duplex_ragged")

    def duplex_strided(self, enc_in, enc_out, enc_first, enc_stride, enc_npayloads, enc_payload_bytes, dec_in, dec_out,
                       dec_first, dec_stride, dec_npayloads, dec_payload_bytes, enc_key=0, dec_key=0, stream=None):
        """Encrypt one relay stream and decrypt another in one launch (cyaes_gpu_duplex_strided)."""
        _check(self._lib.cyaes_gpu_duplex_strided(self._h, _p(enc_in), _p(enc_out), enc_first, enc_stride,
                                                  enc_npayloads, enc_payload_bytes, enc_key, _p(dec_in), _p(dec_out),
                                                  dec_first, dec_stride, dec_npayloads, dec_payload_bytes, dec_key,
                                                  _p(stream)), "duplex_strided")

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

    def encrypt_strided(self, d_in, d_out, first_offset, stride, npayloads, payload_bytes, key_idx=None,
                        payloads_per_key=0, stream=None):
        """Payload p at byte first_offset + p * stride (cyaes_gpu_encrypt_strided)."""
        _check(self._lib.cyaes_gpu_encrypt_strided(self._h, _p(d_in), _p(d_out), first_offset, stride, npayloads,
                                                   payload_bytes, _p(key_idx), payloads_per_key, _p(stream)),
               "encrypt_strided")

    def decrypt_strided(self, d_in, d_out, first_offset, stride, npayloads, payload_bytes, key_idx=None,
                        payloads_per_key=0, stream=None):
        """Payload p at byte first_offset + p * stride (cyaes_gpu_decrypt_strided)."""
        _check(self._lib.cyaes_gpu_decrypt_strided(self._h, _p(d_in), _p(d_out), first_offset, stride, npayloads,
                                                   payload_bytes, _p(key_idx), payloads_per_key, _p(stream)),
               "decrypt_strided")

    def encrypt_host(self, h_in, h_out, npayloads, payload_bytes, payloads_per_key=0, chunk_bytes=0):
        """Host-resident batch (host addresses or CPU tensors), PCIe-inclusive; synchronous."""
        _check(self._lib.cyaes_gpu_encrypt_host(self._h, _p(h_in), _p(h_out), npayloads, payload_bytes,
                                                payloads_per_key, chunk_bytes), "encrypt_host")

    def decrypt_host(self, h_in, h_out, npayloads, payload_bytes, payloads_per_key=0, chunk_bytes=0):
        _check(self._lib.cyaes_gpu_decrypt_host(self._h, _p(h_in), _p(h_out), npayloads, payload_bytes,
                                                payloads_per_key, chunk_bytes), "decrypt_host")

    def check(self):
        """CYAES_OK, or CYAES_ERANGE if a batch clamped a key index (no raise).
        Synchronises the whole device (cyaes_gpu_check)."""
        st = self._lib.cyaes_gpu_check(self._h)
        if st not in (CYAES_OK, CYAES_ERANGE):
            raise CyaesError(st, "check")
        return st

    def check_stream(self, stream=None):
        """As check(), waiting for `stream` only (cyaes_gpu_check_stream)."""
        st = self._lib.cyaes_gpu_check_stream(self._h, _p(stream))
        if st not in (CYAES_OK, CYAES_ERANGE):
            raise CyaesError(st, "check_stream")
        return st

    def fill_synthetic(self, d_buf, p0, npayloads, payload_bytes, seed, stream=None):
        _check(self._lib.cyaes_gpu_fill_synthetic(_p(d_buf), p0, npayloads, payload_bytes, seed, _p(stream)),
               "fill_synthetic")

    def digest(self, d_buf, nbytes, stream=None):
        out = (ctypes.c_uint64 * 2)()
        _check(self._lib.cyaes_gpu_digest(_p(d_buf), nbytes, out, _p(stream)), "digest")
        return int(out[0]), int(out[1])


# ---- relay wire format (include/cyaes_relay.h) ------------------------------
RELAY_HEADSIZE, RELAY_FORWARD, RELAY_PAYLOAD_OFFSET, RELAY_MAX_CHUNK, RELAY_PAD = 4, 103, 12, 0xFF00, 0xCE


def relay_packet_bytes(msg_size):
    return load_library().cyaes_relay_packet_bytes(msg_size)


def relay_build_forward(conn_id, payload):
    """Plaintext RELAY_FORWARD packet (relay_local.cpp:189-201) as bytes."""
    payload = bytes(payload)
    lib = load_library()
    out = (ctypes.c_uint8 * lib.cyaes_relay_packet_bytes(len(payload)))()
    src = (ctypes.c_uint8 * max(1, len(payload))).from_buffer_copy(payload or b"\0")
    n = lib.cyaes_relay_build_forward(out, conn_id, src if payload else None, len(payload))
    if n == 0:
        raise ValueError("chunk larger than RELAY_MAX_CHUNK")
    return bytes(out)[:n]


def relay_parse(stream, max_packets=1 << 20):
    """[(offset, packet_size, packet_id)], consumed bytes (cye_packet.cpp:166-181)."""
    stream = bytes(stream)
    lib = load_library()
    cap = min(max_packets, len(stream) // RELAY_HEADSIZE + 1)
    off = (ctypes.c_uint64 * cap)()
    sz = (ctypes.c_uint32 * cap)()
    ids = (ctypes.c_uint16 * cap)()
    used = ctypes.c_size_t()
    buf = (ctypes.c_uint8 * max(1, len(stream))).from_buffer_copy(stream or b"\0")
    n = lib.cyaes_relay_parse(buf, len(stream), off, sz, ids, cap, ctypes.byref(used))
    return [(off[i], sz[i], ids[i]) for i in range(n)], used.value


def relay_payloads(packets, base=0):
    """(payload offsets, payload sizes) of the RELAY_FORWARD packets of a parsed stream."""
    lib = load_library()
    n = len(packets)
    off = (ctypes.c_uint64 * max(1, n))(*[p[0] for p in packets])
    sz = (ctypes.c_uint32 * max(1, n))(*[p[1] for p in packets])
    ids = (ctypes.c_uint16 * max(1, n))(*[p[2] for p in packets])
    po = (ctypes.c_uint64 * max(1, n))()
    pl = (ctypes.c_uint32 * max(1, n))()
    j = lib.cyaes_relay_payloads(off, sz, ids, n, base, po, pl)
    if j < 0:
        raise ValueError("RELAY_FORWARD packet with a payload that is not a multiple of 16")
    return list(po[:j]), list(pl[:j])


def relay_stride(pay_off, pay_len):
    """(first, stride, payload_bytes) if the payloads are equally strided and sized
    (cyaes_relay_stride; for cyaes_gpu_*_strided), else None."""
    lib = load_library()
    n = len(pay_off)
    off = (ctypes.c_uint64 * max(1, n))(*pay_off)
    ln = (ctypes.c_uint32 * max(1, n))(*pay_len)
    first, stride, pb = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint32()
    if not lib.cyaes_relay_stride(off, ln, n, ctypes.byref(first), ctypes.byref(stride), ctypes.byref(pb)):
        return None
    return first.value, stride.value, pb.value


# ---- asynchronous batching adapter (include/cyaes_batch.h) ------------------
OP_ENCRYPT, OP_DECRYPT, OP_RELAY_SEAL, OP_RELAY_OPEN = 0, 1, 2, 3
_DONE_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_int)


class BatchReq(ctypes.Structure):
    """struct cyaes_batch_req (cyaes_batcher_submit_many)."""

    _fields_ = [("op", ctypes.c_int), ("slot", ctypes.c_uint32), ("conn_id", ctypes.c_int32), ("inp", _vp),
                ("out", _vp), ("size", ctypes.c_uint32), ("done", _DONE_FN), ("user", _vp)]


class PoolReq(ctypes.Structure):
    """struct cyaes_pool_req (cyaes_batcher_submit_pooled)."""

    _fields_ = [("op", ctypes.c_int), ("slot", ctypes.c_uint32), ("conn_id", ctypes.c_int32), ("pool", ctypes.c_uint32),
                ("in_off", ctypes.c_uint64), ("out_off", ctypes.c_uint64), ("size", ctypes.c_uint32),
                ("done", _DONE_FN), ("user", _vp)]


class BatcherConfig(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int), ("max_batch_bytes", ctypes.c_uint32),
                ("max_delay_us", ctypes.c_uint32), ("inflight", ctypes.c_uint32), ("workers", ctypes.c_uint32),
                ("max_sessions", ctypes.c_uint32), ("flags", ctypes.c_uint32)]


BATCHER_POLL = 1


class Batcher:
    """cyaes_batcher: requests from any thread are coalesced into GPU batches.

    Buffers are host buffers (bytearray / writable memoryview); they are kept
    alive by the batcher until the request completes.  `done(status)` runs on
    the batcher's completion thread."""

    def __init__(self, device=0, max_batch_bytes=0, max_delay_us=0, inflight=0, workers=0, max_sessions=0,
                 poll=False, lib=None):
        """poll=True: CYAES_BATCHER_POLL -- requests complete into the submitting
        thread's queue (read with poll()); their `done` value is returned there
        as a tag instead of being called."""
        self._lib = lib if lib is not None else load_library()
        self._poll = bool(poll)
        cfg = BatcherConfig(device, max_batch_bytes, max_delay_us, inflight, workers, max_sessions,
                            BATCHER_POLL if poll else 0)
        h = _vp()
        _check(self._lib.cyaes_batcher_create(ctypes.byref(cfg), ctypes.byref(h)), "cyaes_batcher_create")
        self._h = h
        self._live = {}
        self._next = 1
        self._mu = __import__("threading").Lock()
        self._cb = _DONE_FN(self._on_done)

    def close(self):
        if getattr(self, "_h", None):
            self._lib.cyaes_batcher_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _on_done(self, user, status):
        with self._mu:
            bufs, done = self._live.pop(user)
        if done is not None:
            done(status)

    def _cbp(self):
        return _DONE_FN() if self._poll else self._cb  # (a NULL function pointer in poll mode)

    def poll(self, max_n=65536):
        """Poll mode: [(tag, status)] of this thread's completed requests, oldest first."""
        users = (_vp * max_n)()
        sts = (ctypes.c_int * max_n)()
        n = self._lib.cyaes_batcher_poll(self._h, users, sts, max_n)
        out = []
        with self._mu:
            for i in range(n):
                _, tag = self._live.pop(users[i])
                out.append((tag, int(sts[i])))
        return out

    def _track(self, bufs, done):
        with self._mu:
            token = self._next
            self._next += 1
            self._live[token] = (bufs, done)
        return token

    def _untrack(self, token):
        with self._mu:
            self._live.pop(token, None)

    def session_open(self, key):
        key = bytes(key)
        if len(key) != 16:
            raise ValueError("AES-128 key must be 16 bytes")
        slot = ctypes.c_uint32()
        _check(self._lib.cyaes_batcher_session_open(self._h, (ctypes.c_uint8 * 16).from_buffer_copy(key),
                                                    ctypes.byref(slot)), "session_open")
        return slot.value

    def session_close(self, slot):
        _check(self._lib.cyaes_batcher_session_close(self._h, slot), "session_close")

    def submit(self, op, slot, inp, out, size=None, done=None):
        src = _Buf(inp, False)
        dst = src if out is inp else _Buf(out, True)
        size = src.n if size is None else size
        if size > src.n or size > dst.n:
            raise ValueError("size exceeds buffer")
        token = self._track((src, dst), done)
        st = self._lib.cyaes_batcher_submit(self._h, op, slot, src.ptr, dst.ptr, size, self._cbp(), token)
        if st:
            self._untrack(token)
            raise CyaesError(st, "submit")

    def submit_seal(self, slot, conn_id, payload, packet_out, done=None):
        src = _Buf(payload, False)
        dst = _Buf(packet_out, True)
        if dst.n < relay_packet_bytes(src.n):
            raise ValueError("packet_out too small")
        token = self._track((src, dst), done)
        st = self._lib.cyaes_batcher_submit_seal(self._h, slot, conn_id, src.ptr, src.n, dst.ptr, self._cbp(), token)
        if st:
            self._untrack(token)
            raise CyaesError(st, "submit_seal")

    def submit_open(self, slot, packet, done=None):
        buf = _Buf(packet, True)
        token = self._track((buf,), done)
        st = self._lib.cyaes_batcher_submit_open(self._h, slot, buf.ptr, buf.n, self._cbp(), token)
        if st:
            self._untrack(token)
            raise CyaesError(st, "submit_open")

    def submit_many(self, reqs):
        """reqs: [(op, slot, inp, out, size_or_None, done, conn_id)] in one call
        (cyaes_batcher_submit_many).  Returns the per-request status list; a
        request with a non-zero status was not accepted (its done never runs)."""
        n = len(reqs)
        arr = (BatchReq * max(1, n))()
        tokens = []
        for i, (op, slot, inp, out, size, done, conn) in enumerate(reqs):
            if op == OP_RELAY_OPEN:
                src = dst = _Buf(out if out is not None else inp, True)
            else:
                src = _Buf(inp, False)
                dst = src if out is inp else _Buf(out, True)
            if size is None:
                size = src.n
            # native code copies `size` bytes from/to these buffers: bound it as submit() does
            if op == OP_RELAY_SEAL:
                bad = size > src.n or relay_packet_bytes(size) > dst.n
            else:
                bad = size > src.n or size > dst.n
            if bad:
                for t in tokens:
                    self._untrack(t)
                raise ValueError("request %d: size exceeds its buffer" % i)
            token = self._track((src, dst), done)
            tokens.append(token)
            arr[i] = BatchReq(op, slot, conn or 0, src.ptr, dst.ptr, size, self._cbp(), token)
        st = (ctypes.c_int * max(1, n))()
        self._lib.cyaes_batcher_submit_many(self._h, arr, n, st)
        for i, token in enumerate(tokens):
            if st[i]:
                self._untrack(token)
        return [int(st[i]) for i in range(n)]

    def register_pool(self, buf):
        """Registers a writable host buffer (bytearray, numpy array, ...) as a
        zero-copy packet pool; returns its id.  The buffer is kept alive until
        unregister_pool."""
        b = _Buf(buf, True)
        pool = ctypes.c_uint32()
        _check(self._lib.cyaes_batcher_register_pool(self._h, b.ptr, b.n, ctypes.byref(pool)), "register_pool")
        self._pools = getattr(self, "_pools", {})
        self._pools[pool.value] = b
        return pool.value

    def unregister_pool(self, pool):
        _check(self._lib.cyaes_batcher_unregister_pool(self._h, pool), "unregister_pool")
        getattr(self, "_pools", {}).pop(pool, None)

    def submit_pooled(self, reqs):
        """reqs: [(op, slot, pool, in_off, out_off, size, done, conn_id)] by pool
        offsets (cyaes_batcher_submit_pooled); returns the per-request status list."""
        n = len(reqs)
        arr = (PoolReq * max(1, n))()
        tokens = []
        for i, (op, slot, pool, in_off, out_off, size, done, conn) in enumerate(reqs):
            token = self._track((), done)
            tokens.append(token)
            arr[i] = PoolReq(op, slot, conn or 0, pool, in_off, out_off or 0, size, self._cbp(), token)
        st = (ctypes.c_int * max(1, n))()
        self._lib.cyaes_batcher_submit_pooled(self._h, arr, n, st)
        for i, token in enumerate(tokens):
            if st[i]:
                self._untrack(token)
        return [int(st[i]) for i in range(n)]

    def flush(self):
        """Waits for every request submitted so far; returns the first error status (0 = none)."""
        return self._lib.cyaes_batcher_flush(self._h)

    def stats(self):
        out = (ctypes.c_uint64 * 6)()
        _check(self._lib.cyaes_batcher_stats(self._h, out), "stats")
        keys = ("completed", "batches", "bytes", "max_batch", "errors", "pending")
        return dict(zip(keys, (int(v) for v in out)))


# ---- single-process multi-GPU (include/cyaes_mgpu.h, libcyaes_mgpu.so) -----
_MGPU_SIGS = {
    "cyaes_mgpu_create": (ctypes.c_int, [ctypes.c_int, _vp, ctypes.POINTER(_vp)]),
    "cyaes_mgpu_destroy": (ctypes.c_int, [_vp]),
    "cyaes_mgpu_ndev": (ctypes.c_int, [_vp]),
    "cyaes_mgpu_context": (_vp, [_vp, ctypes.c_int]),
    "cyaes_mgpu_broadcast_keys": (ctypes.c_int, [_vp, _vp, ctypes.c_uint32, ctypes.c_int]),
    "cyaes_mgpu_shard": (ctypes.c_int, [ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_uint64, _u64p, _u64p]),
    "cyaes_mgpu_encrypt_uniform": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, ctypes.c_uint32, ctypes.c_uint32]),
    "cyaes_mgpu_decrypt_uniform": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, ctypes.c_uint32, ctypes.c_uint32]),
}
_mgpu_lib = None


def load_mgpu_library(path=MGPU_LIB_PATH):
    """Loads libcyaes_mgpu.so (RCCL); fails loudly if it is not built."""
    global _mgpu_lib
    if _mgpu_lib is not None:
        return _mgpu_lib
    load_library()  # torch first, then libcyaes.so (see load_library)
    if not os.path.exists(path):
        raise ImportError("cyclone_amd: %s is not built (run `make`)" % path)
    lib = ctypes.CDLL(path)
    for name, (res, args) in _MGPU_SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _mgpu_lib = lib
    return lib


def mgpu_shard(total, ndev, i, align=1):
    first, count = ctypes.c_uint64(), ctypes.c_uint64()
    _check(load_mgpu_library().cyaes_mgpu_shard(total, ndev, i, align, ctypes.byref(first), ctypes.byref(count)),
           "cyaes_mgpu_shard")
    return first.value, count.value


class MultiGpu:
    """cyaes_mgpu: one context per device + an RCCL clique for key broadcast."""

    def __init__(self, devices):
        self._lib = load_mgpu_library()
        devs = (ctypes.c_int * len(devices))(*devices)
        h = _vp()
        _check(self._lib.cyaes_mgpu_create(len(devices), devs, ctypes.byref(h)), "cyaes_mgpu_create")
        self._h = h
        self.devices = list(devices)

    def close(self):
        if getattr(self, "_h", None):
            h, self._h = self._h, None
            _check(self._lib.cyaes_mgpu_destroy(h), "cyaes_mgpu_destroy")

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def ndev(self):
        return self._lib.cyaes_mgpu_ndev(self._h)

    def broadcast_keys(self, keys, root=0):
        keys = bytes(keys)
        buf = (ctypes.c_uint8 * len(keys)).from_buffer_copy(keys)
        _check(self._lib.cyaes_mgpu_broadcast_keys(self._h, buf, len(keys) // 16, root), "broadcast_keys")

    def _run(self, fn, d_in, d_out, npayloads, first, payload_bytes, ppk):
        n = len(self.devices)
        ins = (_vp * n)(*[_p(x) for x in d_in])
        outs = (_vp * n)(*[_p(x) for x in d_out])
        cnt = (ctypes.c_uint64 * n)(*npayloads)
        fst = (ctypes.c_uint64 * n)(*(first or [0] * n))
        _check(fn(self._h, ins, outs, cnt, fst, payload_bytes, ppk), fn.__name__)

    def encrypt_uniform(self, d_in, d_out, npayloads, first, payload_bytes, payloads_per_key=0):
        self._run(self._lib.cyaes_mgpu_encrypt_uniform, d_in, d_out, npayloads, first, payload_bytes,
                  payloads_per_key)

    def decrypt_uniform(self, d_in, d_out, npayloads, first, payload_bytes, payloads_per_key=0):
        self._run(self._lib.cyaes_mgpu_decrypt_uniform, d_in, d_out, npayloads, first, payload_bytes,
                  payloads_per_key)
