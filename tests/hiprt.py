"""The HIP runtime the test process runs on (torch's, which libcyaes.so shares),
through ctypes: raw streams, and the tests' own host registrations.

Every hipHostRegister a test makes goes through `host_register` /
`host_unregister`, which keep the session's history of registered ranges, so
tests/conftest.py can check after every GPU test that the runtime no longer
answers for any of them.  Host-side
queries only: nothing here hands the GPU an address.
"""
import ctypes
import errno
import os

_rt = None
_libc = None

# [lo, hi) of every range a test registered this session, and how many of
# them were found unmapped when unregistered (a registration that outlived
# its memory).
HISTORY = []
LIVE = {}
OUTLIVED = [0]

PAGE = 4096


def runtime():
    """torch's libamdhip64 (already loaded by `import torch`: the same handle)."""
    global _rt
    if _rt is None:
        import torch
        path = os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so")
        rt = ctypes.CDLL(path if os.path.exists(path) else "libamdhip64.so")
        vp = ctypes.c_void_p
        rt.hipHostRegister.argtypes = [vp, ctypes.c_size_t, ctypes.c_uint]
        rt.hipHostUnregister.argtypes = [vp]
        rt.hipMemGetAddressRange.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(ctypes.c_size_t), vp]
        rt.hipStreamCreateWithFlags.argtypes = [ctypes.POINTER(vp), ctypes.c_uint]
        rt.hipStreamDestroy.argtypes = [vp]
        rt.hipStreamSynchronize.argtypes = [vp]
        rt.hipGetLastError.argtypes = []
        rt.hipHostMalloc.argtypes = [ctypes.POINTER(vp), ctypes.c_size_t, ctypes.c_uint]
        rt.hipHostFree.argtypes = [vp]
        _rt = rt
    return _rt


def _mapped(lo, hi):
    """Every page of [lo, hi) mapped (msync answers ENOMEM otherwise)."""
    global _libc
    if _libc is None:
        _libc = ctypes.CDLL(None, use_errno=True)
        _libc.msync.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    plo = lo & ~(PAGE - 1)
    phi = (hi + PAGE - 1) & ~(PAGE - 1)
    if _libc.msync(plo, phi - plo, 1) == 0:  # MS_ASYNC
        return True
    return ctypes.get_errno() != errno.ENOMEM


def host_register(ptr, nbytes, flags=0):
    """hipHostRegister(ptr, nbytes, flags), recorded in the session history."""
    st = int(runtime().hipHostRegister(ptr, nbytes, flags))
    if st == 0:
        HISTORY.append((ptr, ptr + nbytes))
        LIVE[ptr] = ptr + nbytes
    else:
        runtime().hipGetLastError()
    return st


def host_unregister(ptr):
    hi = LIVE.pop(ptr, None)
    if hi is not None and not _mapped(ptr, hi):
        OUTLIVED[0] += 1
    st = int(runtime().hipHostUnregister(ptr))
    if st:
        runtime().hipGetLastError()
    return st


def answers_for(lo, hi):
    """The runtime still holds a host record for exactly [lo, hi): the stale
    state tools/hostreg_stale_probe.hip showed (a record that answers for new
    memory at the same address).  A later, different allocation that happens to
    cover the address (torch pinned memory) has another base or size."""
    rt = runtime()
    base, size = ctypes.c_void_p(), ctypes.c_size_t()
    st = int(rt.hipMemGetAddressRange(ctypes.byref(base), ctypes.byref(size), lo))
    if st:
        rt.hipGetLastError()
        return False
    plo, phi = lo & ~(PAGE - 1), (hi + PAGE - 1) & ~(PAGE - 1)
    return ((base.value or 0), size.value) in ((lo, hi - lo), (plo, phi - plo))


def host_malloc(nbytes):
    """hipHostMalloc (pinned, mapped): an allocation of exactly nbytes as the runtime records it."""
    p = ctypes.c_void_p()
    st = int(runtime().hipHostMalloc(ctypes.byref(p), nbytes, 0))
    assert st == 0, "hipHostMalloc: %d" % st
    return p.value


def host_free(p):
    assert int(runtime().hipHostFree(p)) == 0


def stream_create(nonblocking=True):
    s = ctypes.c_void_p()
    st = int(runtime().hipStreamCreateWithFlags(ctypes.byref(s), 1 if nonblocking else 0))
    assert st == 0, "hipStreamCreateWithFlags: %d" % st
    return s.value


def stream_destroy(s):
    assert int(runtime().hipStreamDestroy(s)) == 0


def stream_sync(s):
    assert int(runtime().hipStreamSynchronize(s)) == 0
