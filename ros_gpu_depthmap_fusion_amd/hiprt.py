"""Minimal ctypes access to the HIP runtime for device buffers and events (bench/test plumbing).

Loads the runtime by its SONAME (libamdhip64.so.7) so that, when torch is imported too, the
process keeps ONE HIP runtime (torch's bundled copy or /opt/rocm's, whichever loaded first).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

_hip = None
H2D, D2H, D2D = 1, 2, 3


def hip():
    global _hip
    if _hip is None:
        _hip = C.CDLL("libamdhip64.so.7", mode=C.RTLD_GLOBAL)
        _hip.hipGetErrorString.restype = C.c_char_p
        _hip.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
        _hip.hipFree.argtypes = [C.c_void_p]
        _hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
        _hip.hipMemcpyAsync.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
        _hip.hipMemset.argtypes = [C.c_void_p, C.c_int, C.c_size_t]
        _hip.hipSetDevice.argtypes = [C.c_int]
        _hip.hipEventCreate.argtypes = [C.POINTER(C.c_void_p)]
        _hip.hipEventRecord.argtypes = [C.c_void_p, C.c_void_p]
        _hip.hipEventSynchronize.argtypes = [C.c_void_p]
        _hip.hipEventElapsedTime.argtypes = [C.POINTER(C.c_float), C.c_void_p, C.c_void_p]
        _hip.hipEventDestroy.argtypes = [C.c_void_p]
        _hip.hipHostMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
        _hip.hipHostFree.argtypes = [C.c_void_p]
    return _hip


def check(rc: int, what: str = "hip"):
    if rc != 0:
        raise RuntimeError(f"{what} failed: {hip().hipGetErrorString(rc).decode()} ({rc})")


def device_count() -> int:
    n = C.c_int(0)
    rc = hip().hipGetDeviceCount(C.byref(n))
    return n.value if rc == 0 else 0


def set_device(d: int):
    check(hip().hipSetDevice(d), "hipSetDevice")


def copy_async(dst: int, src: int, nbytes: int, kind: int, stream: int):
    """hipMemcpyAsync on `stream` (ordered with the engine / torch work of that stream)."""
    check(hip().hipMemcpyAsync(C.c_void_p(dst), C.c_void_p(src), int(nbytes), kind,
                               C.c_void_p(stream)), "hipMemcpyAsync")


def synchronize():
    check(hip().hipDeviceSynchronize(), "hipDeviceSynchronize")


class DeviceArray:
    """A hipMalloc'ed buffer (freed on close/del)."""

    def __init__(self, nbytes: int):
        p = C.c_void_p()
        check(hip().hipMalloc(C.byref(p), max(int(nbytes), 1)), "hipMalloc")
        self.ptr = p.value
        self.nbytes = int(nbytes)

    @classmethod
    def from_numpy(cls, a: np.ndarray) -> "DeviceArray":
        a = np.ascontiguousarray(a)
        d = cls(a.nbytes)
        check(hip().hipMemcpy(C.c_void_p(d.ptr), a.ctypes.data_as(C.c_void_p), a.nbytes, H2D),
              "hipMemcpy H2D")
        return d

    def to_numpy(self, dtype, count) -> np.ndarray:
        out = np.empty(count, dtype)
        check(hip().hipMemcpy(out.ctypes.data_as(C.c_void_p), C.c_void_p(self.ptr), out.nbytes, D2H),
              "hipMemcpy D2H")
        return out

    def close(self):
        if self.ptr:
            hip().hipFree(C.c_void_p(self.ptr))
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class PinnedArray:
    """Page-locked host memory (hipHostMalloc) holding a copy of a numpy array: a sensor driver's
    DMA-able frame buffer.  `.ptr` is the host address, `.array` a numpy view of it."""

    def __init__(self, nbytes: int):
        p = C.c_void_p()
        check(hip().hipHostMalloc(C.byref(p), max(int(nbytes), 1), 0), "hipHostMalloc")
        self.ptr = p.value
        self.nbytes = int(nbytes)
        self.array = None

    @classmethod
    def from_numpy(cls, a: np.ndarray) -> "PinnedArray":
        a = np.ascontiguousarray(a)
        h = cls(a.nbytes)
        buf = (C.c_char * a.nbytes).from_address(h.ptr)
        h.array = np.frombuffer(buf, dtype=a.dtype).reshape(a.shape)
        h.array[...] = a
        return h

    def close(self):
        if self.ptr:
            self.array = None
            hip().hipHostFree(C.c_void_p(self.ptr))
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
