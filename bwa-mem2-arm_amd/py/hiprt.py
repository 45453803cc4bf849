"""Minimal ctypes binding of the HIP runtime C API (device buffers for bench / tests).

libbsw_hip.so is linked against libamdhip64.so.7; loading that runtime here, before any
`import torch`, makes the whole process share ONE HIP runtime instance (torch's bundled
copy has the same SONAME and is then not loaded a second time).  Only plain device
buffers, copies and synchronisation are needed, so nothing else is bound.
"""

from __future__ import annotations

import ctypes
import os

import numpy as np

_rt = None
H2D, D2H, D2D = 1, 2, 3


def rt():
    global _rt
    if _rt is None:
        for name in ("libamdhip64.so.7", "/opt/rocm/lib/libamdhip64.so.7", "libamdhip64.so"):
            try:
                _rt = ctypes.CDLL(name, mode=ctypes.RTLD_GLOBAL)
                break
            except OSError:
                continue
        if _rt is None:
            raise RuntimeError("HIP runtime (libamdhip64.so.7) not found")
        P = ctypes.c_void_p
        _rt.hipMalloc.argtypes = [ctypes.POINTER(P), ctypes.c_size_t]
        _rt.hipFree.argtypes = [P]
        _rt.hipMemcpy.argtypes = [P, P, ctypes.c_size_t, ctypes.c_int]
        _rt.hipMemset.argtypes = [P, ctypes.c_int, ctypes.c_size_t]
        _rt.hipSetDevice.argtypes = [ctypes.c_int]
        _rt.hipGetDeviceCount.argtypes = [ctypes.POINTER(ctypes.c_int)]
        _rt.hipGetErrorString.restype = ctypes.c_char_p
        _rt.hipGetErrorString.argtypes = [ctypes.c_int]
        _rt.hipMemGetInfo.argtypes = [ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_size_t)]
    return _rt


def check(rc):
    if rc != 0:
        raise RuntimeError(f"HIP error {rc}: {rt().hipGetErrorString(rc).decode()}")


def device_count() -> int:
    n = ctypes.c_int(0)
    rc = rt().hipGetDeviceCount(ctypes.byref(n))
    return n.value if rc == 0 else 0


def set_device(d: int):
    check(rt().hipSetDevice(d))


def mem_get_info() -> tuple:
    """(free, total) bytes of the current device (hipMemGetInfo)"""
    f, t = ctypes.c_size_t(0), ctypes.c_size_t(0)
    check(rt().hipMemGetInfo(ctypes.byref(f), ctypes.byref(t)))
    return int(f.value), int(t.value)


def synchronize():
    check(rt().hipDeviceSynchronize())


class DeviceBuffer:
    """Owned device allocation; .ptr is the raw device address."""

    def __init__(self, nbytes: int):
        self.nbytes = max(int(nbytes), 1)
        p = ctypes.c_void_p()
        check(rt().hipMalloc(ctypes.byref(p), self.nbytes))
        self.ptr = p.value

    @classmethod
    def from_array(cls, a: np.ndarray) -> "DeviceBuffer":
        a = np.ascontiguousarray(a)
        b = cls(a.nbytes)
        if a.nbytes:
            check(rt().hipMemcpy(ctypes.c_void_p(b.ptr), ctypes.c_void_p(a.ctypes.data), a.nbytes, H2D))
        return b

    def upload(self, a: np.ndarray):
        a = np.ascontiguousarray(a)
        assert a.nbytes <= self.nbytes
        check(rt().hipMemcpy(ctypes.c_void_p(self.ptr), ctypes.c_void_p(a.ctypes.data), a.nbytes, H2D))

    def download(self, out: np.ndarray) -> np.ndarray:
        assert out.flags.c_contiguous and out.nbytes <= self.nbytes
        check(rt().hipMemcpy(ctypes.c_void_p(out.ctypes.data), ctypes.c_void_p(self.ptr), out.nbytes, D2H))
        return out

    def free(self):
        if self.ptr:
            rt().hipFree(ctypes.c_void_p(self.ptr))
            self.ptr = 0

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass
