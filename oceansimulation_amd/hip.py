"""Minimal HIP runtime access over ctypes (plumbing for tests/bench: copies and syncs of the
library-owned HBM maps, which torch cannot wrap without a DLPack producer)."""
from __future__ import annotations

import ctypes

import numpy as np

_hip = None
H2D, D2H, D2D = 1, 2, 3


def hip():
    global _hip
    if _hip is None:
        for name in ("libamdhip64.so", "/opt/rocm/lib/libamdhip64.so"):
            try:
                _hip = ctypes.CDLL(name)
                break
            except OSError:
                continue
        if _hip is None:
            raise ImportError("libamdhip64.so not found")
        _hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        _hip.hipMemcpy.restype = ctypes.c_int
        _hip.hipDeviceSynchronize.restype = ctypes.c_int
        _hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
        _hip.hipStreamSynchronize.restype = ctypes.c_int
    return _hip


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed with hipError {rc}")


def to_host(dev_ptr: int, shape, dtype=np.float32) -> np.ndarray:
    out = np.empty(shape, dtype)
    _check(hip().hipMemcpy(out.ctypes.data, ctypes.c_void_p(dev_ptr), out.nbytes, D2H), "hipMemcpy D2H")
    return out


def from_host(dev_ptr: int, arr: np.ndarray) -> None:
    arr = np.ascontiguousarray(arr)
    _check(hip().hipMemcpy(ctypes.c_void_p(dev_ptr), arr.ctypes.data, arr.nbytes, H2D), "hipMemcpy H2D")


def stream_with_cu_mask(cus, n_cus: int) -> int:
    """hipExtStreamCreateWithCUMask: a non-default stream whose kernels run only on the CUs listed in
    `cus` (logical CU indices < n_cus). Returns the hipStream_t as an int (wrap it with
    torch.cuda.ExternalStream); release with stream_destroy."""
    h = hip()
    words = (n_cus + 31) // 32
    mask = (ctypes.c_uint32 * words)()
    for c in cus:
        mask[c // 32] |= 1 << (c % 32)
    h.hipExtStreamCreateWithCUMask.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32,
                                               ctypes.POINTER(ctypes.c_uint32)]
    h.hipExtStreamCreateWithCUMask.restype = ctypes.c_int
    s = ctypes.c_void_p()
    _check(h.hipExtStreamCreateWithCUMask(ctypes.byref(s), words, mask), "hipExtStreamCreateWithCUMask")
    return int(s.value)


def stream_destroy(stream: int) -> None:
    h = hip()
    h.hipStreamDestroy.argtypes = [ctypes.c_void_p]
    h.hipStreamDestroy.restype = ctypes.c_int
    _check(h.hipStreamDestroy(ctypes.c_void_p(stream)), "hipStreamDestroy")


def synchronize() -> None:
    _check(hip().hipDeviceSynchronize(), "hipDeviceSynchronize")


class DeviceBuffer:
    """hipMalloc'd scratch owned by Python (tests/bench inputs)."""

    def __init__(self, nbytes: int):
        h = hip()
        h.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
        h.hipMalloc.restype = ctypes.c_int
        h.hipFree.argtypes = [ctypes.c_void_p]
        h.hipFree.restype = ctypes.c_int
        p = ctypes.c_void_p()
        _check(h.hipMalloc(ctypes.byref(p), nbytes), f"hipMalloc({nbytes})")
        self.ptr = int(p.value)
        self.nbytes = nbytes

    @classmethod
    def from_array(cls, arr: np.ndarray) -> "DeviceBuffer":
        arr = np.ascontiguousarray(arr)
        b = cls(arr.nbytes)
        from_host(b.ptr, arr)
        return b

    def to_host(self, shape, dtype=np.float32) -> np.ndarray:
        return to_host(self.ptr, shape, dtype)

    def free(self) -> None:
        if self.ptr:
            hip().hipFree(ctypes.c_void_p(self.ptr))
            self.ptr = 0

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def copy_d2d(dst_ptr: int, src_ptr: int, nbytes: int) -> None:
    _check(hip().hipMemcpy(ctypes.c_void_p(dst_ptr), ctypes.c_void_p(src_ptr), nbytes, D2D), "hipMemcpy D2D")
