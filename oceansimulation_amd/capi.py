"""ctypes binding of liboceanfft.so — every entry point declared in include/oceanfft.h.

The library is the product path (HIP kernels for gfx950). There is no CPU fallback: if the
shared object is missing, `lib()` raises, and every compute call fails loudly without a GPU.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liboceanfft.so")

OCEAN_OK = 0
OCEAN_ERR_INVALID = 1
OCEAN_ERR_HIP = 2
OCEAN_ERR_NO_DEVICE = 3
OCEAN_ERR_OOM = 4
OCEAN_ERR_TIMEOUT = 5
OCEAN_MAX_CASCADES = 64
OCEAN_COMM_ID_BYTES = 128
OCEAN_PEER_HANDLE_BYTES = 256


class OceanSettings(ctypes.Structure):
    """ocean_settings == Waves::GeneratorSettings (reference src/Generator.h:12-30), 64 bytes."""

    _fields_ = [
        ("seed", ctypes.c_int32 * 2),
        ("U_10", ctypes.c_float),
        ("theta_0", ctypes.c_float),
        ("F", ctypes.c_float),
        ("g", ctypes.c_float),
        ("swell", ctypes.c_float),
        ("h", ctypes.c_float),
        ("displacement", ctypes.c_float),
        ("time", ctypes.c_float),
        ("planeSize", ctypes.c_float),
        ("scale", ctypes.c_float),
        ("spread", ctypes.c_float),
        ("boundWavelength", ctypes.c_int32),
        ("wavelengthMin", ctypes.c_float),
        ("wavelengthMax", ctypes.c_float),
    ]


assert ctypes.sizeof(OceanSettings) == 64

_vp = ctypes.c_void_p
_i = ctypes.c_int
_f = ctypes.c_float
_sz = ctypes.c_size_t
_fp = ctypes.POINTER(ctypes.c_float)
_sp = ctypes.POINTER(OceanSettings)

# name -> (restype, argtypes); mirrors include/oceanfft.h one to one.
SIGNATURES = {
    "ocean_last_error": (ctypes.c_char_p, []),
    "ocean_version": (ctypes.c_char_p, []),
    "ocean_default_settings": (None, [_sp]),
    "ocean_device_count": (_i, []),
    "ocean_fft_create": (_i, [ctypes.POINTER(_vp), _sz, _vp]),
    "ocean_fft_destroy": (_i, [_vp]),
    "ocean_fft_texture_resolution": (_sz, [_vp]),
    "ocean_fft_encode_ifft": (_i, [_vp, _vp]),
    "ocean_fft_encode_ifft_batch": (_i, [_vp, _vp, _i]),
    "ocean_fft_synchronize": (_i, [_vp]),
    "ocean_fft_device_cus": (_i, [_vp]),
    "ocean_fft_set_cu_budget": (_i, [_vp, _i]),
    "ocean_generator_create": (_i, [ctypes.POINTER(_vp), _vp, _i]),
    "ocean_generator_destroy": (_i, [_vp]),
    "ocean_generator_cascades": (_i, [_vp]),
    "ocean_generator_settings": (_sp, [_vp, _i]),
    "ocean_generator_calculate": (_i, [_vp, _f, _i]),
    "ocean_generator_generate_spectrum": (_i, [_vp]),
    "ocean_generator_height_map": (_vp, [_vp, _i]),
    "ocean_generator_displacement_map": (_vp, [_vp, _i]),
    "ocean_generator_jacobian_map": (_vp, [_vp, _i]),
    "ocean_generator_initial_spectrum": (_vp, [_vp, _i]),
    "ocean_generator_spectrum_block": (_i, [_vp]),
    "ocean_generator_create_slab": (_i, [ctypes.POINTER(_vp), _vp, _i, _i]),
    "ocean_generator_exchange_bytes": (_sz, [_vp]),
    "ocean_generator_slab_columns": (_i, [_vp, _f, _i, _vp]),
    "ocean_generator_slab_rows": (_i, [_vp, _vp]),
    "ocean_generator_slab_info": (_i, [_vp, ctypes.POINTER(_i), ctypes.POINTER(_i), ctypes.POINTER(_i), ctypes.POINTER(_i)]),
    "ocean_generator_set_profiling": (_i, [_vp, _i]),
    "ocean_generator_kernel_times": (_i, [_vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64)]),
    "ocean_debug_hash": (_i, [_vp, _i, _vp, _vp, _vp]),
    "ocean_debug_copy": (_i, [_vp, _vp, _sz, _i, _vp]),
    "ocean_surface_sample": (_i, [_vp, _vp, _i, _vp, ctypes.c_int64, _vp]),
    "ocean_surface_sample_plane": (_i, [_vp, _vp, _i, _vp, _i, _vp]),
    "ocean_generator_set_half_spectrum": (_i, [_vp, _i]),
    "ocean_generator_set_four_step": (_i, [_vp, _i]),
    "ocean_generator_set_h0_memo": (_i, [_vp, _i]),
    "ocean_generator_set_frame_overlap": (_i, [_vp, _i]),
    "ocean_generator_frame_bytes": (_i, [_vp, _vp]),
    "ocean_slab_layout": (_i, [_sz, _i, _i, _i, ctypes.POINTER(ctypes.c_int64)]),
    "ocean_comm_unique_id": (_i, [_vp]),
    "ocean_comm_create": (_i, [ctypes.POINTER(_vp), _vp, _i, _i]),
    "ocean_comm_wrap": (_i, [ctypes.POINTER(_vp), _vp, _i, _i]),
    "ocean_comm_destroy": (_i, [_vp]),
    "ocean_comm_all_to_all": (_i, [_vp, _vp, _vp, _sz, _vp]),
    "ocean_generator_slab_frame": (_i, [_vp, _vp, _f, _i]),
    "ocean_generator_slab_frame_pipelined": (_i, [_vp, _vp, _f, _i]),
    "ocean_generator_slab_flush": (_i, [_vp]),
    "ocean_peers_create": (_i, [ctypes.POINTER(_vp), _vp]),
    "ocean_peers_destroy": (_i, [_vp]),
    "ocean_peers_handle": (_i, [_vp, _vp]),
    "ocean_peers_connect": (_i, [_vp, _vp]),
    "ocean_peers_connect_local": (_i, [ctypes.POINTER(_vp), _i]),
    "ocean_peers_set_timeout": (_i, [_vp, _i]),
    "ocean_peers_set_put_cus": (_i, [_vp, _i]),
    "ocean_peers_set_streams": (_i, [_vp, _vp, _vp, _vp]),
    "ocean_peers_set_row_cus": (_i, [_vp, _i]),
    "ocean_peers_set_put_cu_mask": (_i, [_vp, _i]),
    "ocean_generator_kernel_times4": (_i, [_vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64)]),
    "ocean_generator_slab_frame_put": (_i, [_vp, _vp, _f, _i]),
    "ocean_generator_slab_frame_put_pipelined": (_i, [_vp, _vp, _f, _i]),
    "ocean_peers_flush": (_i, [_vp]),
    "ocean_frame_plan": (_i, [_sz, _i, _i, ctypes.POINTER(ctypes.c_int32)]),
    "ocean_peers_debug_slot": (_i, [_vp, _i, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(_sz)]),
    "ocean_generator_slab_put_columns": (_i, [_vp, _vp, _f, _i]),
    "ocean_generator_slab_put_rows": (_i, [_vp, _vp]),
    "ocean_peers_synchronize": (_i, [_vp]),
}

_lib = None


class OceanError(RuntimeError):
    def __init__(self, code: int, where: str):
        msg = lib().ocean_last_error().decode(errors="replace")
        super().__init__(f"{where} failed with status {code}: {msg}")
        self.code = code


def lib():
    """Load liboceanfft.so (built in-tree by `make`); raises if it is absent."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing — run `make` (or __graft_entry__.build()) first; "
                              "there is no CPU fallback for the ocean hot path")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(code: int, where: str) -> None:
    if code != OCEAN_OK:
        raise OceanError(code, where)
