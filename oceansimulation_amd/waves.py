"""Python mirror of the reference's Waves::FFTCalculator / Waves::Generator over the C ABI.

Same names and argument meaning as src/FFTCalculator.h:11-59 and src/Generator.h:33-93 (snake_case
aliases added); errors raise OceanError (the reference has no error path). Outputs are device
pointers into HBM owned by the objects; `*_host()` helpers copy them out for checking.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import capi, hip
from .capi import OceanSettings, check, lib


def default_settings(**overrides) -> OceanSettings:
    """GeneratorSettings defaults (src/Generator.h:14-29) with keyword overrides."""
    s = OceanSettings()
    lib().ocean_default_settings(ctypes.byref(s))
    apply_settings(s, **overrides)
    return s


def apply_settings(s: OceanSettings, **overrides) -> OceanSettings:
    for k, v in overrides.items():
        if k == "seed":
            s.seed[0], s.seed[1] = int(v[0]), int(v[1])
        else:
            setattr(s, k, v)
    return s


class FFTCalculator:
    """Waves::FFTCalculator (src/FFTCalculator.h:11-59)."""

    def __init__(self, texture_size: int = 512, stream: int | None = None):
        h = ctypes.c_void_p()
        check(lib().ocean_fft_create(ctypes.byref(h), texture_size, ctypes.c_void_p(stream or 0)),
              "ocean_fft_create")
        self._h = h
        self.texture_size = texture_size

    def GetTextureResolution(self) -> int:
        return int(lib().ocean_fft_texture_resolution(self._h))

    get_texture_resolution = GetTextureResolution

    def EncodeIFFT(self, image_ptr: int) -> None:
        """In-place iFFT of a device RGBA32F N x N image (src/FFTCalculator.cpp:73-114)."""
        check(lib().ocean_fft_encode_ifft(self._h, ctypes.c_void_p(image_ptr)), "ocean_fft_encode_ifft")

    encode_ifft = EncodeIFFT

    def encode_ifft_batch(self, images_ptr: int, n_images: int) -> None:
        check(lib().ocean_fft_encode_ifft_batch(self._h, ctypes.c_void_p(images_ptr), n_images),
              "ocean_fft_encode_ifft_batch")

    def synchronize(self) -> None:
        check(lib().ocean_fft_synchronize(self._h), "ocean_fft_synchronize")

    @property
    def cus(self) -> int:
        return int(lib().ocean_fft_device_cus(self._h))

    def set_cu_budget(self, cus: int) -> None:
        """Size this plan's persistent grids for `cus` CUs (0 = all); see ocean_fft_set_cu_budget."""
        check(lib().ocean_fft_set_cu_budget(self._h, int(cus)), "ocean_fft_set_cu_budget")

    @property
    def handle(self):
        return self._h

    def close(self) -> None:
        if self._h:
            lib().ocean_fft_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Generator:
    """Waves::Generator (src/Generator.h:33-93), batched over `cascades` cascades sharing N."""

    def __init__(self, fft: FFTCalculator, cascades: int = 1):
        h = ctypes.c_void_p()
        check(lib().ocean_generator_create(ctypes.byref(h), fft.handle, cascades), "ocean_generator_create")
        self._h = h
        self.fft = fft
        self.n = fft.GetTextureResolution()
        self.cascades = cascades

    @property
    def handle(self):
        return self._h

    def set_half_spectrum(self, enable: bool) -> None:
        """Select the half-spectrum (default where supported) or the full-spectrum frame path."""
        check(lib().ocean_generator_set_half_spectrum(self._h, 1 if enable else 0), "ocean_generator_set_half_spectrum")

    def set_four_step(self, enable: bool) -> None:
        """Whole grids of 8192 / 16384 on one rank: the four-step column pass (default) or the
        strip-dealt column pass + transposes that multi-rank slabs run (bit-identical to them)."""
        check(lib().ocean_generator_set_four_step(self._h, 1 if enable else 0), "ocean_generator_set_four_step")

    def set_h0_memo(self, enable: bool) -> None:
        """Skip requested re-seeds whose h0 inputs are unchanged (default) or re-seed every time."""
        check(lib().ocean_generator_set_h0_memo(self._h, 1 if enable else 0), "ocean_generator_set_h0_memo")

    def set_frame_overlap(self, enable: bool) -> None:
        """Run frame f + 1's column pass beside frame f's row pass (whole grids of 1024..4096, half
        spectrum; bit-identical results; pays at 1-2 cascades)."""
        check(lib().ocean_generator_set_frame_overlap(self._h, 1 if enable else 0),
              "ocean_generator_set_frame_overlap")

    def frame_bytes(self):
        """Algorithmic HBM bytes per point of the column and row pass of the current path."""
        out = (ctypes.c_double * 2)()
        check(lib().ocean_generator_frame_bytes(self._h, out), "ocean_generator_frame_bytes")
        return float(out[0]), float(out[1])

    def GetOceanSettings(self, cascade: int = 0) -> OceanSettings:
        p = lib().ocean_generator_settings(self._h, cascade)
        if not p:
            raise capi.OceanError(capi.OCEAN_ERR_INVALID, "ocean_generator_settings")
        return p.contents

    get_ocean_settings = GetOceanSettings

    def CalculateOcean(self, timestep: float, update_ocean: bool = False) -> None:
        check(lib().ocean_generator_calculate(self._h, ctypes.c_float(timestep), 1 if update_ocean else 0),
              "ocean_generator_calculate")

    calculate_ocean = CalculateOcean

    def GenerateSpectrum(self) -> None:
        check(lib().ocean_generator_generate_spectrum(self._h), "ocean_generator_generate_spectrum")

    def GetHeightMap(self, cascade: int = 0) -> int:
        return int(lib().ocean_generator_height_map(self._h, cascade))

    def GetDisplacementMap(self, cascade: int = 0) -> int:
        return int(lib().ocean_generator_displacement_map(self._h, cascade))

    def GetJacobianMap(self, cascade: int = 0) -> int:
        return int(lib().ocean_generator_jacobian_map(self._h, cascade))

    def GetInitialSpectrum(self, cascade: int = 0) -> int:
        return int(lib().ocean_generator_initial_spectrum(self._h, cascade))

    # ---- host copies (checking / export) ----
    def height_map_host(self, cascade: int = 0) -> np.ndarray:
        self.fft.synchronize()
        return hip.to_host(self.GetHeightMap(cascade), (self.n, self.n, 4))

    def displacement_map_host(self, cascade: int = 0) -> np.ndarray:
        self.fft.synchronize()
        return hip.to_host(self.GetDisplacementMap(cascade), (self.n, self.n, 4))

    def jacobian_map_host(self, cascade: int = 0) -> np.ndarray:
        self.fft.synchronize()
        return hip.to_host(self.GetJacobianMap(cascade), (self.n, self.n))

    def initial_spectrum_host(self, cascade: int = 0) -> np.ndarray:
        """h0 as an N x N x 4 row-major image (de-blocked from the device's strip-blocked layout)."""
        self.fft.synchronize()
        b = int(lib().ocean_generator_spectrum_block(self._h))
        blocked = hip.to_host(self.GetInitialSpectrum(cascade), (self.n // b, self.n, b, 4))
        return np.ascontiguousarray(blocked.transpose(1, 0, 2, 3).reshape(self.n, self.n, 4))

    # ---- instrumentation ----
    def set_profiling(self, enable: bool) -> None:
        check(lib().ocean_generator_set_profiling(self._h, 1 if enable else 0), "ocean_generator_set_profiling")

    def kernel_times(self):
        """(ms totals, launch counts) for [spectrum, column pass, row pass] since the last call."""
        ms = (ctypes.c_double * 3)()
        cnt = (ctypes.c_int64 * 3)()
        check(lib().ocean_generator_kernel_times(self._h, ms, cnt), "ocean_generator_kernel_times")
        return list(ms), list(cnt)

    def close(self) -> None:
        if self._h:
            lib().ocean_generator_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def debug_copy(dst_ptr: int, src_ptr: int, nbytes: int, workgroups: int, stream: int | None = None) -> None:
    """ocean_debug_copy: a copy on exactly `workgroups` 256-thread workgroups (a rate-limited HBM stream)."""
    check(lib().ocean_debug_copy(ctypes.c_void_p(dst_ptr), ctypes.c_void_p(src_ptr), nbytes, workgroups,
                                 ctypes.c_void_p(stream or 0)), "ocean_debug_copy")


def debug_hash(xy_dev_ptr: int, count: int, raw_dev_ptr: int, uv_dev_ptr: int, stream: int | None = None) -> None:
    check(lib().ocean_debug_hash(ctypes.c_void_p(xy_dev_ptr), count, ctypes.c_void_p(raw_dev_ptr),
                                 ctypes.c_void_p(uv_dev_ptr), ctypes.c_void_p(stream or 0)), "ocean_debug_hash")
