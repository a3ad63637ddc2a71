"""Surface consumer of the generator maps: resources/waveShader.glsl's vertex
displacement (:101-110) and fragment slope normal / Jacobian (:127-144), per mesh vertex, through
ocean_surface_sample / ocean_surface_sample_plane (include/oceanfft.h)."""
from __future__ import annotations

import ctypes

import numpy as np

from . import hip
from .capi import check, lib
from .hip import DeviceBuffer

FLOATS_PER_VERTEX = 8  # x, y, z, jacobian, nx, ny, nz, 0


class SurfaceSampler:
    """The renderer's view of `pairs` = [(Generator, cascade), ...] (src/Renderer.cpp:62-72)."""

    def __init__(self, pairs):
        self.pairs = list(pairs)
        n = len(self.pairs)
        self._gens = (ctypes.c_void_p * n)(*[g.handle.value for g, _ in self.pairs])
        self._cas = (ctypes.c_int * n)(*[int(c) for _, c in self.pairs])
        self.fft = self.pairs[0][0].fft

    def sample(self, xz_ptr: int, points: int, out_ptr: int) -> None:
        check(lib().ocean_surface_sample(self._gens, self._cas, len(self.pairs), ctypes.c_void_p(xz_ptr),
                                         ctypes.c_int64(points), ctypes.c_void_p(out_ptr)), "ocean_surface_sample")

    def sample_plane(self, camera, res: int, out_ptr: int) -> None:
        cam = (ctypes.c_float * 5)(*[float(v) for v in camera])
        check(lib().ocean_surface_sample_plane(self._gens, self._cas, len(self.pairs), cam, int(res),
                                               ctypes.c_void_p(out_ptr)), "ocean_surface_sample_plane")

    def sample_host(self, xz: np.ndarray) -> np.ndarray:
        xz = np.ascontiguousarray(xz, np.float32)
        pts = xz.shape[0]
        src = DeviceBuffer.from_array(xz)
        out = DeviceBuffer(pts * FLOATS_PER_VERTEX * 4)
        self.sample(src.ptr, pts, out.ptr)
        self.fft.synchronize()
        return out.to_host((pts, FLOATS_PER_VERTEX))

    def plane_host(self, camera, res: int) -> np.ndarray:
        pts = (res + 1) * (res + 1)
        out = DeviceBuffer(pts * FLOATS_PER_VERTEX * 4)
        self.sample_plane(camera, res, out.ptr)
        self.fft.synchronize()
        return out.to_host((pts, FLOATS_PER_VERTEX))


def host_cascades(pairs):
    """[(height, disp, jac, planeSize, displacement)] host copies, for the CPU oracle."""
    out = []
    for g, c in pairs:
        s = g.GetOceanSettings(c)
        out.append((g.height_map_host(c), g.displacement_map_host(c), g.jacobian_map_host(c), s.planeSize,
                    s.displacement))
    return out


__all__ = ["SurfaceSampler", "host_cascades", "FLOATS_PER_VERTEX", "hip"]
