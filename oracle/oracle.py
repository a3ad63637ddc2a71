"""ctypes wrapper of the CPU oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module, and only
as the checker / the timed CPU baseline — never as the product path. Parity status: UNPINNED by
reference outputs (see ocean_oracle.h and DESIGN.md §Oracle).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboceanoracle.so")


class OracleCascadeMaps(ctypes.Structure):
    """oracle_cascade_maps: one cascade's maps as the renderer binds them."""

    _fields_ = [
        ("height", ctypes.POINTER(ctypes.c_float)),
        ("disp", ctypes.POINTER(ctypes.c_float)),
        ("jac", ctypes.POINTER(ctypes.c_float)),
        ("n", ctypes.c_int),
        ("planeSize", ctypes.c_float),
        ("displacement", ctypes.c_float),
    ]


class OracleSettings(ctypes.Structure):
    """Waves::GeneratorSettings (src/Generator.h:12-30), 64 bytes."""

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


_lib = None


def build() -> str:
    """Compile the oracle with its own Makefile (gcc)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        fp = ctypes.POINTER(ctypes.c_float)
        sp = ctypes.POINTER(OracleSettings)
        L.oracle_default_settings.argtypes = [sp]
        L.oracle_hash.argtypes = [ctypes.c_uint32, ctypes.c_uint32, fp, ctypes.POINTER(ctypes.c_uint32)]
        L.oracle_generate_spectrum.argtypes = [sp, ctypes.c_int, fp]
        L.oracle_spectrum_texels.argtypes = [sp, ctypes.c_int, ctypes.c_int64, ctypes.POINTER(ctypes.c_int32), fp]
        L.oracle_prepare_fft.argtypes = [sp, ctypes.c_int, fp, fp, fp]
        L.oracle_prepare_fft_rows.argtypes = [sp, ctypes.c_int, ctypes.c_int, ctypes.c_int, fp, fp, fp]
        L.oracle_encode_ifft.argtypes = [ctypes.c_int, fp, fp]
        L.oracle_compute_foam.argtypes = [sp, ctypes.c_int, fp, fp]
        L.oracle_calculate_ocean.argtypes = [sp, ctypes.c_int, ctypes.c_float, ctypes.c_int, fp, fp, fp, fp, fp]
        cp = ctypes.POINTER(OracleCascadeMaps)
        L.oracle_surface_points.argtypes = [cp, ctypes.c_int, fp, ctypes.c_int64, fp]
        L.oracle_surface_plane.argtypes = [cp, ctypes.c_int, fp, ctypes.c_int, fp]
        L.oracle_set_threads.argtypes = [ctypes.c_int]
        L.oracle_get_threads.restype = ctypes.c_int
        _lib = L
    return _lib


def _fp(a: np.ndarray):
    assert a.dtype == np.float32 and a.flags.c_contiguous
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def default_settings(**overrides) -> OracleSettings:
    s = OracleSettings()
    lib().oracle_default_settings(ctypes.byref(s))
    for k, v in overrides.items():
        if k == "seed":
            s.seed[0], s.seed[1] = int(v[0]), int(v[1])
        else:
            setattr(s, k, v)
    return s


def set_threads(n: int) -> None:
    lib().oracle_set_threads(int(n))


def get_threads() -> int:
    return int(lib().oracle_get_threads())


def hash_uv(x: int, y: int):
    out = (ctypes.c_float * 2)()
    raw = ctypes.c_uint32()
    lib().oracle_hash(x, y, out, ctypes.byref(raw))
    return float(out[0]), float(out[1]), int(raw.value)


def generate_spectrum(s: OracleSettings, n: int) -> np.ndarray:
    h0 = np.zeros((n, n, 4), np.float32)
    lib().oracle_generate_spectrum(ctypes.byref(s), n, _fp(h0))
    return h0


def spectrum_texels(s: OracleSettings, n: int, xy: np.ndarray) -> np.ndarray:
    """generateSpectrum's texels at the (x, y) index pairs `xy` ([count, 2]) of an N x N image."""
    xy = np.ascontiguousarray(xy, np.int32)
    out = np.zeros((len(xy), 4), np.float32)
    lib().oracle_spectrum_texels(ctypes.byref(s), n, len(xy), xy.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                 _fp(out))
    return out


def prepare_fft(s: OracleSettings, n: int, h0: np.ndarray):
    height = np.zeros((n, n, 4), np.float32)
    disp = np.zeros((n, n, 4), np.float32)
    lib().oracle_prepare_fft(ctypes.byref(s), n, _fp(np.ascontiguousarray(h0, np.float32)), _fp(height), _fp(disp))
    return height, disp


def spectrum_rows(s: OracleSettings, n: int, y0: int, rows: int) -> np.ndarray:
    """generateSpectrum's texels on rows [y0, y0 + rows) of an N x N image -> (rows, N, 4)."""
    y, x = np.meshgrid(np.arange(y0, y0 + rows, dtype=np.int32), np.arange(n, dtype=np.int32), indexing="ij")
    return spectrum_texels(s, n, np.stack([x.ravel(), y.ravel()], 1)).reshape(rows, n, 4)


def prepare_fft_rows(s: OracleSettings, n: int, y0: int, h0_rows: np.ndarray):
    """prepareFFT on the spectrum rows [y0, y0 + len(h0_rows)) -> (height, disp) rows."""
    rows = h0_rows.shape[0]
    height = np.zeros((rows, n, 4), np.float32)
    disp = np.zeros((rows, n, 4), np.float32)
    lib().oracle_prepare_fft_rows(ctypes.byref(s), n, y0, rows, _fp(np.ascontiguousarray(h0_rows, np.float32)),
                                  _fp(height), _fp(disp))
    return height, disp


def sampled_frame(s: OracleSettings, n: int, xs, ys, chunk: int = 256, progress: bool = False):
    """The frame's maps at the sample points (xs x ys) without a full-size transform: the oracle's h0
    and prepareFFT (fp32, the reference's arithmetic) on spectrum rows in chunks, then the 2D inverse
    DFT of EncodeIFFT (N^2 ifft2(ifftshift), src/FFTCalculator.cpp:73-114) evaluated in float64 at
    those points only: out(x, y) = sum_{i, j} X[j][i] exp(2 pi i ((i - N/2) x + (j - N/2) y) / N).
    Returns (height, disp, jacobian) of shape (len(ys), len(xs), 4 | 4 | -)."""
    xs, ys = np.asarray(xs), np.asarray(ys)
    idx = np.arange(n, dtype=np.float64) - n / 2
    ex = np.exp(2j * np.pi * np.outer(idx, xs) / n)  # [N, X]
    ey = np.exp(2j * np.pi * np.outer(idx, ys) / n)  # [N, Y]
    acc = np.zeros((4, len(ys), n), np.complex128)   # lanes: height xy, zw; disp xy, zw
    for y0 in range(0, n, chunk):
        if progress and y0 % (16 * chunk) == 0:
            print(f"sampled_frame: spectrum rows {y0} / {n}", flush=True)
        rows = min(chunk, n - y0)
        h, d = prepare_fft_rows(s, n, y0, spectrum_rows(s, n, y0, rows))
        for k, (img, lane) in enumerate(((h, 0), (h, 1), (d, 0), (d, 1))):
            z = img[..., 2 * lane].astype(np.float64) + 1j * img[..., 2 * lane + 1].astype(np.float64)
            acc[k] += ey[y0:y0 + rows].T @ z
    out = acc @ ex  # [4, Y, X]
    height = np.stack([out[0].real, out[0].imag, out[1].real, out[1].imag], -1)
    disp = np.stack([out[2].real, out[2].imag, out[3].real, out[3].imag], -1)
    lam = float(s.displacement)
    jac = (1 + lam * disp[..., 1]) * (1 + lam * disp[..., 2]) - lam * lam * disp[..., 3] ** 2
    return height, disp, jac


def encode_ifft(img: np.ndarray) -> np.ndarray:
    """FFTCalculator::EncodeIFFT on a copy of img (N x N x 4 float32)."""
    n = img.shape[0]
    out = np.array(img, dtype=np.float32, order="C", copy=True)
    work = np.zeros_like(out)
    lib().oracle_encode_ifft(n, _fp(out), _fp(work))
    return out


def compute_foam(s: OracleSettings, disp: np.ndarray) -> np.ndarray:
    n = disp.shape[0]
    jac = np.zeros((n, n), np.float32)
    lib().oracle_compute_foam(ctypes.byref(s), n, _fp(np.ascontiguousarray(disp, np.float32)), _fp(jac))
    return jac


def _cascade_table(cascades):
    """cascades: [(height N*N*4, disp N*N*4, jac N*N, planeSize, displacement)] float32 arrays."""
    keep = []
    table = (OracleCascadeMaps * len(cascades))()
    for i, (h, d, j, L, disp) in enumerate(cascades):
        h, d, j = (np.ascontiguousarray(a, np.float32) for a in (h, d, j))
        keep += [h, d, j]
        table[i] = OracleCascadeMaps(_fp(h), _fp(d), _fp(j), h.shape[0], L, disp)
    return table, keep


def surface_points(cascades, xz: np.ndarray) -> np.ndarray:
    """waveShader.glsl displacement + normal + Jacobian at base positions xz (P x 2) -> (P, 8)."""
    table, keep = _cascade_table(cascades)
    xz = np.ascontiguousarray(xz, np.float32)
    out = np.zeros((xz.shape[0], 8), np.float32)
    lib().oracle_surface_points(table, len(cascades), _fp(xz), xz.shape[0], _fp(out))
    return out


def surface_plane(cascades, cam, res: int) -> np.ndarray:
    """The reference plane mesh through the camera warp -> ((res+1)^2, 8)."""
    table, keep = _cascade_table(cascades)
    c = np.asarray(cam, np.float32)
    out = np.zeros(((res + 1) * (res + 1), 8), np.float32)
    lib().oracle_surface_plane(table, len(cascades), _fp(c), res, _fp(out))
    return out


class OracleGenerator:
    """Generator::CalculateOcean state machine (src/Generator.cpp:45-83) on the CPU."""

    def __init__(self, n: int, settings: OracleSettings | None = None):
        self.n = n
        self.settings = settings if settings is not None else default_settings()
        self.h0 = np.zeros((n, n, 4), np.float32)
        self.height = np.zeros((n, n, 4), np.float32)
        self.disp = np.zeros((n, n, 4), np.float32)
        self.jac = np.zeros((n, n), np.float32)
        self.work = np.zeros((n, n, 4), np.float32)
        self._update = True  # Generator.h:72 updateSpectrum = true

    def calculate_ocean(self, timestep: float, update_ocean: bool = False) -> None:
        upd = 1 if (self._update or update_ocean) else 0
        self._update = False
        lib().oracle_calculate_ocean(
            ctypes.byref(self.settings), self.n, ctypes.c_float(timestep), upd,
            _fp(self.h0), _fp(self.height), _fp(self.disp), _fp(self.jac), _fp(self.work))
