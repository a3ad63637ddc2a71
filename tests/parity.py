"""Parity metrics and tolerances used by the tests (stated once, here).

lane_err:    for a packed RGBA32F image, the two complex lanes (xy, zw) are compared separately:
             max |got - ref| over the lane / max |ref| over the lane (complex modulus). Used for
             EncodeIFFT on arbitrary inputs, where a lane is one transform.
channel_err: each of the 4 real channels of a map on its own: max |got - ref| / max |ref| per
             channel. The generator's maps are 8 real fields (src/Generator.h:76-80: heightMap =
             (h, dh/dx, dh/dz, Dx), displacementMap = (Dz, dDx/dx, dDz/dz, dDx/dz)); a lane pairs a
             height with a slope up to |k|max ~ 1e3 times larger, so the lane metric would judge h
             against the slope's scale. Frames are checked per channel.
Tolerances (float32 path):
  FFT_TOL   = 2e-5  — EncodeIFFT alone. The reference's own fp32 radix-2 structure is 0.2-5e-6 from
                      float64 at N <= 1024 (oracle vs numpy, tests/test_oracle.py); the HIP Stockham
                      radix-16 path must land within this of the oracle.
  FRAME_TOL = 1e-4  — full CalculateOcean from h0 against the oracle, per lane. The oracle repeats the
                      reference's fp32 radix-2 FFT (per-butterfly cos/sin), which alone is up to
                      1.9e-5 per channel from float64 at 4096^2 (L = 5 m, Dx; tools/parity_probe.py).
  FRAME_TOL_GPU = 1e-5 — full frames, per channel, against the oracle's own fp32 spectrum (h0 and
                      prepareFFT at the frame's time, the reference's arithmetic) transformed in
                      float64: the GPU's error with the oracle's FFT rounding taken out. Observed
                      0.4-5.7e-6 over N = 256 .. 16384, t up to 3600 s (profiles/r03_parity_report.md).
  H0_TOL    = 1e-5  — generateSpectrum (relative to max |h0| per lane).
  Hash: bit-exact.
"""
import numpy as np

FFT_TOL = 2e-5
FRAME_TOL = 1e-4
FRAME_TOL_GPU = 1e-5
H0_TOL = 1e-5


def channel_err(got: np.ndarray, ref: np.ndarray):
    out = []
    for ch in range(got.shape[-1]):
        r = ref[..., ch].astype(np.float64)
        scale = np.max(np.abs(r))
        err = np.max(np.abs(got[..., ch].astype(np.float64) - r))
        out.append(float(err / scale) if scale > 0 else float(err))
    return out


def lane_err(got: np.ndarray, ref: np.ndarray):
    out = []
    for lane in range(2):
        g = got[..., 2 * lane].astype(np.float64) + 1j * got[..., 2 * lane + 1].astype(np.float64)
        r = ref[..., 2 * lane].astype(np.float64) + 1j * ref[..., 2 * lane + 1].astype(np.float64)
        scale = np.max(np.abs(r))
        err = np.max(np.abs(g - r))
        out.append(float(err / scale) if scale > 0 else float(err))
    return out


def scalar_err(got: np.ndarray, ref: np.ndarray) -> float:
    ref = np.asarray(ref, np.float64)
    scale = np.max(np.abs(ref))
    err = np.max(np.abs(np.asarray(got, np.float64) - ref))
    return float(err / scale) if scale > 0 else float(err)
