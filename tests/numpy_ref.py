"""Independent numpy formulation of the reference hot path (TEST INFRASTRUCTURE).

Written separately from oracle/ocean_oracle.c, directly from the GLSL, to cross-check it:
  * spectrum: resources/spectrum.compute:38-172, vectorised in float32;
  * evolve/pack: resources/spectrum.compute:183-240, float32;
  * iFFT: the *meaning* of src/FFTCalculator.cpp:73-114 (fftShift + bit-reverse + radix-2 DIT with
    a +i twiddle, no normalisation) == N^2 * ifft2(ifftshift(X)), evaluated with numpy's float64 FFT;
  * foam: resources/spectrum.compute:246-259.
numpy's float32 transcendentals differ from libm in the last ulps, so comparisons with the C oracle
use tolerances (stated in tests/test_oracle.py).
"""
from __future__ import annotations

import numpy as np

PI = np.float32(3.14159265358)
F32 = np.float32


def settings_dict(s) -> dict:
    """Plain dict from an OracleSettings/OceanSettings ctypes struct or a dict."""
    if isinstance(s, dict):
        return dict(s)
    names = ["U_10", "theta_0", "F", "g", "swell", "h", "displacement", "time", "planeSize", "scale",
             "spread", "boundWavelength", "wavelengthMin", "wavelengthMax"]
    d = {k: getattr(s, k) for k in names}
    d["seed"] = (int(s.seed[0]), int(s.seed[1]))
    return d


def hash2(x: np.ndarray, y: np.ndarray):
    """spectrum.compute:109-117 on uint32 arrays. Returns (u0, u1, n)."""
    x = x.astype(np.uint32)
    y = y.astype(np.uint32)
    with np.errstate(over="ignore"):
        h = (y + np.uint32(374761393) + x * np.uint32(3266489917)).astype(np.uint32)
        h = (np.uint32(2246822519) * (h ^ (h >> np.uint32(15)))).astype(np.uint32)
        h = (np.uint32(3266489917) * (h ^ (h >> np.uint32(13)))).astype(np.uint32)
        n = (h ^ (h >> np.uint32(16))).astype(np.uint32)
        rz1 = (n * np.uint32(48271)).astype(np.uint32)
    denom = F32(2147483648.0)  # float(0x7FFFFFFF)
    u0 = ((n >> np.uint32(1)) & np.uint32(0x7FFFFFFF)).astype(np.float32) / denom
    u1 = ((rz1 >> np.uint32(1)) & np.uint32(0x7FFFFFFF)).astype(np.float32) / denom
    return u0, u1, n


def _dispersion(k, g, h):
    sigma, rho = F32(0.072), F32(1000.0)
    kh = k * h
    tanh_kh = np.where(kh >= F32(2.0) * PI, F32(1.0), np.tanh(kh)).astype(np.float32)
    return np.sqrt((g * k + sigma / rho * k * k * k) * tanh_kh).astype(np.float32)


def _amplitude(s: dict, tx: np.ndarray, ty: np.ndarray, dim: float):
    g, h, U, F = F32(s["g"]), F32(s["h"]), F32(s["U_10"]), F32(s["F"])
    dk = F32(2.0) * PI / F32(s["planeSize"])
    kx = ((tx - F32(dim) / F32(2.0)) * dk).astype(np.float32)
    ky = ((ty - F32(dim) / F32(2.0)) * dk).astype(np.float32)
    k = np.sqrt(kx * kx + ky * ky).astype(np.float32)
    theta = (np.arctan2(ky, kx) - F32(s["theta_0"])).astype(np.float32)
    zero = k == 0
    ks = np.where(zero, F32(1.0), k).astype(np.float32)  # avoid 0-division; zeroed below
    with np.errstate(all="ignore"):
        omega = _dispersion(ks, g, h)
        omega_p = F32(22.0) * np.power(g * g / (U * F), F32(0.333), dtype=np.float32)
        # JONSWAP (spectrum.compute:60-78)
        alpha = F32(0.076) * np.power(U * U / (F * g), F32(0.22), dtype=np.float32)
        sig = np.where(omega > omega_p, F32(0.09), F32(0.07)).astype(np.float32)
        diff = np.abs(omega - omega_p)
        ratio = omega_p / omega
        r = np.exp(-diff * diff / (F32(2.0) * sig * sig * omega_p * omega_p)).astype(np.float32)
        S = (alpha * g * g / np.power(omega, F32(5.0), dtype=np.float32) *
             np.exp(F32(-1.25) * np.power(ratio, F32(4.0), dtype=np.float32)) *
             np.power(F32(3.3), r, dtype=np.float32)).astype(np.float32)
        w_h = np.minimum(omega * np.sqrt(h / g), F32(2.0))
        t = np.clip(w_h / F32(2.2), F32(0.0), F32(1.0))
        Sj = (S * (t * t * (F32(3.0) - F32(2.0) * t))).astype(np.float32)
        # Hasselmann + Longuet-Higgins (spectrum.compute:81-106)
        p = omega / omega_p
        sh = np.where(omega <= omega_p, F32(6.97) * np.power(np.abs(p), F32(4.06), dtype=np.float32),
                      F32(9.77) * np.power(np.abs(p), F32(-2.33) - F32(1.45) * (U * omega_p / g - F32(1.17)),
                                           dtype=np.float32)).astype(np.float32)
        sh = (sh + F32(16.0) * np.tanh(omega_p / omega) * F32(s["swell"]) * F32(s["swell"])).astype(np.float32)
        a = np.sqrt(sh)
        norm = np.where(sh < F32(0.4),
                        F32(0.5) / PI + sh * (F32(0.220636) + sh * (F32(-0.109) + sh * F32(0.090))),
                        (F32(1.0) / np.sqrt(PI)) * (a * F32(0.5) + (F32(1.0) / a) * F32(0.0625))).astype(np.float32)
        D = (norm * np.power(np.abs(np.cos(theta * F32(0.5))), F32(2.0) * sh, dtype=np.float32)).astype(np.float32)
        spread = F32(s["spread"])
        d = ((F32(1.0) - spread) * D + spread / (F32(2.0) * PI)).astype(np.float32)
        # DispersionDerivative (spectrum.compute:50-57)
        sech = (F32(1.0) / np.cosh(h * ks)).astype(np.float32)
        num = (h * (F32(0.072) / F32(1000.0) * ks * ks * ks + g * ks) * sech * sech + omega * omega).astype(np.float32)
        dwdk = (num / (F32(2.0) * omega)).astype(np.float32)
        chain = (dwdk / ks * dk * dk).astype(np.float32)
        hx = (tx + F32(s["seed"][0])).astype(np.int64).astype(np.uint32)
        hy = (ty + F32(s["seed"][1])).astype(np.int64).astype(np.uint32)
        u0, u1, _ = hash2(hx, hy)
        rr = np.sqrt(F32(-2.0) * np.log(u0)).astype(np.float32)
        th = (F32(2.0) * PI * u1).astype(np.float32)
        amp = np.sqrt(F32(2.0) * Sj * d * chain).astype(np.float32)
        c = F32(0.1) * F32(s["scale"])
        ax = (c * (rr * np.cos(th)) * amp).astype(np.float32)
        ay = (c * (rr * np.sin(th)) * amp).astype(np.float32)
    ax = np.where(zero, F32(0.0), ax)
    ay = np.where(zero, F32(0.0), ay)
    return ax, ay


def generate_spectrum(s, n: int) -> np.ndarray:
    s = settings_dict(s)
    y, x = np.meshgrid(np.arange(n, dtype=np.float32), np.arange(n, dtype=np.float32), indexing="ij")
    a = _amplitude(s, x, y, n)
    b = _amplitude(s, F32(n) - x, F32(n) - y, n)
    return np.stack([a[0], a[1], b[0], -b[1]], axis=-1).astype(np.float32)


def prepare_fft(s, n: int, h0: np.ndarray):
    s = settings_dict(s)
    y, x = np.meshgrid(np.arange(n, dtype=np.float32), np.arange(n, dtype=np.float32), indexing="ij")
    dk = F32(2.0) * PI / F32(s["planeSize"])
    kx = ((x - F32(n) / F32(2.0)) * dk).astype(np.float32)
    kz = ((y - F32(n) / F32(2.0)) * dk).astype(np.float32)
    ln = np.sqrt(kx * kx + kz * kz).astype(np.float32)
    zero = (kx == 0) & (kz == 0)
    with np.errstate(all="ignore"):
        dx = np.where(zero, F32(0), kx / ln).astype(np.float32)
        dz = np.where(zero, F32(0), kz / ln).astype(np.float32)
    k = (ln + F32(1e-6)).astype(np.float32)
    phase = (_dispersion(k, F32(s["g"]), F32(s["h"])) * F32(s["time"])).astype(np.float32)
    c, sn = np.cos(phase), np.sin(phase)
    a = h0
    H = (a[..., 0] + 1j * a[..., 1]) * (c + 1j * sn) + (a[..., 2] + 1j * a[..., 3]) * (c - 1j * sn)
    H = H.astype(np.complex64)
    iH = 1j * H
    A = H + 1j * (kx * iH)
    B = kz * iH + 1j * (dx * iH)
    C = dz * iH + 1j * (-kx * dx * H)
    D = -kz * dz * H + 1j * (-kz * dx * H)
    height = np.stack([A.real, A.imag, B.real, B.imag], -1).astype(np.float32)
    disp = np.stack([C.real, C.imag, D.real, D.imag], -1).astype(np.float32)
    return height, disp


def encode_ifft(img: np.ndarray) -> np.ndarray:
    """N^2 * ifft2(ifftshift(.)) per complex lane, float64 accumulation, float32 result."""
    n = img.shape[0]
    out = np.empty_like(img, dtype=np.float32)
    for lane in range(2):
        z = img[..., 2 * lane].astype(np.float64) + 1j * img[..., 2 * lane + 1].astype(np.float64)
        y = np.fft.ifft2(np.fft.ifftshift(z, axes=(0, 1)), axes=(0, 1)) * (n * n)
        out[..., 2 * lane] = y.real
        out[..., 2 * lane + 1] = y.imag
    return out


def compute_foam(s, disp: np.ndarray) -> np.ndarray:
    lam = F32(settings_dict(s)["displacement"])
    return ((F32(1) + lam * disp[..., 1]) * (F32(1) + lam * disp[..., 2]) -
            lam * lam * disp[..., 3] * disp[..., 3]).astype(np.float32)


def rel_err(got: np.ndarray, ref: np.ndarray) -> float:
    """max |got - ref| / max |ref| (the parity metric used throughout the tests)."""
    ref64 = np.asarray(ref, np.float64)
    scale = np.max(np.abs(ref64))
    err = np.max(np.abs(np.asarray(got, np.float64) - ref64))
    return float(err / scale) if scale > 0 else float(err)
