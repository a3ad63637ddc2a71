"""Half-spectrum formulation of the reference frame (TEST INFRASTRUCTURE, float64 numpy).

The reference packs 8 real fields into 4 complex lanes (resources/spectrum.compute:218-239) and
transforms each lane over the full N x N grid (src/FFTCalculator.cpp:73-114). Every lane is a
real multiplier of the evolved amplitude H(u, v) (u, v = x - N/2, y - N/2 the frequency indices):

  lane0 = H + i (i kx H)              = (1 - kx) A
  lane1 = i kz H + i (i dirx H)       = i B - kx C
  lane2 = i dirz H + i (-kx dirx H)   = i (D - kx^2 C)
  lane3 = -kz dirz H + i (-kz dirx H) = -E - i kx D

with A = H, B = kz H, C = H/len, D = kz H/len, E = kz^2 H/len (len = |k|, dirx = kx/len; C, D, E
are 0 at k = 0). The kx factors commute with the transform along y, so after it only the five
G_F(q, u) = sum_v F(v, u) e^{2 pi i v q / N} are needed, and H(-u, -v) = conj(H(u, v)) for v != -N/2
makes each of them (anti-)Hermitian in u:

  G_F(q, -u) = s_F conj(G_F(q, u)) + (-1)^q Delta_F(u),
  Delta_F(u) = F(-N/2, -u) - s_F conj(F(-N/2, u)),      s_F = +1 (A, C, E), -1 (B, D),

the (-1)^q term carrying the reference's non-Hermitian Nyquist row (its partner texel is evaluated
at +N/2, spectrum.compute:165). So the columns u in [0, N/2) plus the Nyquist column u = -N/2 and
one Delta row per field determine the whole frame. This module reconstructs the four lanes from
those and is checked against the direct transform (tests/test_half_spectrum.py); the GPU
half-spectrum path follows the same algebra.
"""
from __future__ import annotations

import numpy as np


def evolve_fields(H: np.ndarray, dk: float):
    """A..E on the [v, u] grid (array index [y, x]) from H, in float64 (reference pack order)."""
    n = H.shape[0]
    idx = np.arange(n) - n // 2
    kz = (idx * dk)[:, None] * np.ones((1, n))
    kx = np.ones((n, 1)) * (idx * dk)[None, :]
    ln = np.hypot(kx, kz)
    inv = np.where(ln == 0, 0.0, 1.0 / np.where(ln == 0, 1.0, ln))
    A = H
    B = kz * H
    C = inv * H
    D = kz * inv * H
    E = kz * kz * inv * H
    return (A, B, C, D, E), kx[0]


def direct_lanes(H: np.ndarray, dk: float):
    """The reference's four packed lanes transformed directly: N^2 ifft2(ifftshift(lane))."""
    (A, B, C, D, E), kx = evolve_fields(H, dk)
    lanes = [(1 - kx) * A, 1j * B - kx * C, 1j * (D - kx * kx * C), -E - 1j * kx * D]
    n = H.shape[0]
    return [np.fft.ifft2(np.fft.ifftshift(L)) * n * n for L in lanes]


SIGN = (1, -1, 1, -1, 1)  # s_F for A, B, C, D, E


def half_spectrum(H: np.ndarray, dk: float):
    """What the column pass keeps: G_F(q, u) for u in [0, N/2) (array columns N/2..N-1), the
    Nyquist column u = -N/2 (array column 0), and Delta_F(u) for u in (0, N/2)."""
    n = H.shape[0]
    fields, _ = evolve_fields(H, dk)
    G, nyq, delta = [], [], []
    for F, s in zip(fields, SIGN):
        # transform along v (array axis 0), frequency index v = y - N/2 -> ifftshift on axis 0
        g = np.fft.ifft(np.fft.ifftshift(F, axes=0), axis=0) * n  # g[q, x]
        G.append(g[:, n // 2:])      # u = 0 .. N/2-1
        nyq.append(g[:, 0])          # u = -N/2
        row = F[0, :]                # v = -N/2 (array row 0), indexed by x = u + N/2
        d = np.zeros(n // 2, complex)
        for u in range(1, n // 2):
            d[u] = row[n // 2 - u] - s * np.conj(row[n // 2 + u])
        delta.append(d)
    return G, nyq, delta


def lanes_from_half(G, nyq, delta, dk: float, n: int):
    """Rebuild the full G_F(q, u) for every u, apply the kx factors, transform along u."""
    q = np.arange(n)
    alt = np.where(q % 2 == 0, 1.0, -1.0)[:, None]
    full = []
    for g, ny, d, s in zip(G, nyq, delta, SIGN):
        f = np.zeros((n, n), complex)  # [q, x]
        f[:, n // 2:] = g
        f[:, 0] = ny
        for u in range(1, n // 2):
            f[:, n // 2 - u] = s * np.conj(g[:, u]) + alt[:, 0] * d[u]
        full.append(f)
    GA, GB, GC, GD, GE = full
    kx = (np.arange(n) - n // 2) * dk
    lanes = [(1 - kx) * GA, 1j * GB - kx * GC, 1j * (GD - kx * kx * GC), -GE - 1j * kx * GD]
    # transform along u (array axis 1, ifftshift on that axis)
    return [np.fft.ifft(np.fft.ifftshift(L, axes=1), axis=1) * n for L in lanes]
