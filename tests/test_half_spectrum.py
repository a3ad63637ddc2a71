"""The half-spectrum factorisation the GPU generator uses (tests/half_spectrum_ref.py) reproduces
the reference's four packed lanes exactly (float64), including the non-Hermitian Nyquist row the
reference creates (spectrum.compute:165)."""
import numpy as np
import pytest

import half_spectrum_ref as HS


def _hermitian_h(n, seed, nyquist_noise=True):
    rng = np.random.default_rng(seed)
    h0 = rng.standard_normal((n, n)) + 1j * rng.standard_normal((n, n))
    # H(k) = h0(k) e + conj(h0(-k)) e*, -k taken as index N - i like the reference (so the
    # Nyquist row/column pair with the off-grid index N: a separate draw)
    hN = rng.standard_normal((n + 1, n + 1)) + 1j * rng.standard_normal((n + 1, n + 1))
    hN[:n, :n] = h0
    if not nyquist_noise:
        hN[n, :] = hN[0, :]
        hN[:, n] = hN[:, 0]
    y, x = np.meshgrid(np.arange(n), np.arange(n), indexing="ij")
    e = np.exp(1j * 0.37 * np.hypot(x - n / 2, y - n / 2))
    return h0 * e + np.conj(hN[n - y, n - x]) * np.conj(e)


@pytest.mark.parametrize("n", [16, 64, 256])
def test_half_spectrum_rebuilds_the_reference_lanes(n):
    H = _hermitian_h(n, n)
    dk = 2 * np.pi / 17.0
    direct = HS.direct_lanes(H, dk)
    G, nyq, delta = HS.half_spectrum(H, dk)
    rebuilt = HS.lanes_from_half(G, nyq, delta, dk, n)
    for r, d in zip(rebuilt, direct):
        assert np.max(np.abs(r - d)) <= 1e-12 * np.max(np.abs(d))


def test_nyquist_row_correction_is_needed():
    """Without Delta the rebuild misses the reference's Nyquist-row asymmetry."""
    n = 64
    H = _hermitian_h(n, 5)
    dk = 2 * np.pi / 17.0
    direct = HS.direct_lanes(H, dk)
    G, nyq, delta = HS.half_spectrum(H, dk)
    wrong = HS.lanes_from_half(G, nyq, [np.zeros_like(d) for d in delta], dk, n)
    assert max(np.max(np.abs(w - d)) / np.max(np.abs(d)) for w, d in zip(wrong, direct)) > 1e-3
