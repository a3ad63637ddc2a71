"""CPU tests of the oracle (test infrastructure) against an independent numpy formulation, analytic
FFT known answers and the committed golden fixtures. No GPU needed.

Parity status: the reference has no tests/fixtures and its GLSL cannot run here,
so the oracle is cross-validated (numpy_ref.py, written separately from the GLSL) rather than pinned.
"""
import os

import numpy as np
import pytest

import numpy_ref as R
from parity import lane_err, scalar_err

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ocean_golden.npz")


def _hash_python(x: int, y: int):
    """Third, scalar-integer restatement of spectrum.compute:109-117 (mod 2^32 by hand)."""
    M = 0xFFFFFFFF
    h = (y + 374761393 + x * 3266489917) & M
    h = (2246822519 * (h ^ (h >> 15))) & M
    h = (3266489917 * (h ^ (h >> 13))) & M
    n = h ^ (h >> 16)
    rz1 = (n * 48271) & M
    return n, np.float32((n >> 1) & 0x7FFFFFFF) / np.float32(2147483648.0), \
        np.float32((rz1 >> 1) & 0x7FFFFFFF) / np.float32(2147483648.0)


def test_hash_three_way_bit_exact(oracle):
    rng = np.random.default_rng(3)
    xy = rng.integers(0, 2**32, size=(2000, 2), dtype=np.uint64).astype(np.uint32)
    xy[:4] = [[0, 0], [12342, 8934], [2**32 - 1, 0], [7, 2**32 - 1]]
    u0, u1, n = R.hash2(xy[:, 0], xy[:, 1])
    for k in range(len(xy)):
        a, b, raw = oracle.hash_uv(int(xy[k, 0]), int(xy[k, 1]))
        pn, pa, pb = _hash_python(int(xy[k, 0]), int(xy[k, 1]))
        assert raw == pn == int(n[k])
        assert np.float32(a) == pa == u0[k] and np.float32(b) == pb == u1[k]


def test_hash_no_zero_uniform_for_default_seed_region():
    """Gaussian() takes log(u0): u0 == 0 would give inf amplitudes (spectrum.compute:124)."""
    y, x = np.meshgrid(np.arange(0, 1025, dtype=np.uint32), np.arange(0, 1025, dtype=np.uint32), indexing="ij")
    u0, _, _ = R.hash2(x + np.uint32(12342), y + np.uint32(8934))
    assert np.all(u0 > 0)


@pytest.mark.parametrize("n", [16, 64, 128])
@pytest.mark.parametrize("plane", [5.0, 17.0, 40.0, 101.0, 4093.0])
def test_spectrum_and_evolve_vs_numpy(oracle, n, plane):
    s = oracle.default_settings(planeSize=plane, time=1.25)
    h0 = oracle.generate_spectrum(s, n)
    assert np.isfinite(h0).all()
    assert max(lane_err(R.generate_spectrum(s, n), h0)) < 1e-6
    # k == 0 texel (centre) carries no energy (spectrum.compute:137-138)
    assert h0[n // 2, n // 2, 0] == 0 and h0[n // 2, n // 2, 1] == 0
    hm, dm = oracle.prepare_fft(s, n, h0)
    hmn, dmn = R.prepare_fft(s, n, h0)
    assert max(lane_err(hmn, hm) + lane_err(dmn, dm)) < 1e-6


@pytest.mark.parametrize("n", [16, 32, 64, 128, 256, 512])
def test_oracle_ifft_vs_float64(oracle, n):
    rng = np.random.default_rng(n)
    img = rng.standard_normal((n, n, 4)).astype(np.float32)
    got = oracle.encode_ifft(img)
    # the reference's fp32 radix-2 structure itself: <= ~5e-6 of the lane maximum at these sizes
    assert max(lane_err(got, R.encode_ifft(img))) < 1e-5


def test_oracle_ifft_known_answers(oracle):
    n = 64
    img = np.zeros((n, n, 4), np.float32)
    img[n // 2, n // 2, 0] = 2.0  # centred DC -> constant 2
    kx, ky = 5, -3
    img[n // 2 + ky, n // 2 + kx, 2] = 1.0  # one bin -> plane wave
    out = oracle.encode_ifft(img)
    assert np.allclose(out[..., 0], 2.0, atol=1e-6) and np.allclose(out[..., 1], 0.0, atol=1e-6)
    y, x = np.meshgrid(np.arange(n), np.arange(n), indexing="ij")
    ph = 2 * np.pi * (kx * x + ky * y) / n
    assert np.max(np.abs(out[..., 2] - np.cos(ph))) < 1e-5
    assert np.max(np.abs(out[..., 3] - np.sin(ph))) < 1e-5
    # Parseval with the unnormalised N^2 factor
    rng = np.random.default_rng(1)
    a = rng.standard_normal((n, n, 4)).astype(np.float32)
    fa = oracle.encode_ifft(a)
    ratio = np.sum(fa.astype(np.float64) ** 2) / (n * n * np.sum(a.astype(np.float64) ** 2))
    assert abs(ratio - 1) < 1e-5


def test_foam_matches_formula(oracle):
    rng = np.random.default_rng(2)
    disp = rng.standard_normal((32, 32, 4)).astype(np.float32)
    s = oracle.default_settings(displacement=0.7)
    assert np.array_equal(oracle.compute_foam(s, disp), R.compute_foam(s, disp))


def test_calculate_ocean_state_machine(oracle):
    """time accumulates in fp32 (Generator.cpp:50); h0 only re-seeded on first call or request."""
    g = oracle.OracleGenerator(16)
    t = np.float32(0)
    for dt in [1 / 60, 1 / 60, 0.1, 0.0]:
        g.calculate_ocean(dt)
        t = np.float32(t + np.float32(dt))
        assert np.float32(g.settings.time) == t
    h0 = g.h0.copy()
    g.settings.U_10 = 10.0
    g.calculate_ocean(0.0)
    assert np.array_equal(g.h0, h0)
    g.calculate_ocean(0.0, update_ocean=True)
    assert not np.array_equal(g.h0, h0)


def test_golden_fixtures_reproduce(oracle):
    import json

    z = np.load(GOLDEN)
    manifest = json.load(open(os.path.join(os.path.dirname(GOLDEN), "manifest.json")))
    for name, case in manifest["cases"].items():
        g = oracle.OracleGenerator(case["n"], oracle.default_settings(**case["settings"]))
        for dt in case["timesteps"]:
            g.calculate_ocean(dt)
        for key, arr in (("h0", g.h0), ("height", g.height), ("disp", g.disp), ("jac", g.jac)):
            ref = z[f"{name}/{key}"]
            assert ref.shape == arr.shape
            assert scalar_err(arr, ref) < 1e-6, (name, key)


# ---- surface consumer restatement (resources/waveShader.glsl) --------------------------------
def _flat_maps(n, h=0.0, dh=(0.0, 0.0), dx=0.0, dz=0.0, jac=1.0):
    height = np.zeros((n, n, 4), np.float32)
    disp = np.zeros((n, n, 4), np.float32)
    height[..., 0], height[..., 1], height[..., 2], height[..., 3] = h, dh[0], dh[1], dx
    disp[..., 0] = dz
    return height, disp, np.full((n, n), jac, np.float32)


def test_surface_constant_maps(oracle):
    """Constant fields: displacement is the sum over cascades, the normal follows the slopes."""
    h, d, j = _flat_maps(16, h=0.5, dh=(0.1, -0.2), dx=2.0, dz=-1.0, jac=0.8)
    c = [(h, d, j, 10.0, 0.4), (h, d, j, 30.0, 0.4)]
    out = oracle.surface_points(c, np.array([[1.0, 2.0], [-7.5, 100.0]], np.float32))
    np.testing.assert_allclose(out[:, 0], [1.0 + 2 * 0.4 * 2.0, -7.5 + 2 * 0.4 * 2.0], rtol=1e-6)
    np.testing.assert_allclose(out[:, 1], 1.0, rtol=1e-6)
    np.testing.assert_allclose(out[:, 2], [2.0 - 0.8, 100.0 - 0.8], rtol=1e-6)
    np.testing.assert_allclose(out[:, 3], 0.8, rtol=1e-6)
    nrm = np.array([-0.2, 1.0, 0.4]) / np.linalg.norm([-0.2, 1.0, 0.4])  # slopes summed: (0.2, -0.4)
    np.testing.assert_allclose(out[0, 4:7], nrm, rtol=1e-5)


def test_surface_bilinear_texel_centres_and_repeat(oracle):
    """GL_LINEAR + GL_REPEAT: texel centres return the texel; the field repeats every planeSize."""
    n, L = 16, 8.0
    rng = np.random.default_rng(3)
    h = rng.standard_normal((n, n, 4)).astype(np.float32)
    _, d, j = _flat_maps(n)
    c = [(h, d, j, L, 0.0)]
    ij = np.array([[3, 5], [0, 0], [15, 15], [7, 0]])
    xz = ((ij + 0.5) / n * L).astype(np.float32)  # texel centres (x from i, z from j)
    out = oracle.surface_points(c, xz)
    np.testing.assert_allclose(out[:, 1], h[ij[:, 1], ij[:, 0], 0], rtol=1e-6, atol=1e-6)
    shifted = oracle.surface_points(c, xz + np.float32(L) * np.array([[3, -2]], np.float32))
    np.testing.assert_allclose(shifted[:, 1], out[:, 1], rtol=1e-5, atol=1e-5)


def test_surface_vertex_stage_is_sequential(oracle):
    """Cascade i samples where cascades < i already moved the vertex (waveShader.glsl:101-110)."""
    n = 16
    h1, d1, j1 = _flat_maps(n, dx=4.0)  # first cascade moves x by 4 * scale
    h2 = np.zeros((n, n, 4), np.float32)
    h2[:, :, 0] = np.arange(n, dtype=np.float32)[None, :]  # height ramps with x in cascade 2
    _, d2, j2 = _flat_maps(n)
    c = [(h1, d1, j1, 16.0, 1.0), (h2, d2, j2, 16.0, 1.0)]
    out = oracle.surface_points(c, np.array([[0.5, 0.5]], np.float32))  # texel (0, 0) centre
    assert out[0, 0] == np.float32(4.5) and out[0, 1] == np.float32(4.0)  # sampled at texel 4


def test_spectrum_texels_equal_whole_image(oracle):
    """The sampled h0 entry point (used at N = 16384, where the whole image would take minutes) is
    the whole-image generateSpectrum body, bit for bit, including the k = 0 and Nyquist texels."""
    import numpy as np

    n = 64
    s = oracle.default_settings(planeSize=17.0)
    full = oracle.generate_spectrum(s, n)
    y, x = np.meshgrid(np.arange(n), np.arange(n), indexing="ij")
    xy = np.stack([x.ravel(), y.ravel()], axis=1)
    assert np.array_equal(oracle.spectrum_texels(s, n, xy).reshape(n, n, 4), full)
    assert np.array_equal(oracle.spectrum_texels(s, n, xy[[0, n * n // 2 + n // 2]]),
                          full.reshape(-1, 4)[[0, n * n // 2 + n // 2]])
