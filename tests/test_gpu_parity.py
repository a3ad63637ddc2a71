"""GPU parity: liboceanfft.so (HIP, gfx950) against the CPU oracle on the same seeded inputs.

Every call goes through the C ABI (include/oceanfft.h) via oceansimulation_amd.capi; the oracle is
only the checker. Tolerances and metrics: tests/parity.py.
"""
import os
import subprocess

import numpy as np
import pytest

import numpy_ref as R
from parity import FFT_TOL, FRAME_TOL, FRAME_TOL_GPU, H0_TOL, channel_err, lane_err, scalar_err

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def ocean():
    import oceansimulation_amd as o
    from oceansimulation_amd import capi

    assert capi.lib().ocean_device_count() > 0, "no GPU visible to liboceanfft.so"
    return o


def _rand_image(n, seed):
    rng = np.random.default_rng(seed)
    return rng.standard_normal((n, n, 4)).astype(np.float32)


def _gpu_ifft(ocean, img):
    from oceansimulation_amd.hip import DeviceBuffer

    n = img.shape[0]
    fft = ocean.FFTCalculator(n)
    buf = DeviceBuffer.from_array(img)
    fft.EncodeIFFT(buf.ptr)
    fft.synchronize()
    out = buf.to_host(img.shape)
    buf.free()
    fft.close()
    return out


# ---- Hash: bit exact (spectrum.compute:109-117) --------------------------------------------
def test_hash_bit_exact(ocean, oracle):
    from oceansimulation_amd.hip import DeviceBuffer

    rng = np.random.default_rng(7)
    xy = rng.integers(0, 2**32, size=(4096, 2), dtype=np.uint64).astype(np.uint32)
    xy[:8] = [[0, 0], [1, 0], [0, 1], [12342, 8934], [12342 + 16384, 8934 + 16384],
              [2**32 - 1, 2**32 - 1], [2**31, 7], [5, 2**31]]
    dxy = DeviceBuffer.from_array(xy)
    raw = DeviceBuffer(4 * len(xy))
    uv = DeviceBuffer(8 * len(xy))
    ocean.waves.debug_hash(dxy.ptr, len(xy), raw.ptr, uv.ptr)
    from oceansimulation_amd import hip
    hip.synchronize()
    g_raw = raw.to_host((len(xy),), np.uint32)
    g_uv = uv.to_host((len(xy), 2), np.float32)
    u0, u1, n = R.hash2(xy[:, 0], xy[:, 1])
    assert np.array_equal(g_raw, n)
    assert np.array_equal(g_uv[:, 0].view(np.uint32), u0.view(np.uint32))
    assert np.array_equal(g_uv[:, 1].view(np.uint32), u1.view(np.uint32))
    for i in range(16):
        a, b, r = oracle.hash_uv(int(xy[i, 0]), int(xy[i, 1]))
        assert r == int(g_raw[i]) and np.float32(a) == g_uv[i, 0] and np.float32(b) == g_uv[i, 1]


# ---- generateSpectrum (spectrum.compute:157-172) ---------------------------------------------
@pytest.mark.parametrize("n", [16, 64, 256, 1024, 4096])
@pytest.mark.parametrize("plane", [5.0, 17.0, 40.0, 101.0])
def test_generate_spectrum(ocean, oracle, n, plane):
    """h0 against the oracle, also weighted by |k|: the slope and choppy-derivative channels
    multiply h0 by up to |k| (~10^3 rad/m), so an error at small-amplitude high-k texels that
    max|err|/max|h0| hides shows up in the maps (the anti-wind cos(theta/2)^(2s) factor once did
    exactly that with a hardware cosine)."""
    fft = ocean.FFTCalculator(n)
    gen = ocean.Generator(fft, 1)
    ocean.apply_settings(gen.GetOceanSettings(0), planeSize=plane)
    gen.GenerateSpectrum()
    got = gen.initial_spectrum_host(0)
    ref = oracle.generate_spectrum(oracle.default_settings(planeSize=plane), n)
    assert np.isfinite(got).all()
    errs = lane_err(got, ref)
    assert max(errs) <= H0_TOL, errs
    y, x = np.meshgrid(np.arange(n), np.arange(n), indexing="ij")
    k = np.hypot(x - n / 2, y - n / 2)[..., None]
    assert max(lane_err(got * k, ref * k)) <= 10 * H0_TOL, (n, plane, lane_err(got * k, ref * k))


# ---- EncodeIFFT (src/FFTCalculator.cpp:73-114) ----------------------------------------------
@pytest.mark.parametrize("n", [16, 32, 64, 128, 256, 512, 1024, 2048])
def test_encode_ifft_vs_oracle(ocean, oracle, n):
    img = _rand_image(n, n)
    got = _gpu_ifft(ocean, img)
    ref = oracle.encode_ifft(img)
    errs = lane_err(got, ref)
    assert max(errs) <= FFT_TOL, errs


@pytest.mark.parametrize("n", [4096, 8192])
def test_encode_ifft_large_vs_float64(ocean, n):
    """Full-size transform against numpy float64 (the oracle's radix-2 is too slow here)."""
    img = _rand_image(n, 99)
    got = _gpu_ifft(ocean, img)
    ref = R.encode_ifft(img)
    errs = lane_err(got, ref)
    assert max(errs) <= FFT_TOL, errs


@pytest.mark.parametrize("n", [8192, 16384])
def test_encode_ifft_separable_vs_float64(ocean, n):
    """EncodeIFFT at the slab sizes (16384: rows, then the four-step column transform through its
    work slab) on an input that is a sum of two outer products per lane, whose float64 reference is
    the sum of the outer products of the two 1D transforms: N^2 ifft2(ifftshift(a b^T)) =
    (N ifft(ifftshift a)) (N ifft(ifftshift b))^T. Checked on 256 random rows."""
    from oceansimulation_amd.hip import DeviceBuffer

    rng = np.random.default_rng(n)
    a = rng.standard_normal((2, 2, n)) + 1j * rng.standard_normal((2, 2, n))  # [term, lane, y]
    b = rng.standard_normal((2, 2, n)) + 1j * rng.standard_normal((2, 2, n))  # [term, lane, x]
    img = np.empty((n, n, 4), np.float32)
    for lane in range(2):
        m = np.einsum("ty,tx->yx", a[:, lane].astype(np.complex64), b[:, lane].astype(np.complex64))
        img[..., 2 * lane] = m.real
        img[..., 2 * lane + 1] = m.imag
        del m
    a64 = a[:, :, :].astype(np.complex64).astype(np.complex128)  # the values the GPU sees
    b64 = b[:, :, :].astype(np.complex64).astype(np.complex128)
    fa = n * np.fft.ifft(np.fft.ifftshift(a64, axes=-1), axis=-1)
    fb = n * np.fft.ifft(np.fft.ifftshift(b64, axes=-1), axis=-1)
    fft = ocean.FFTCalculator(n)
    buf = DeviceBuffer.from_array(img)
    del img
    fft.EncodeIFFT(buf.ptr)
    fft.synchronize()
    got = buf.to_host((n, n, 4))
    rows = np.sort(rng.choice(n, 256, replace=False))
    for lane in range(2):
        ref = np.einsum("ty,tx->yx", fa[:, lane, rows], fb[:, lane])
        g = got[rows][..., 2 * lane] + 1j * got[rows][..., 2 * lane + 1]
        err = np.abs(g - ref).max() / np.abs(ref).max()
        assert err <= FFT_TOL, (n, lane, err)


@pytest.mark.parametrize("n,b", [(512, 5), (4096, 10), (8192, 3)])
def test_encode_ifft_batch_matches_single(ocean, n, b):
    """Batched == one image at a time, bit for bit (at 4096: the column-first path through its
    work image, in chunks of 8 images, so 10 images cross a chunk boundary; at 8192: the pre-stage
    path, chunks of 2)."""
    from oceansimulation_amd.hip import DeviceBuffer

    imgs = np.stack([_rand_image(n, 100 + i) for i in range(b)])
    fft = ocean.FFTCalculator(n)
    buf = DeviceBuffer.from_array(imgs)
    fft.encode_ifft_batch(buf.ptr, b)
    fft.synchronize()
    got = buf.to_host(imgs.shape)
    for i in range(b):
        single = _gpu_ifft(ocean, imgs[i])
        assert np.array_equal(got[i], single)


# ---- FFT known-answer tests (size-independent properties) --------------------------------
@pytest.mark.parametrize("n", [256, 4096])
def test_kat_delta_and_plane_wave(ocean, n):
    img = np.zeros((n, n, 4), np.float32)
    # delta at the centred DC (index N/2, N/2 after the reference's fftShift convention) -> constant
    img[n // 2, n // 2, 0] = 1.0
    # a single bin on lane 2 -> plane wave exp(+2 pi i (kx x + ky y)/N)
    kx, ky = 3, n // 2 - 5
    img[n // 2 + ky, n // 2 + kx, 2] = 1.0
    got = _gpu_ifft(ocean, img)
    assert np.allclose(got[..., 0], 1.0, atol=1e-6) and np.allclose(got[..., 1], 0.0, atol=1e-6)
    y, x = np.meshgrid(np.arange(n), np.arange(n), indexing="ij")
    ph = 2 * np.pi * ((kx * x + ky * y) % n) / n
    assert np.max(np.abs(got[..., 2] - np.cos(ph))) < 2e-5
    assert np.max(np.abs(got[..., 3] - np.sin(ph))) < 2e-5


@pytest.mark.parametrize("n", [1024, 4096])
def test_property_parseval_linearity_hermitian(ocean, n):
    rng = np.random.default_rng(5)
    a = rng.standard_normal((n, n, 4)).astype(np.float32)
    b = rng.standard_normal((n, n, 4)).astype(np.float32)
    fa, fb = _gpu_ifft(ocean, a), _gpu_ifft(ocean, b)
    fab = _gpu_ifft(ocean, (2.0 * a - 0.5 * b).astype(np.float32))
    # linearity
    assert max(lane_err(fab, 2.0 * fa.astype(np.float64) - 0.5 * fb.astype(np.float64))) < FFT_TOL
    # Parseval with the unnormalised N^2 factor: sum |y|^2 = N^2 sum |x|^2 per lane
    for lane in range(2):
        ex = np.sum(a[..., 2 * lane:2 * lane + 2].astype(np.float64) ** 2)
        ey = np.sum(fa[..., 2 * lane:2 * lane + 2].astype(np.float64) ** 2)
        assert abs(ey / (n * n * ex) - 1.0) < 1e-5
    # Hermitian input (in the shifted index convention) -> real output
    z = a[..., 0] + 1j * a[..., 1]
    zs = np.fft.ifftshift(z)
    herm = 0.5 * (zs + np.conj(np.roll(np.flip(zs, (0, 1)), 1, (0, 1))))
    hz = np.fft.fftshift(herm)
    h = np.zeros_like(a)
    h[..., 0], h[..., 1] = hz.real, hz.imag
    fh = _gpu_ifft(ocean, h)
    assert np.max(np.abs(fh[..., 1])) < 2e-5 * np.max(np.abs(fh[..., 0]))


# ---- Full CalculateOcean frames (src/Generator.cpp:45-83) -----------------------------------
def _f64_frame(o):
    """The frame of OracleGenerator o with its FFT in float64: the oracle's fp32 h0 and prepareFFT at
    o's time (the reference's arithmetic), N^2 ifft2(ifftshift) in float64 (the meaning of
    src/FFTCalculator.cpp:73-114), foam from those maps (spectrum.compute:246-259)."""
    from oracle import oracle as O

    hp, dp = O.prepare_fft(o.settings, o.n, o.h0)
    h64, d64 = R.encode_ifft(hp), R.encode_ifft(dp)
    return h64, d64, R.compute_foam(o.settings, d64)


def _frame_check(got_h, got_d, got_j, o):
    """Against the oracle per lane and per channel (FRAME_TOL), and per channel against the float64
    transform of the oracle's spectrum (FRAME_TOL_GPU; tests/parity.py)."""
    eh, ed = lane_err(got_h, o.height), lane_err(got_d, o.disp)
    ej = scalar_err(got_j - 1.0, o.jac - 1.0)
    assert max(eh + ed) <= FRAME_TOL and ej <= FRAME_TOL, (eh, ed, ej)
    # SURVEY §8(c)'s bar for the full pipeline: per channel against the oracle
    eo = channel_err(got_h, o.height) + channel_err(got_d, o.disp)
    assert max(eo) <= FRAME_TOL, eo
    h64, d64, j64 = _f64_frame(o)
    ec = channel_err(got_h, h64) + channel_err(got_d, d64)
    ej64 = scalar_err(got_j - 1.0, j64 - 1.0)
    assert max(ec) <= FRAME_TOL_GPU and ej64 <= FRAME_TOL_GPU, (ec, ej64)


@pytest.mark.parametrize("n", [64, 256, 1024])
def test_calculate_ocean_three_cascades(ocean, oracle, n):
    """WaveApp's scene (src/Waves.cpp:20-39) as one batched generator, 4 frames at dt = 1/60."""
    planes = [5.0, 17.0, 101.0]
    fft = ocean.FFTCalculator(n)
    gen = ocean.Generator(fft, 3)
    refs = []
    for c, L in enumerate(planes):
        kw = dict(planeSize=L, boundWavelength=1, wavelengthMax=L / 2.0,
                  wavelengthMin=0.0 if c == 0 else planes[c - 1] / 2.0)
        ocean.apply_settings(gen.GetOceanSettings(c), **kw)
        refs.append(oracle.OracleGenerator(n, oracle.default_settings(**kw)))
    for f in range(4):
        gen.CalculateOcean(1.0 / 60.0, update_ocean=(f == 0))
        for r in refs:
            r.calculate_ocean(1.0 / 60.0, update_ocean=(f == 0))
    for c in range(3):
        assert gen.GetOceanSettings(c).time == refs[c].settings.time
        _frame_check(gen.height_map_host(c), gen.displacement_map_host(c), gen.jacobian_map_host(c), refs[c])


@pytest.mark.parametrize("n", [256, 2048])
def test_calculate_ocean_default_t1(ocean, oracle, n):
    """Default settings (L = 40 m) at t = 1.0 s: the configuration the golden fixtures pin."""
    fft = ocean.FFTCalculator(n)
    gen = ocean.Generator(fft, 1)
    gen.CalculateOcean(1.0)
    ref = oracle.OracleGenerator(n)
    ref.calculate_ocean(1.0)
    _frame_check(gen.height_map_host(0), gen.displacement_map_host(0), gen.jacobian_map_host(0), ref)


@pytest.mark.parametrize("n", [16, 32, 128, 512, 4096])
def test_calculate_ocean_every_kernel_shape(ocean, oracle, n):
    """Full frames at the sizes whose kernels differ in shape from the ones above (first-stage
    radix 2/4/8/16, blocks of 1-4 texels, strips per workgroup, KEEP 16/4), two frames so the
    second reuses h0 (src/Generator.cpp:55-59)."""
    fft = ocean.FFTCalculator(n)
    gen = ocean.Generator(fft, 1)
    ocean.apply_settings(gen.GetOceanSettings(0), planeSize=23.0)
    ref = oracle.OracleGenerator(n, oracle.default_settings(planeSize=23.0))
    for dt in (0.75, 1.0 / 60.0):
        gen.CalculateOcean(dt)
        ref.calculate_ocean(dt)
    _frame_check(gen.height_map_host(0), gen.displacement_map_host(0), gen.jacobian_map_host(0), ref)


@pytest.mark.parametrize("half", [True, False])
def test_calculate_ocean_8192_vs_float64(ocean, oracle, half):
    """A full frame at 8192^2 (blocks of 2 texels, 4-stage transforms; half: the strip-dealt
    half-spectrum path with its transposes, else the full-spectrum path with KEEP 0): h0 and the
    packed spectra from the oracle, their transform in float64 (N^2 ifft2(ifftshift), the meaning
    of src/FFTCalculator.cpp:73-114; the oracle's own fp32 radix-2 is 6e-7 from it at 4096), foam
    from the float64 maps (spectrum.compute:246-259)."""
    import numpy_ref as R

    n, L = 8192, 61.0
    fft = ocean.FFTCalculator(n)
    gen = ocean.Generator(fft, 1)
    gen.set_half_spectrum(half)
    ocean.apply_settings(gen.GetOceanSettings(0), planeSize=L)
    gen.CalculateOcean(1.25)
    s = oracle.default_settings(planeSize=L)
    s.time = 1.25
    hp, dp = oracle.prepare_fft(s, n, oracle.generate_spectrum(s, n))
    h64, d64 = R.encode_ifft(hp), R.encode_ifft(dp)
    ec = channel_err(gen.height_map_host(0), h64) + channel_err(gen.displacement_map_host(0), d64)
    assert max(ec) <= FRAME_TOL_GPU, ec
    assert scalar_err(gen.jacobian_map_host(0) - 1.0, R.compute_foam(s, d64) - 1.0) <= FRAME_TOL_GPU


@pytest.mark.parametrize("n", [1024, 2048, 4096])
def test_half_spectrum_path_matches_full_path_and_oracle(ocean, oracle, n):
    """The half-spectrum frame (5 fields over the u >= 0 half, Hermitian rebuild, Nyquist-row
    term) against the full-spectrum frame and the oracle, over several frames and 3 cascades."""
    planes = [5.0, 23.0, 101.0]
    fft = ocean.FFTCalculator(n)
    gh, gf = ocean.Generator(fft, 3), ocean.Generator(fft, 3)
    gf.set_half_spectrum(False)
    assert gh.frame_bytes()[0] < 30 and gf.frame_bytes() == (48.0, 68.0)
    refs = []
    for c, L in enumerate(planes):
        for g in (gh, gf):
            ocean.apply_settings(g.GetOceanSettings(c), planeSize=L)
        refs.append(oracle.OracleGenerator(n, oracle.default_settings(planeSize=L)))
    for dt in (0.6, 1.0 / 60.0):
        gh.CalculateOcean(dt)
        gf.CalculateOcean(dt)
        for r in refs:
            r.calculate_ocean(dt)
    for c in range(3):
        for get in ("height_map_host", "displacement_map_host"):
            a, b = getattr(gh, get)(c), getattr(gf, get)(c)
            assert max(lane_err(a, b)) <= 1e-5, (c, get, lane_err(a, b))
        _frame_check(gh.height_map_host(c), gh.displacement_map_host(c), gh.jacobian_map_host(c), refs[c])


def test_frames_deterministic_run_twice(ocean):
    """The same frames computed twice (two generators, the bench's 8 x 4096^2 batch: persistent
    grids, the H scratch shared by the workgroups of a CU slot) are bit-identical: no result depends on
    scheduling. A build that passed the column pass's piece offsets in the buffer instructions' SGPR
    offset field differed in ~3 % of the floats from run to run (tools/microbench/detbench,
    profiles/r03_detbench_*.log); production folds them into the VGPR offset."""
    n, planes = 4096, [5.0, 17.0, 101.0, 251.0, 509.0, 1021.0, 2039.0, 4093.0]
    fft = ocean.FFTCalculator(n)
    runs = []
    for _ in range(2):
        gen = ocean.Generator(fft, len(planes))
        for c, L in enumerate(planes):
            ocean.apply_settings(gen.GetOceanSettings(c), planeSize=L)
        for dt in (0.5, 1.0 / 60.0):
            gen.CalculateOcean(dt)
        runs.append(gen)
    for c in range(len(planes)):
        for get in ("height_map_host", "displacement_map_host", "jacobian_map_host"):
            assert np.array_equal(getattr(runs[0], get)(c), getattr(runs[1], get)(c)), (c, get)


def test_sixty_four_cascades_in_one_launch(ocean):
    """The ABI's cascade limit (OCEAN_MAX_CASCADES = 64) in one batched generator: every cascade
    equals the same cascade computed alone, bit for bit; 65 is rejected."""
    from oceansimulation_amd.capi import OceanError

    n = 64
    fft = ocean.FFTCalculator(n)
    gen = ocean.Generator(fft, 64)
    for c in range(64):
        ocean.apply_settings(gen.GetOceanSettings(c), planeSize=3.0 + 7.0 * c, seed=(100 + c, 7 * c))
    gen.CalculateOcean(0.5)
    for c in (0, 17, 63):
        one = ocean.Generator(fft, 1)
        ocean.apply_settings(one.GetOceanSettings(0), planeSize=3.0 + 7.0 * c, seed=(100 + c, 7 * c))
        one.CalculateOcean(0.5)
        assert np.array_equal(gen.height_map_host(c), one.height_map_host(0))
        assert np.array_equal(gen.jacobian_map_host(c), one.jacobian_map_host(0))
    with pytest.raises(OceanError):
        ocean.Generator(fft, 65)


def test_calculate_ocean_long_time(ocean, oracle):
    """An hour of simulated time. The phase w*t (spectrum.compute:198) multiplies any ulp of w by
    t, so |k| and w are computed bit-identically to the oracle (correctly rounded sqrt, unfused
    float order); the frame error must stay at the t ~ 0 level, not grow with t."""
    planes = [5.0, 101.0]
    fft = ocean.FFTCalculator(256)
    gen = ocean.Generator(fft, len(planes))
    refs = []
    for c, L in enumerate(planes):
        ocean.apply_settings(gen.GetOceanSettings(c), planeSize=L)
        refs.append(oracle.OracleGenerator(256, oracle.default_settings(planeSize=L)))
    for dt in (600.0, 3000.0):
        gen.CalculateOcean(dt)
        for r in refs:
            r.calculate_ocean(dt)
        for c in range(len(planes)):
            assert gen.GetOceanSettings(c).time == refs[c].settings.time
            _frame_check(gen.height_map_host(c), gen.displacement_map_host(c), gen.jacobian_map_host(c), refs[c])


def test_batched_cascades_equal_individual(ocean):
    """A cascade's maps do not depend on which batch it runs in (bit-exact)."""
    n = 512
    planes = [5.0, 17.0, 101.0, 251.0]
    fft = ocean.FFTCalculator(n)
    batch = ocean.Generator(fft, len(planes))
    for c, L in enumerate(planes):
        ocean.apply_settings(batch.GetOceanSettings(c), planeSize=L, seed=(12342 + 4097 * c, 8934))
    batch.CalculateOcean(0.75)
    for c, L in enumerate(planes):
        one = ocean.Generator(fft, 1)
        ocean.apply_settings(one.GetOceanSettings(0), planeSize=L, seed=(12342 + 4097 * c, 8934))
        one.CalculateOcean(0.75)
        assert np.array_equal(one.height_map_host(0), batch.height_map_host(c))
        assert np.array_equal(one.displacement_map_host(0), batch.displacement_map_host(c))
        assert np.array_equal(one.jacobian_map_host(0), batch.jacobian_map_host(c))


@pytest.mark.parametrize("n", [2048, 4096])
def test_half_strip_shape_bit_exact_across_cascade_counts(ocean, n):
    """At 2048 and 4096 the column pass runs on half strips (FB = 2 fields, 2T-thread workgroups) when
    a launch holds <= 2 cascades and on whole strips above (launch_common.h half_fields_fb). A
    cascade's maps and Jacobian are bit-identical in 1-, 2- and 3-cascade generators, for plain
    frames and for the fused re-seed frames of the reference app's loop (src/Generator.cpp:45-83,
    src/Waves.cpp:91-94)."""
    planes = [5.0, 251.0, 4093.0]
    fft = ocean.FFTCalculator(n)
    gens = {k: ocean.Generator(fft, k) for k in (1, 2, 3)}
    for k, g in gens.items():
        g.set_h0_memo(False)
        for c in range(k):
            ocean.apply_settings(g.GetOceanSettings(c), planeSize=planes[c], seed=(12342 + 4097 * c, 8934))
    for dt, upd in ((0.5, False), (1.0 / 60.0, True), (1.0 / 60.0, False)):
        for g in gens.values():
            g.CalculateOcean(dt, update_ocean=upd)
        for k in (1, 2):
            for c in range(k):
                for get in ("height_map_host", "displacement_map_host", "jacobian_map_host"):
                    assert np.array_equal(getattr(gens[k], get)(c), getattr(gens[3], get)(c)), (dt, upd, k, c, get)
    for g in gens.values():
        g.close()
    fft.close()


def test_update_spectrum_semantics(ocean, oracle):
    """h0 is regenerated on the first call and when update_ocean is set (src/Generator.cpp:55-59)."""
    n = 128
    fft = ocean.FFTCalculator(n)
    gen = ocean.Generator(fft, 1)
    gen.CalculateOcean(0.5)
    h0_a = gen.initial_spectrum_host(0)
    ocean.apply_settings(gen.GetOceanSettings(0), U_10=20.0)
    gen.CalculateOcean(0.5)  # settings changed but no update flag: h0 unchanged
    assert np.array_equal(gen.initial_spectrum_host(0), h0_a)
    gen.CalculateOcean(0.5, update_ocean=True)
    ref = oracle.generate_spectrum(oracle.default_settings(U_10=20.0), n)
    assert max(lane_err(gen.initial_spectrum_host(0), ref)) <= H0_TOL
    assert gen.GetOceanSettings(0).time == np.float32(1.5)


def test_fused_reseed_frames(ocean, oracle):
    """CalculateOcean(dt, update=True) on the half-spectrum path evaluates h0 inside the column pass
    (the reference app's every-frame re-seed, src/Waves.cpp:91-94) without writing the h0 image.
    Frames match the oracle; the h0 image, materialised on the next plain frame or on the getter,
    holds the settings of the re-seed, not later edits (src/Generator.cpp:55-59)."""
    n, planes = 1024, [5.0, 23.0, 101.0]
    fft = ocean.FFTCalculator(n)
    fused, plain = ocean.Generator(fft, 3), ocean.Generator(fft, 3)
    fused.set_h0_memo(False)  # re-seed on every request (unchanged settings would skip it)
    refs = []
    for c, L in enumerate(planes):
        for g in (fused, plain):
            ocean.apply_settings(g.GetOceanSettings(c), planeSize=L)
        refs.append(oracle.OracleGenerator(n, oracle.default_settings(planeSize=L)))
    for dt in (0.4, 1.0 / 60.0):
        fused.CalculateOcean(dt, update_ocean=True)
        plain.GenerateSpectrum()
        plain.CalculateOcean(dt)
        for r in refs:
            r.calculate_ocean(dt, update_ocean=True)
    for c in range(3):
        for get in ("height_map_host", "displacement_map_host"):
            assert max(lane_err(getattr(fused, get)(c), getattr(plain, get)(c))) <= 1e-5, (c, get)
        _frame_check(fused.height_map_host(c), fused.displacement_map_host(c), fused.jacobian_map_host(c), refs[c])
    # an edit without the update flag: the next frame evolves the re-seeded h0 (materialised now)
    for g in (fused, plain):
        ocean.apply_settings(g.GetOceanSettings(0), U_10=20.0)
        g.CalculateOcean(0.1)
    assert np.array_equal(fused.initial_spectrum_host(0), plain.initial_spectrum_host(0))
    assert max(lane_err(fused.height_map_host(0), plain.height_map_host(0))) <= 1e-5
    fused.CalculateOcean(0.0, update_ocean=True)  # getter after a fused frame: the new settings
    ref = oracle.generate_spectrum(oracle.default_settings(U_10=20.0, planeSize=5.0), n)
    assert max(lane_err(fused.initial_spectrum_host(0), ref)) <= H0_TOL


@pytest.mark.parametrize("n,cascades", [(1024, 3), (4096, 1)])
def test_frame_overlap_bit_identical(ocean, n, cascades):
    """ocean_generator_set_frame_overlap: frame f + 1's column pass runs on an internal stream into a
    second field slot beside frame f's row pass. Frames issued back to back without synchronising —
    plain frames, the reference app's fused re-seeds (src/Waves.cpp:91-94, memo off), an h0 edit
    with the update flag, h0 written through the getter's pointer, and the mode switched off and on
    again — give the serial generator's bits (maps and Jacobian), frame for frame."""
    fft = ocean.FFTCalculator(n)
    ov, ser = ocean.Generator(fft, cascades), ocean.Generator(fft, cascades)
    for g in (ov, ser):
        g.set_h0_memo(False)
        for c in range(cascades):
            ocean.apply_settings(g.GetOceanSettings(c), planeSize=[5.0, 17.0, 101.0][c % 3] * (1 + c // 3))
    ov.set_frame_overlap(True)

    def same(tag):
        for c in range(cascades):
            for get in ("height_map_host", "displacement_map_host", "jacobian_map_host"):
                assert np.array_equal(getattr(ov, get)(c), getattr(ser, get)(c)), (tag, c, get)

    script = [(1.0 / 60.0, False), (0.5, False), (1.0 / 60.0, True), (1.0 / 60.0, False), (2.0, True),
              (1.0 / 60.0, False), (1.0 / 60.0, False)]
    for k, (dt, upd) in enumerate(script):
        if k == 4:
            for g in (ov, ser):
                ocean.apply_settings(g.GetOceanSettings(0), U_10=25.0)
        for g in (ov, ser):
            g.CalculateOcean(dt, update_ocean=upd)
        if k in (1, 4, 6):
            same(("frame", k))
    # the h0 getter (the caller may write through its pointer): the next column pass waits for it
    h0 = ov.initial_spectrum_host(0)
    for g in (ov, ser):
        g.CalculateOcean(1.0 / 60.0)
        g.CalculateOcean(1.0 / 60.0)
    same("after getter")
    ov.set_frame_overlap(False)
    for g in (ov, ser):
        g.CalculateOcean(1.0 / 60.0, update_ocean=True)
        g.CalculateOcean(1.0 / 60.0)
    same("overlap off")
    ov.set_frame_overlap(True)
    for _ in range(3):
        for g in (ov, ser):
            g.CalculateOcean(1.0 / 30.0)
    same("overlap on again")
    assert h0.shape[0] > 0
    # the mode exists on the blocked half path only
    full = ocean.Generator(fft, 1)
    full.set_half_spectrum(False)
    with pytest.raises(RuntimeError):
        full.set_frame_overlap(True)


def test_h0_memo_skips_identical_reseeds(ocean, oracle):
    """The reference app requests a re-seed every frame (src/Waves.cpp:91-94). With unchanged h0
    inputs the re-seed is skipped (default): frames are bit-identical to frames without the request;
    an edit of any h0 input (here U_10, then planeSize) with the request re-seeds (h0 equals the
    oracle's for the new settings); `time` alone never re-seeds."""
    n = 256
    fft = ocean.FFTCalculator(n)
    memo, plain = ocean.Generator(fft, 2), ocean.Generator(fft, 2)
    for g in (memo, plain):
        ocean.apply_settings(g.GetOceanSettings(1), planeSize=17.0)
    for dt in (0.5, 1.0 / 60.0, 1.0 / 60.0):
        memo.CalculateOcean(dt, update_ocean=True)
        plain.CalculateOcean(dt)
        for c in range(2):
            assert np.array_equal(memo.height_map_host(c), plain.height_map_host(c))
            assert np.array_equal(memo.displacement_map_host(c), plain.displacement_map_host(c))
    ocean.apply_settings(memo.GetOceanSettings(0), U_10=20.0)
    memo.CalculateOcean(1.0 / 60.0, update_ocean=True)
    ref = oracle.generate_spectrum(oracle.default_settings(U_10=20.0), n)
    assert max(lane_err(memo.initial_spectrum_host(0), ref)) <= H0_TOL
    ocean.apply_settings(memo.GetOceanSettings(1), planeSize=23.0)
    memo.CalculateOcean(1.0 / 60.0, update_ocean=True)
    ref = oracle.generate_spectrum(oracle.default_settings(planeSize=23.0), n)
    assert max(lane_err(memo.initial_spectrum_host(1), ref)) <= H0_TOL
    memo.close()
    plain.close()
    fft.close()


def test_errors_fail_loudly(ocean):
    from oceansimulation_amd.capi import OceanError

    with pytest.raises(OceanError):
        ocean.FFTCalculator(300)
    with pytest.raises(OceanError):
        ocean.FFTCalculator(32768)
    fft = ocean.FFTCalculator(64)
    with pytest.raises(OceanError):
        ocean.Generator(fft, 0)
    with pytest.raises(OceanError):
        ocean.Generator(fft, 65)


def test_cpp_dropin_binary():
    """The C++ Waves:: drop-in (reference signatures) driven like WaveApp, checked vs the oracle."""
    exe = os.path.join(ROOT, "tests", "cpp", "test_waves")
    assert os.path.exists(exe), "build with `make` first"
    r = subprocess.run([exe, "256", "3"], capture_output=True, text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr


# ---- committed golden vectors (tests/golden/make_golden.py) ---------------------------------
def test_golden_fixtures_gpu(ocean):
    import json

    gdir = os.path.join(ROOT, "tests", "golden")
    z = np.load(os.path.join(gdir, "ocean_golden.npz"))
    manifest = json.load(open(os.path.join(gdir, "manifest.json")))
    for name, case in manifest["cases"].items():
        fft = ocean.FFTCalculator(case["n"])
        gen = ocean.Generator(fft, 1)
        ocean.apply_settings(gen.GetOceanSettings(0), **case["settings"])
        for dt in case["timesteps"]:
            gen.CalculateOcean(dt)
        assert gen.GetOceanSettings(0).time == np.float32(case["final_time"])
        assert max(lane_err(gen.initial_spectrum_host(0), z[f"{name}/h0"])) <= H0_TOL, name
        assert max(lane_err(gen.height_map_host(0), z[f"{name}/height"])) <= FRAME_TOL, name
        assert max(lane_err(gen.displacement_map_host(0), z[f"{name}/disp"])) <= FRAME_TOL, name
        assert scalar_err(gen.jacobian_map_host(0) - 1.0, z[f"{name}/jac"] - 1.0) <= FRAME_TOL, name


# ---- slab decomposition (one grid over P ranks, emulated in one process) --------------------
def _slab_run(ocean, n, ranks, steps, settings):
    from oceansimulation_amd.hip import DeviceBuffer
    from oceansimulation_amd.slab import SlabGenerator, emulate_frame

    fft = ocean.FFTCalculator(n)
    slabs = [SlabGenerator(fft, r, ranks) for r in range(ranks)]
    for g in slabs:
        ocean.apply_settings(g.GetOceanSettings(), **settings)
    sends = [DeviceBuffer(g.exchange_bytes) for g in slabs]
    recvs = [DeviceBuffer(g.exchange_bytes) for g in slabs]
    for k, dt in enumerate(steps):
        emulate_frame(slabs, sends, recvs, dt, update_ocean=(k == 0))
    h = np.concatenate([g.height_map_host() for g in slabs])
    d = np.concatenate([g.displacement_map_host() for g in slabs])
    j = np.concatenate([g.jacobian_map_host() for g in slabs])
    return h, d, j


@pytest.mark.parametrize("n,ranks", [(512, 2), (256, 2), (256, 4), (64, 4), (1024, 1), (1024, 8), (4096, 4), (2048, 16),
                                     (1024, 16)])
def test_slab_decomposition_matches_whole_grid(ocean, n, ranks):
    """Rank-split column pass + all-to-all + rank-split row pass == the single-GPU generator,
    bit for bit. N >= 1024: the strip-dealt half-spectrum path (strips dealt over the ranks, the
    fields moved to row-major after the exchange) against the whole grid's blocked half-spectrum
    path; (1024, 16) leaves the last rank without strips. N < 1024: the full-spectrum kernels."""
    settings = dict(planeSize=17.0)
    steps = [0.25, 1.0 / 60.0]
    h, d, j = _slab_run(ocean, n, ranks, steps, settings)
    fft = ocean.FFTCalculator(n)
    gen = ocean.Generator(fft, 1)
    if n < 1024:
        gen.set_half_spectrum(False)  # what slabs below 1024 run
    ocean.apply_settings(gen.GetOceanSettings(0), **settings)
    for dt in steps:
        gen.CalculateOcean(dt)
    assert np.array_equal(h, gen.height_map_host(0))
    assert np.array_equal(d, gen.displacement_map_host(0))
    assert np.array_equal(j, gen.jacobian_map_host(0))


def _whole_grid_frames(ocean, n, steps, settings):
    fft = ocean.FFTCalculator(n)
    gen = ocean.Generator(fft, 1)
    if n < 1024:
        gen.set_half_spectrum(False)  # the formulation the slabs run
    ocean.apply_settings(gen.GetOceanSettings(0), **settings)
    frames = []
    for dt in steps:
        gen.CalculateOcean(dt)
        frames.append((gen.height_map_host(0), gen.displacement_map_host(0), gen.jacobian_map_host(0)))
    return frames


@pytest.mark.parametrize("n,ranks,budget", [(512, 2, 0), (1024, 4, 200), (4096, 2, 0)])
def test_slab_pipeline_matches_whole_grid(ocean, n, ranks, budget):
    """SlabPipeline (exchange of frame f on its own stream beside the column pass of f+1 and the
    row pass of f-1, two buffer slots) == the single-GPU generator, bit for bit, frame by frame
    (maps lag one step) and after an unsynchronised run + flush."""
    import torch

    from oceansimulation_amd.slab import LocalExchangeSlots, SlabGenerator, SlabPipeline

    settings = dict(planeSize=17.0)
    steps = [0.25, 1.0 / 60.0, 0.5, 1.0 / 60.0, 2.0]
    ref = _whole_grid_frames(ocean, n, steps, settings)
    fft = ocean.FFTCalculator(n)
    fft.set_cu_budget(budget)
    slabs = [SlabGenerator(fft, r, ranks) for r in range(ranks)]
    for g in slabs:
        ocean.apply_settings(g.GetOceanSettings(), **settings)
    ex = LocalExchangeSlots(ranks, slabs[0].exchange_bytes, torch.device("cuda", 0))
    sends, recvs = ex.ptrs()

    def maps():
        torch.cuda.synchronize()
        return (np.concatenate([g.height_map_host() for g in slabs]),
                np.concatenate([g.displacement_map_host() for g in slabs]),
                np.concatenate([g.jacobian_map_host() for g in slabs]))

    pipe = SlabPipeline(slabs, sends, recvs, ex)
    for k, dt in enumerate(steps):
        pipe.step(dt, update_ocean=(k == 0))
        if k > 0:  # the row pass of frame k-1 has been issued
            for got, want in zip(maps(), ref[k - 1]):
                assert np.array_equal(got, want), f"frame {k - 1}"
    pipe.flush()
    for got, want in zip(maps(), ref[-1]):
        assert np.array_equal(got, want), "last frame"
    # unsynchronised run over the same buffers from t = 0 (fresh generators)
    slabs2 = [SlabGenerator(fft, r, ranks) for r in range(ranks)]
    for g in slabs2:
        ocean.apply_settings(g.GetOceanSettings(), **settings)
    pipe2 = SlabPipeline(slabs2, sends, recvs, ex)
    for k, dt in enumerate(steps):
        pipe2.step(dt, update_ocean=(k == 0))
    pipe2.flush()
    slabs = slabs2
    for got, want in zip(maps(), ref[-1]):
        assert np.array_equal(got, want), "unsynchronised run"


def test_16384_row_pass_resident_grid_under_cu_budget(ocean):
    """The 16384 row pass loops over rows on a resident grid (k_rows_xs EARLY 4: each image's loads
    issued before the previous image's stores, the next row's before this row's): with a CU budget of
    100 (100 workgroups, ~164 rows each) the maps equal the full device's (256 workgroups) bit for bit."""
    from oceansimulation_amd import capi

    L = capi.lib()
    n = 16384
    outs = []
    for budget in (0, 100):
        fft = ocean.FFTCalculator(n)
        fft.set_cu_budget(budget)
        gen = ocean.Generator(fft, 1)
        for dt in (0.5, 1.0 / 60.0):
            gen.CalculateOcean(dt)
        fft.synchronize()
        outs.append((fft, gen))
    from oceansimulation_amd import hip
    import torch

    for get, tex in ((L.ocean_generator_height_map, 16), (L.ocean_generator_displacement_map, 16),
                     (L.ocean_generator_jacobian_map, 4)):
        nb = n * n * tex
        a = torch.empty(nb, dtype=torch.uint8, device="cuda")
        b = torch.empty_like(a)
        hip.copy_d2d(a.data_ptr(), int(get(outs[0][1].handle, 0)), nb)
        hip.copy_d2d(b.data_ptr(), int(get(outs[1][1].handle, 0)), nb)
        assert torch.equal(a, b), get.__name__
    for fft, gen in outs:
        gen.close()
        fft.close()


def test_cu_budget_validation(ocean):
    from oceansimulation_amd.capi import OceanError

    fft = ocean.FFTCalculator(256)
    with pytest.raises(OceanError):
        fft.set_cu_budget(-1)
    with pytest.raises(OceanError):
        fft.set_cu_budget(fft.cus + 1)
    fft.set_cu_budget(1)  # one CU still computes the right answer
    gen = ocean.Generator(fft, 1)
    gen.CalculateOcean(1.0)
    h1 = gen.height_map_host(0)
    fft.set_cu_budget(0)
    gen2 = ocean.Generator(fft, 1)
    gen2.CalculateOcean(1.0)
    assert np.array_equal(h1, gen2.height_map_host(0))


def test_slab_rejects_too_narrow_slabs(ocean):
    from oceansimulation_amd.capi import OceanError
    from oceansimulation_amd.slab import SlabGenerator

    fft = ocean.FFTCalculator(64)
    with pytest.raises(OceanError):
        SlabGenerator(fft, 0, 8)  # 8-wide slabs < the 16-column work item at N = 64 (one wave's strips)
    with pytest.raises(OceanError):
        SlabGenerator(ocean.FFTCalculator(256), 0, 3)  # not a power of two


@pytest.mark.parametrize("n,ranks", [(256, 4), (1024, 4)])
def test_slab_small_grid_vs_oracle(ocean, oracle, n, ranks):
    """Slab frames (full spectrum at 256, strip-dealt half spectrum at 1024) against the oracle."""
    h, d, j = _slab_run(ocean, n, ranks, [1.0], dict(planeSize=5.0))
    ref = oracle.OracleGenerator(n, oracle.default_settings(planeSize=5.0))
    ref.calculate_ocean(1.0)
    _frame_check(h, d, j, ref)


def _sample_lines(n, extra=10, seed=16384):
    """Rows / columns 0, 1, N/2 - 1, N/2, N/2 + 1, N - 1 and `extra` random ones: 16 x 16 = 256
    sample points per map channel, including the Nyquist and k = 0 lines."""
    rng = np.random.default_rng(seed)
    fixed = [0, 1, n // 2 - 1, n // 2, n // 2 + 1, n - 1]
    rest = sorted(set(rng.integers(2, n - 2, 4 * extra).tolist()) - set(fixed))[:extra]
    return np.array(sorted(fixed + rest))


@pytest.mark.slow
@pytest.mark.parametrize("four_step", [True, False])
def test_generator_16384_sampled_vs_oracle(ocean, oracle, four_step):
    """A 16384^2 frame (too large for the whole-grid CPU oracle) at 256 sampled points per channel —
    rows and columns 0, 1, N/2 - 1, N/2, N/2 + 1, N - 1 (the k = 0 and Nyquist lines and their
    partners) and 10 random ones — against the ORACLE's h0 and prepareFFT (fp32, the reference's
    arithmetic, computed on the full spectrum in row chunks) followed by a float64 inverse DFT at the
    sample points (oracle.sampled_frame). Four-step path (default) and strip-dealt path; per-channel
    metric at FRAME_TOL_GPU."""
    n, plane, dt = 16384, 40.0, 0.25
    fft = ocean.FFTCalculator(n)
    gen = ocean.Generator(fft, 1)
    gen.set_four_step(four_step)
    ocean.apply_settings(gen.GetOceanSettings(0), planeSize=plane)
    gen.CalculateOcean(dt)
    s = oracle.default_settings(planeSize=plane)
    s.time = gen.GetOceanSettings(0).time
    xs = ys = _sample_lines(n)
    h, d, j = oracle.sampled_frame(s, n, xs, ys)
    gh = gen.height_map_host(0)[np.ix_(ys, xs)]
    gd = gen.displacement_map_host(0)[np.ix_(ys, xs)]
    gj = gen.jacobian_map_host(0)[np.ix_(ys, xs)]
    e = channel_err(gh, h) + channel_err(gd, d)
    ej = scalar_err(gj - 1.0, j - 1.0)
    assert max(e) <= FRAME_TOL_GPU and ej <= FRAME_TOL_GPU, (e, ej)
    gen.close()
    fft.close()


# ---- surface consumer (resources/waveShader.glsl), SURVEY §8f rank 3 -------------------------
def _scene(ocean, n, t=1.0, planes=(5.0, 17.0, 101.0)):
    """WaveApp's three cascades (src/Waves.cpp:20-39) as three generators, as Renderer binds them."""
    fft = ocean.FFTCalculator(n)
    gens = []
    for L in planes:
        g = ocean.Generator(fft, 1)
        ocean.apply_settings(g.GetOceanSettings(0), planeSize=L)
        g.CalculateOcean(t)
        gens.append(g)
    return fft, gens


def test_surface_points_bit_exact_vs_oracle(ocean, oracle):
    """Vertex displacement + slope normal + Jacobian average at arbitrary positions (negative,
    multi-period, texel centres and edges): bit-exact with the oracle restatement on the same maps."""
    from oceansimulation_amd.surface import SurfaceSampler, host_cascades

    fft, gens = _scene(ocean, 256)
    pairs = [(g, 0) for g in gens]
    rng = np.random.default_rng(7)
    xz = np.concatenate([rng.uniform(-300.0, 300.0, (20000, 2)),
                         np.stack(np.meshgrid(np.arange(-8, 8) * 5.0 / 256.0, [0.0, -5.0, 1e3]), -1).reshape(-1, 2)])
    xz = xz.astype(np.float32)
    got = SurfaceSampler(pairs).sample_host(xz)
    want = oracle.surface_points(host_cascades(pairs), xz)
    assert np.array_equal(got, want), np.max(np.abs(got - want))
    assert np.all(np.abs(np.linalg.norm(got[:, 4:7], axis=1) - 1.0) < 1e-6)


def test_surface_plane_mesh_vs_oracle(ocean, oracle):
    """The reference plane mesh through the camera warp (waveShader.glsl:77-98), in two checks:
    the warp alone (zero-amplitude cascades: scale = 0) within a few ulp of the oracle (its pow is
    ocml vs glibc, ~1 ulp apart; at the far field, uv ~ 1e5 texels, one ulp of position moves the
    sample visibly, so the sampled output is not compared through two different warps), then the
    sampling on the GPU's own warped positions bit-exact against the oracle."""
    from oceansimulation_amd.surface import SurfaceSampler, host_cascades

    cam = [3.0, 5.0, -2.0, -0.6, 0.8]  # WaveRenderer's camera height (src/Renderer.cpp:15)
    res = 128
    fft0, flat = _scene(ocean, 256)
    for g in flat:
        ocean.apply_settings(g.GetOceanSettings(0), scale=0.0)
        g.CalculateOcean(0.0, update_ocean=True)
    flat_pairs = [(g, 0) for g in flat]
    base = SurfaceSampler(flat_pairs).plane_host(cam, res)
    want_base = oracle.surface_plane(host_cascades(flat_pairs), cam, res)
    rel = np.abs(base[:, [0, 2]] - want_base[:, [0, 2]]) / np.maximum(1.0, np.abs(want_base[:, [0, 2]]))
    assert np.max(rel) < 2e-6, np.max(rel)
    assert np.all(base[:, 1] == 0.0) and np.allclose(base[:, 3], 1.0, atol=1e-6)  # 3 x fp32(1/3)

    fft, gens = _scene(ocean, 256)
    pairs = [(g, 0) for g in gens]
    got = SurfaceSampler(pairs).plane_host(cam, res)
    want = oracle.surface_points(host_cascades(pairs), base[:, [0, 2]].copy())
    assert np.array_equal(got, want), np.max(np.abs(got - want))


def test_surface_atlas_path_bit_exact_vs_oracle(ocean, oracle):
    """Requests of >= 4 vertices per map texel sample a repacked atlas of the maps (launch_surface,
    surface_use_atlas): the plane mesh at 1024^2 quads and 1.1 M explicit positions, bit-exact with the
    oracle as the direct path below that size; a smaller request after them takes the direct path again
    on the same plan."""
    from oceansimulation_amd.surface import SurfaceSampler, host_cascades

    cam = [3.0, 5.0, -2.0, -0.6, 0.8]
    res = 1024  # 1025^2 vertices against 3 x 256^2 texels: the atlas path
    fft0, flat = _scene(ocean, 256)
    for g in flat:
        ocean.apply_settings(g.GetOceanSettings(0), scale=0.0)
        g.CalculateOcean(0.0, update_ocean=True)
    base = SurfaceSampler([(g, 0) for g in flat]).plane_host(cam, res)
    fft, gens = _scene(ocean, 256)
    pairs = [(g, 0) for g in gens]
    sampler = SurfaceSampler(pairs)
    host = host_cascades(pairs)
    got = sampler.plane_host(cam, res)
    want = oracle.surface_points(host, base[:, [0, 2]].copy())
    assert np.array_equal(got, want), np.max(np.abs(got - want))
    rng = np.random.default_rng(11)
    xz = rng.uniform(-400.0, 400.0, (1 << 20 | 4096, 2)).astype(np.float32)
    got = sampler.sample_host(xz)
    assert np.array_equal(got, oracle.surface_points(host, xz))
    small = xz[:3000].copy()  # direct path
    assert np.array_equal(sampler.sample_host(small), got[:3000])


def test_surface_batched_generator_and_errors(ocean):
    """(generator, cascade) pairs from one batched generator equal three single generators;
    invalid requests fail loudly."""
    from oceansimulation_amd.capi import OceanError
    from oceansimulation_amd.slab import SlabGenerator
    from oceansimulation_amd.surface import SurfaceSampler

    fft, gens = _scene(ocean, 64)
    gb = ocean.Generator(fft, 3)
    for c, L in enumerate((5.0, 17.0, 101.0)):
        ocean.apply_settings(gb.GetOceanSettings(c), planeSize=L)
    gb.CalculateOcean(1.0)
    xz = np.random.default_rng(1).uniform(-50, 50, (512, 2)).astype(np.float32)
    a = SurfaceSampler([(g, 0) for g in gens]).sample_host(xz)
    b = SurfaceSampler([(gb, c) for c in range(3)]).sample_host(xz)
    assert np.array_equal(a, b)
    with pytest.raises(OceanError):
        SurfaceSampler([(gb, 3)]).sample_host(xz)
    with pytest.raises(OceanError):
        SurfaceSampler([(gens[0], 0), (ocean.Generator(ocean.FFTCalculator(128), 1), 0)]).sample_host(xz)
    with pytest.raises(OceanError):
        SurfaceSampler([(SlabGenerator(ocean.FFTCalculator(256), 0, 2), 0)]).sample_host(xz)
    with pytest.raises(OceanError):
        SurfaceSampler([(gb, 0)]).plane_host([0, 5, 0, 0, 0], 8)


# ---- headless WaveApp driver -------------------------------------------
def _run_app(tmp, *args):
    exe = os.path.join(ROOT, "examples", "waveapp_headless")
    r = subprocess.run([exe, *args, "--dump", str(tmp)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    import json

    return json.loads(r.stdout.strip().splitlines()[-1])


def test_waveapp_headless_matches_oracle(ocean, oracle, tmp_path):
    """WaveApp::OnUpdate driven headless: Q-freeze frames (dt = 0), a settings edit that re-seeds
    and redoes the wavelength bookkeeping, the renderer's surface step; the dumped maps equal the
    oracle replaying the same script, and both re-seed policies give identical maps."""
    n, frames, mesh = 64, 20, 32
    script = ["--n", str(n), "--frames", str(frames), "--freeze", "5:8", "--edit", "10:1.U_10=20",
              "--mesh", str(mesh)]
    a, b = tmp_path / "ref", tmp_path / "onedit"
    a.mkdir()
    b.mkdir()
    out = _run_app(a, *script)
    _run_app(b, *script, "--reseed", "on-edit")
    assert out["frozen_frames"] == 3 and out["reseeded_frames"] == frames
    primes = [5.0, 17.0, 101.0]
    refs = []
    for i, L in enumerate(primes):
        s = oracle.default_settings(planeSize=L, boundWavelength=1, wavelengthMax=L / 2.0,
                                    wavelengthMin=0.0 if i == 0 else primes[i - 1] / 2.0)
        refs.append(oracle.OracleGenerator(n, s))
    for f in range(frames):
        if f == 10:
            refs[1].settings.U_10 = 20.0
        dt = 0.0 if 5 <= f < 8 else np.float32(1.0 / 60.0)
        for r in refs:
            r.calculate_ocean(dt, update_ocean=True)
    for i in range(3):
        h, d, j = (np.load(a / f"{k}_{i}.npy") for k in ("height", "disp", "jac"))
        for k in ("height", "disp", "jac"):
            assert np.array_equal(np.load(a / f"{k}_{i}.npy"), np.load(b / f"{k}_{i}.npy")), (k, i)
        _frame_check(h, d, j, refs[i])
        assert np.float32(out["final_time"][i]) == refs[i].settings.time
    surf = np.load(a / "surface.npy")
    cas = [(r.height, r.disp, r.jac, L, r.settings.displacement) for r, L in zip(refs, primes)]
    want = oracle.surface_plane(cas, [0.0, 5.0, 0.0, -0.70711, 0.70711], mesh)
    near = np.hypot(want[:, 0], want[:, 2]) < 60.0
    assert near.sum() > 100
    assert np.max(np.abs(surf[near] - want[near])) < 1e-3
