"""GPU parity at the BASELINE.json configurations themselves (configs[3] and configs[4] geometry),
and bench.py's multi-rank launch on a one-GPU box.

- configs[3]: the 8 x 4096^2 batch bench.py times (same plane sizes and seeds, the persistent
  xcd-paired item mapping of an 8-cascade launch) against the oracle, and bit-exact against the
  same cascades run one per generator.
- configs[4]: the single 16384^2 grid split over 8 ranks (strip-dealt half spectrum, equal-split
  all-to-all emulated by device copies in one process) against the whole-grid generator, bit for
  bit, compared on the device (17 GB of maps never leave HBM); h0 at 16384 against the oracle on
  sampled texels (the whole image would take the CPU oracle minutes).
All compute goes through the C ABI (liboceanfft.so); the oracle is only the checker.
"""
import importlib.util
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from parity import FRAME_TOL, FRAME_TOL_GPU, H0_TOL, channel_err, lane_err, scalar_err

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def ocean():
    import oceansimulation_amd as o
    from oceansimulation_amd import capi

    assert capi.lib().ocean_device_count() > 0, "no GPU visible to liboceanfft.so"
    return o


def _bench():
    spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _dev_equal(ptr_a: int, ptr_b: int, nbytes: int) -> bool:
    """Bit-exact comparison of two device ranges without host copies (torch shares the HIP
    runtime with liboceanfft.so, see conftest.py)."""
    import torch

    from oceansimulation_amd import hip

    a = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    b = torch.empty_like(a)
    hip.copy_d2d(a.data_ptr(), ptr_a, nbytes)
    hip.copy_d2d(b.data_ptr(), ptr_b, nbytes)
    eq = bool(torch.equal(a, b))
    del a, b
    return eq


# ---- configs[0..2]: bench.py's `configs` leg ------------------------------------------------------
def test_bench_configs_leg_reports_every_small_config(ocean):
    """bench.py's `configs` leg (BASELINE configs 1-3 on one GPU beside the CPU oracle), on a few steps:
    every config reports points/s, kernel time and its roofline fraction against its own byte count
    (116 B/pt on the 256^2 full-spectrum path, 64 B per EncodeIFFT texel, 84 B/pt at 2048^2), the
    CPU oracle's rate beside it, and config 1's maps agree with the oracle's (1e-4 of each lane's max)."""
    b = _bench()
    out = b.configs_leg(steps=5, cpu_seconds=0.2)
    for k in ("config1_256_scene", "config2_1024_encode_ifft", "config3_2048_full_payload", "config3_2048_x4_cascades"):
        g, c = out[k]["gpu"], out[k]["cpu"]
        assert g["points_per_s"] > 0 and c["points_per_s"] > 0, k
        assert 0.0 < g["frac_hbm_peak"] < 1.0, (k, g)
        assert out[k]["gpu_over_cpu"] > 1.0, k
    assert out["config1_256_scene"]["gpu"]["frame_hbm_bytes_per_point"] == 116
    assert abs(out["config3_2048_full_payload"]["gpu"]["frame_hbm_bytes_per_point"] - 84.1875) < 1e-9
    assert out["config2_1024_encode_ifft"]["gpu"]["bytes_per_texel"] == 64
    assert out["config1_256_scene"]["gpu"]["verified"], out["config1_256_scene"]["gpu"]
    assert out["config3_2048_x4_cascades"]["gpu"]["points"] == 4 * 2048 * 2048


# ---- configs[3]: 8 independent 4096^2 cascades, as bench.py times them ---------------------------
def test_headline_batch_vs_oracle(ocean, oracle):
    """bench.py's step (rank 0's 8 cascades of 4096^2, plane sizes 5..4093 m) against the oracle
    after three frames (the first seeds h0): cascades 0, 3 and 7 at FRAME_TOL, and per channel at
    FRAME_TOL_GPU against the float64 transform of the oracle's spectrum; and every cascade of
    the 8-cascade launch bit-exact against the same cascade in a one-cascade generator, so the
    many-cascade item mapping is exercised (src/Generator.cpp:45-83)."""
    b = _bench()
    n, C = 4096, 8
    steps = [1.0 / 60.0] * 3
    fft = ocean.FFTCalculator(n)
    gen = ocean.Generator(fft, C)
    for c in range(C):
        ocean.apply_settings(gen.GetOceanSettings(c), **b.cascade_settings(0, c))
    for dt in steps:
        gen.CalculateOcean(dt)
    fft.synchronize()
    for c in (0, 3, 7):
        s = b.cascade_settings(0, c)
        ref = oracle.OracleGenerator(n, oracle.default_settings(**s))
        for dt in steps:
            ref.calculate_ocean(dt)
        gh, gd, gj = gen.height_map_host(c), gen.displacement_map_host(c), gen.jacobian_map_host(c)
        e = lane_err(gh, ref.height) + lane_err(gd, ref.disp)
        ej = scalar_err(gj - 1.0, ref.jac - 1.0)
        assert max(e) <= FRAME_TOL and ej <= FRAME_TOL, (c, e, ej)
        # per channel against the float64 transform of the oracle's spectrum (tests/parity.py)
        import numpy_ref as R

        hp, dp = oracle.prepare_fft(ref.settings, n, ref.h0)
        h64, d64 = R.encode_ifft(hp), R.encode_ifft(dp)
        ec = channel_err(gh, h64) + channel_err(gd, d64)
        ej64 = scalar_err(gj - 1.0, R.compute_foam(ref.settings, d64) - 1.0)
        assert max(ec) <= FRAME_TOL_GPU and ej64 <= FRAME_TOL_GPU, (c, ec, ej64)
        del ref, hp, dp, h64, d64
    for c in range(C):
        one = ocean.Generator(fft, 1)
        ocean.apply_settings(one.GetOceanSettings(0), **b.cascade_settings(0, c))
        for dt in steps:
            one.CalculateOcean(dt)
        fft.synchronize()
        for get, tex in ((ocean.Generator.GetHeightMap, 16), (ocean.Generator.GetDisplacementMap, 16),
                         (ocean.Generator.GetJacobianMap, 4)):
            assert _dev_equal(get(gen, c), get(one, 0), tex * n * n), (c, get.__name__)
        one.close()
    gen.close()
    fft.close()


# ---- configs[4]: one 16384^2 grid, 8 ranks -------------------------------------------------------
def test_h0_16384_sampled_vs_oracle(ocean, oracle):
    """generateSpectrum at N = 16384 (spectrum.compute:157-172) against the oracle on ~20k texels:
    rows and columns 0, N/2 - 1, N/2, N/2 + 1 and N - 1 (k = 0, the Nyquist row/column and their
    partners N - i), the 96 x 96 block around k = 0 (where the spectrum peaks for the default
    fetch), and random texels; plain and |k|-weighted like test_generate_spectrum."""
    n = 16384
    fft = ocean.FFTCalculator(n)
    gen = ocean.Generator(fft, 1)
    gen.GenerateSpectrum()
    fft.synchronize()
    from oceansimulation_amd import capi, hip

    bsz = int(capi.lib().ocean_generator_spectrum_block(gen.handle))
    blocked = hip.to_host(gen.GetInitialSpectrum(0), (n // bsz, n, bsz, 4))  # [x/B][y][x%B]
    rng = np.random.default_rng(16384)
    lines = np.array([0, n // 2 - 1, n // 2, n // 2 + 1, n - 1])
    pts = []
    for v in lines:
        r = rng.integers(0, n, 1024)
        pts += [np.stack([r, np.full_like(r, v)], 1), np.stack([np.full_like(r, v), r], 1)]
    c = np.arange(n // 2 - 48, n // 2 + 48)
    yy, xx = np.meshgrid(c, c, indexing="ij")
    pts.append(np.stack([xx.ravel(), yy.ravel()], 1))
    pts.append(rng.integers(0, n, (4096, 2)))
    for v in lines:
        pts.append(np.stack([lines, np.full_like(lines, v)], 1))
    xy = np.concatenate(pts).astype(np.int32)
    got = blocked[xy[:, 0] // bsz, xy[:, 1], xy[:, 0] % bsz]
    del blocked
    ref = oracle.spectrum_texels(oracle.default_settings(), n, xy)
    assert np.isfinite(got).all()
    errs = lane_err(got, ref)
    assert max(errs) <= H0_TOL, errs
    k = np.hypot(xy[:, 0] - n / 2, xy[:, 1] - n / 2)[:, None]
    assert max(lane_err(got * k, ref * k)) <= 10 * H0_TOL, lane_err(got * k, ref * k)
    kzero = (xy[:, 0] == n // 2) & (xy[:, 1] == n // 2)
    assert kzero.any() and not got[kzero, :2].any()  # spectrum.compute:137-138
    gen.close()
    fft.close()


def _slabs_vs_whole(ocean, n, P, steps, four_step=True, settings=None):
    """P SlabGenerators over one n x n grid, frames emulated in one process (equal-split all-to-all
    as device copies), against the whole-grid generator on the same path, compared bit for bit on
    the device after every frame (the first seeds h0)."""
    from oceansimulation_amd import capi, hip
    from oceansimulation_amd.hip import DeviceBuffer
    from oceansimulation_amd.slab import SlabGenerator, emulate_frame

    settings = settings or {}
    fft = ocean.FFTCalculator(n)
    whole = ocean.Generator(fft, 1)
    whole.set_four_step(four_step)
    ocean.apply_settings(whole.GetOceanSettings(0), **settings)
    slabs = [SlabGenerator(fft, r, P) for r in range(P)]
    for g in slabs:
        g.set_four_step(four_step)
        ocean.apply_settings(g.GetOceanSettings(), **settings)
    sends = [DeviceBuffer(g.exchange_bytes) for g in slabs]
    recvs = [DeviceBuffer(g.exchange_bytes) for g in slabs]
    L = capi.lib()
    w = n // P
    for k, dt in enumerate(steps):
        emulate_frame(slabs, sends, recvs, dt, update_ocean=(k == 0))
        whole.CalculateOcean(dt)
        hip.synchronize()
        for r, g in enumerate(slabs):
            for get, tex in ((L.ocean_generator_height_map, 16), (L.ocean_generator_displacement_map, 16),
                             (L.ocean_generator_jacobian_map, 4)):
                slab_ptr = int(get(g.handle, 0))
                whole_ptr = int(get(whole.handle, 0)) + r * w * n * tex
                assert _dev_equal(slab_ptr, whole_ptr, w * n * tex), (n, P, four_step, k, r, get.__name__)
    for buf in sends + recvs:
        buf.free()
    for g in slabs:
        g.close()
    whole.close()
    fft.close()


@pytest.mark.slow
def test_config5_geometry_16384_eight_ranks_bit_exact(ocean):
    """BASELINE configs[4] geometry on one GPU: 8 SlabGenerators over the single 16384^2 grid
    (default settings). Each seeds its 1024 kept columns (rank 7 also the Nyquist column), runs the
    four-step column pass whose second step writes the 8 destination blocks, the equal-split
    all-to-all runs as device copies, and the row pass reads its 2048 rows from the 8 received
    blocks (no transpose). The stitched maps and Jacobian equal the whole-grid generator's bit for
    bit, frame after frame (src/Generator.cpp:45-83 split over ranks)."""
    _slabs_vs_whole(ocean, 16384, 8, [0.25, 1.0 / 60.0, 2.0])


@pytest.mark.parametrize("n,P", [(8192, 2), (8192, 8), (8192, 16), (16384, 16)])
def test_four_step_slabs_bit_exact(ocean, n, P):
    """The four-step slab path at the other rank counts the launcher accepts: 16 ranks put 256
    (8192) or 512 (16384) kept columns on each rank and make every destination block's rows a
    single 16-row group of step 2's output."""
    _slabs_vs_whole(ocean, n, P, [0.5, 1.0 / 60.0], settings=dict(planeSize=777.0))


def test_dealt_slabs_8192_bit_exact(ocean):
    """The strip-dealt slab path (ocean_generator_set_four_step(0): one-column items, transposes after
    the exchange) against the whole grid on the same path."""
    _slabs_vs_whole(ocean, 8192, 4, [0.5, 1.0 / 60.0], four_step=False, settings=dict(planeSize=777.0))


@pytest.mark.parametrize("n", [8192, 16384])
def test_four_step_whole_grid_matches_dealt_path(ocean, n):
    """Whole grids of 8192 / 16384 on one rank: the four-step column pass (default; 16-point step
    in registers, N/16-point step straight into the row-major fields) against the strip-dealt column
    pass + transposes (ocean_generator_set_four_step(0), the multi-rank path), over frames with an
    h0 re-layout in between (the switch re-seeds h0 from the settings it was seeded with, not the
    edited ones), within the cross-path bound; a P = 1 slab generator takes the four-step path too."""
    from oceansimulation_amd.slab import SlabGenerator, emulate_frame
    from oceansimulation_amd.hip import DeviceBuffer

    fft = ocean.FFTCalculator(n)
    g4, gd = ocean.Generator(fft, 1), ocean.Generator(fft, 1)
    gd.set_four_step(False)
    for g in (g4, gd):
        ocean.apply_settings(g.GetOceanSettings(0), planeSize=777.0)
        g.CalculateOcean(0.5)
    # an unflagged settings edit must not leak into h0 when the layout switches
    g4.set_four_step(False)
    ocean.apply_settings(g4.GetOceanSettings(0), U_10=3.0)
    g4.CalculateOcean(1.0 / 60.0)
    g4.set_four_step(True)
    ocean.apply_settings(g4.GetOceanSettings(0), U_10=40.0)
    g4.CalculateOcean(1.0 / 60.0)
    gd.CalculateOcean(1.0 / 60.0)
    gd.CalculateOcean(1.0 / 60.0)
    for get in ("height_map_host", "displacement_map_host"):
        a, b = getattr(g4, get)(0), getattr(gd, get)(0)
        assert max(lane_err(a, b)) <= 1e-5, (n, get, lane_err(a, b))
        del a, b
    j4, jd = g4.jacobian_map_host(0), gd.jacobian_map_host(0)
    assert np.abs(j4 - jd).max() <= 1e-5 * np.abs(jd).max()
    del j4, jd
    g4.close()
    gd.close()
    # a slab generator with one rank runs the same four-step path, through caller exchange buffers:
    # bit-identical to a whole grid
    w4, s1 = ocean.Generator(fft, 1), SlabGenerator(fft, 0, 1)
    ocean.apply_settings(w4.GetOceanSettings(0), planeSize=777.0)
    ocean.apply_settings(s1.GetOceanSettings(), planeSize=777.0)
    snd, rcv = DeviceBuffer(s1.exchange_bytes), DeviceBuffer(s1.exchange_bytes)
    from oceansimulation_amd import capi, hip

    L = capi.lib()
    for k, dt in enumerate((0.5, 1.0 / 60.0)):
        w4.CalculateOcean(dt)
        emulate_frame([s1], [snd], [rcv], dt, update_ocean=(k == 0))
        hip.synchronize()
        for get, tex in ((L.ocean_generator_height_map, 16), (L.ocean_generator_displacement_map, 16),
                         (L.ocean_generator_jacobian_map, 4)):
            assert _dev_equal(int(get(s1.handle, 0)), int(get(w4.handle, 0)), n * n * tex), (k, get.__name__)
    snd.free()
    rcv.free()
    s1.close()
    w4.close()
    fft.close()


@pytest.mark.parametrize("n", [1024, 8192])
def test_native_rccl_slab_frames_world1_bit_exact(ocean, n):
    """The C ABI's own exchange (ocean_generator_slab_frame[_pipelined]: grouped ncclSend / ncclRecv
    over an RCCL communicator of the C ABI) at world size 1, the exchange forced through RCCL as a
    self send/receive: serial frames, then pipelined frames + flush, equal the whole-grid generator bit
    for bit (1024: strip-dealt slab path; 8192: four-step slab path)."""
    from oceansimulation_amd import capi
    from oceansimulation_amd.slab import RcclComm, SlabGenerator

    fft = ocean.FFTCalculator(n)
    whole = ocean.Generator(fft, 1)
    g = SlabGenerator(fft, 0, 1)
    for x in (whole.GetOceanSettings(0), g.GetOceanSettings()):
        ocean.apply_settings(x, planeSize=333.0)
    comm = RcclComm(0, 1, lambda uid: uid)
    L = capi.lib()

    def same():
        fft.synchronize()
        return all(_dev_equal(int(get(g.handle, 0)), int(get(whole.handle, 0)), n * n * tex)
                   for get, tex in ((L.ocean_generator_height_map, 16), (L.ocean_generator_displacement_map, 16),
                                    (L.ocean_generator_jacobian_map, 4)))

    for k, dt in enumerate((0.5, 1.0 / 60.0)):
        g.frame(comm, dt, update_ocean=(k == 0))
        whole.CalculateOcean(dt)
        assert same(), ("serial", k)
    # pipelined: the maps lag one frame; after flush they hold the last frame
    steps = [0.25, 1.0 / 30.0, 0.125]
    for dt in steps:
        g.frame_pipelined(comm, dt)
    g.flush()
    for dt in steps:
        whole.CalculateOcean(dt)
    assert same(), "pipelined"
    # a communicator of the wrong size is refused
    with pytest.raises(capi.OceanError):
        SlabGenerator(fft, 0, 2).frame(comm, 0.1)
    comm.close()
    g.close()
    whole.close()
    fft.close()


@pytest.mark.gpu
def test_path_switch_lands_pending_pipelined_frame(ocean):
    """A path switch with a pipelined slab frame in flight (ocean_generator_set_four_step) first issues
    that frame's row pass in the layout its column pass wrote, with the displacement of the settings it
    was issued with (a later edit must not leak into its Jacobian); frames after the switch run the
    strip-dealt path. Both are checked bit for bit against the whole-grid generator on the same path."""
    from oceansimulation_amd import capi
    from oceansimulation_amd.slab import RcclComm, SlabGenerator

    n = 8192
    fft = ocean.FFTCalculator(n)
    whole = ocean.Generator(fft, 1)
    g = SlabGenerator(fft, 0, 1)
    for x in (whole.GetOceanSettings(0), g.GetOceanSettings()):
        ocean.apply_settings(x, planeSize=333.0)
    comm = RcclComm(0, 1, lambda uid: uid)
    L = capi.lib()

    def same():
        fft.synchronize()
        return all(_dev_equal(int(get(g.handle, 0)), int(get(whole.handle, 0)), n * n * tex)
                   for get, tex in ((L.ocean_generator_height_map, 16), (L.ocean_generator_displacement_map, 16),
                                    (L.ocean_generator_jacobian_map, 4)))

    g.frame_pipelined(comm, 0.25, update_ocean=True)  # pending: four-step blocks, displacement 0.4
    ocean.apply_settings(g.GetOceanSettings(), displacement=0.9)
    g.set_four_step(False)  # lands the pending frame first
    whole.CalculateOcean(0.25)
    assert same(), "pending frame after the switch"
    whole.set_four_step(False)
    ocean.apply_settings(whole.GetOceanSettings(0), displacement=0.9)
    g.frame(comm, 0.1)
    whole.CalculateOcean(0.1)
    assert same(), "strip-dealt frame after the switch"
    comm.close()
    g.close()
    whole.close()
    fft.close()


# ---- bench.py --gpus N on a one-GPU box ---------------------------------------------------------
def test_bench_gpus_two_shared_gpu_reports_two_ranks(tmp_path):
    """`bench.py --gpus 2 --shared-gpu` (no launcher) starts 2 ranks under torch.distributed.run,
    both on GPU 0 with gloo standing in for RCCL; rank 0 prints one line with n_gpus = 2 and a
    2-rank slab leg. Small sizes: this checks the launch path, not a measurement. Without
    --shared-gpu, --gpus 2 on a one-GPU box must refuse (rc 2)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    args = ["--gpus", "2", "--shared-gpu", "--n", "1024", "--cascades", "2", "--slab-n", "2048", "--steps", "3",
            "--warmup", "1", "--slab-steps", "2", "--no-cpu-baseline", "--no-surface", "--no-ifft", "--no-reseed"]
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                       timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.strip().startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["value"] > 0
    assert line["slab"]["ranks"] == 2 and "all_to_all_single" in line["slab"]["exchange"]
    import torch

    if torch.cuda.device_count() < 2:
        r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], capture_output=True,
                           text=True, timeout=120, env=env, cwd=ROOT)
        assert r.returncode == 2 and "GPU(s) are visible" in r.stderr, (r.returncode, r.stderr[-2000:])


def test_rccl_all_to_all_large_pieces_world1(ocean):
    """ocean_comm_all_to_all at world size 1 with single transfers above 1 GiB, which RCCL 2.26 got
    wrong in one send/recv pair (profiles/r03_rccl_selfcheck.log): the C ABI cuts each pair into
    512-MiB pieces, so 1.4 GB (two pieces and a ragged third) copies exactly."""
    import torch

    from oceansimulation_amd.slab import RcclComm

    comm = RcclComm(0, 1, lambda uid: uid)
    n = 1400 << 20
    a = torch.randint(0, 255, (n,), dtype=torch.uint8, device="cuda")
    b = torch.zeros_like(a)
    comm.all_to_all(a.data_ptr(), b.data_ptr(), n, 0)
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    del a, b
    torch.cuda.empty_cache()
    comm.close()


def test_debug_copy_exact_and_refuses_bad_arguments(ocean):
    """ocean_debug_copy (the paced exchange traffic of bench.py's 8-rank projection) copies exactly on
    any workgroup count, including a ragged last grid stride, and refuses unaligned or non-multiple-of-16
    sizes and workgroup counts outside [1, 65536]."""
    import torch

    from oceansimulation_amd import capi
    from oceansimulation_amd.waves import debug_copy

    n = (37 << 20) + 48
    a = torch.randint(0, 255, (n,), dtype=torch.uint8, device="cuda")
    for wgs in (1, 7, 96, 4096):
        b = torch.zeros_like(a)
        debug_copy(b.data_ptr(), a.data_ptr(), n, wgs)
        torch.cuda.synchronize()
        assert torch.equal(a, b), wgs
    with pytest.raises(capi.OceanError):
        debug_copy(b.data_ptr(), a.data_ptr(), n - 8, 4)
    with pytest.raises(capi.OceanError):
        debug_copy(b.data_ptr() + 8, a.data_ptr(), 1024, 4)
    with pytest.raises(capi.OceanError):
        debug_copy(b.data_ptr(), a.data_ptr(), 1024, 0)
