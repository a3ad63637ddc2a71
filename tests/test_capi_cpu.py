"""The C ABI library without a GPU: it loads, exports exactly what include/oceanfft.h declares,
the settings layout matches, and every compute entry point fails loudly (no CPU fallback)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "oceanfft.h")


def _declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(ocean_[a-z0-9_]+)\s*\(", text)))


@pytest.fixture(scope="module")
def capi():
    from oceansimulation_amd import capi

    capi.lib()
    return capi


def test_every_declared_symbol_is_exported_and_bound(capi):
    names = _declared_functions()
    assert len(names) >= 20
    for name in names:
        assert hasattr(capi.lib(), name), f"{name} declared in oceanfft.h but not exported"
        assert name in capi.SIGNATURES, f"{name} not bound in oceansimulation_amd/capi.py"
    assert set(capi.SIGNATURES) == set(names)


def test_settings_layout_matches_header(capi):
    text = open(HEADER).read()
    body = text[text.index("typedef struct ocean_settings"):text.index("} ocean_settings;")]
    fields = re.findall(r"^\s*(?:int32_t|float)\s+(\w+)(?:\[2\])?;", body, flags=re.M)
    assert fields == [f[0] for f in capi.OceanSettings._fields_]
    assert ctypes.sizeof(capi.OceanSettings) == 64
    offs = {f[0]: getattr(capi.OceanSettings, f[0]).offset for f in capi.OceanSettings._fields_}
    assert offs["U_10"] == 8 and offs["time"] == 36 and offs["wavelengthMax"] == 60


def test_default_settings_are_the_reference_defaults(capi):
    s = capi.OceanSettings()
    capi.lib().ocean_default_settings(ctypes.byref(s))
    # src/Generator.h:14-29
    assert (s.seed[0], s.seed[1]) == (12342, 8934)
    exp = dict(U_10=40.0, theta_0=25.0, F=800000.0, g=9.8, swell=0.5, h=100.0, displacement=0.4, time=0.0,
               planeSize=40.0, scale=1.0, spread=0.2, boundWavelength=0, wavelengthMin=0.0, wavelengthMax=0.0)
    for k, v in exp.items():
        assert getattr(s, k) == pytest.approx(v, rel=0, abs=1e-6), k


def test_invalid_arguments_fail_without_touching_a_device(capi):
    L = capi.lib()
    h = ctypes.c_void_p()
    for bad in (0, 8, 300, 1000, 32768, 1 << 20):
        assert L.ocean_fft_create(ctypes.byref(h), bad, None) == capi.OCEAN_ERR_INVALID
        assert b"power of two" in L.ocean_last_error()
    assert L.ocean_fft_create(None, 256, None) == capi.OCEAN_ERR_INVALID
    assert L.ocean_fft_encode_ifft(None, None) == capi.OCEAN_ERR_INVALID
    assert L.ocean_generator_calculate(None, ctypes.c_float(0.1), 0) == capi.OCEAN_ERR_INVALID
    assert L.ocean_generator_create(ctypes.byref(h), None, 1) == capi.OCEAN_ERR_INVALID
    assert L.ocean_generator_height_map(None, 0) is None
    assert L.ocean_fft_texture_resolution(None) == 0
    assert L.ocean_debug_hash(None, 4, None, None, None) == capi.OCEAN_ERR_INVALID
    assert L.ocean_fft_set_cu_budget(None, 0) == capi.OCEAN_ERR_INVALID
    for switch in ("ocean_generator_set_frame_overlap", "ocean_generator_set_h0_memo",
                   "ocean_generator_set_half_spectrum", "ocean_generator_set_four_step"):
        assert getattr(L, switch)(None, 1) == capi.OCEAN_ERR_INVALID, switch


def test_no_cpu_fallback_without_gpu(capi):
    L = capi.lib()
    if L.ocean_device_count() > 0:
        pytest.skip("a GPU is visible; covered by the gpu tests")
    h = ctypes.c_void_p()
    assert L.ocean_fft_create(ctypes.byref(h), 256, None) == capi.OCEAN_ERR_NO_DEVICE
    import oceansimulation_amd as ocean

    with pytest.raises(ocean.OceanError):
        ocean.FFTCalculator(256)


def test_cpp_dropin_library_exports_reference_signatures():
    so = os.path.join(ROOT, "oceansimulation_amd", "libwaves.so")
    assert os.path.exists(so), "run make"
    syms = subprocess.run(["nm", "-DC", "--defined-only", so], capture_output=True, text=True).stdout
    for sig in ["Waves::FFTCalculator::FFTCalculator(Vision::RenderDevice*, unsigned long)",
                "Waves::FFTCalculator::EncodeIFFT(unsigned int)",
                "Waves::Generator::Generator(Vision::RenderDevice*, Waves::FFTCalculator*)",
                "Waves::Generator::CalculateOcean(float, bool)",
                "Waves::Generator::GetOceanSettings()",
                "Waves::Generator::LoadShaders(bool)"]:
        assert sig in syms, sig


def test_cpp_headers_compile_standalone(tmp_path):
    """A Renderer-style consumer compiles against the drop-in headers unchanged."""
    src = tmp_path / "consumer.cpp"
    src.write_text(
        '#include "waves/Generator.h"\n'
        "#include <vector>\n"
        "void render(Vision::RenderDevice* d, std::vector<Waves::Generator*>& gens) {\n"
        "  for (size_t i = 0; i < gens.size(); i++) {\n"
        "    Vision::ID h = gens[i]->GetHeightMap(), dm = gens[i]->GetDisplacementMap(), j = gens[i]->GetJacobianMap();\n"
        "    float plane = gens[i]->GetOceanSettings().planeSize, disp = gens[i]->GetOceanSettings().displacement;\n"
        "    (void)d->GetTexturePointer(h); (void)dm; (void)j; (void)plane; (void)disp;\n"
        "  }\n"
        "}\n")
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", f"-I{ROOT}/include", "-I/opt/rocm/include",
                        "-D__HIP_PLATFORM_AMD__", str(src)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_seed_assigns_from_glm_ivec2_shaped_types(tmp_path):
    """Reference code sets the seed as a glm::ivec2 (src/Generator.h:14): the drop-in's seed type
    converts from and to any {x, y} vector type, keeping the 64-byte layout. glm itself is absent
    here, so the test declares a vector type of the same shape."""
    src = tmp_path / "seed.cpp"
    src.write_text(
        '#include "waves/Generator.h"\n'
        "namespace glm { struct ivec2 { int x, y; ivec2() : x(0), y(0) {} ivec2(int a, int b) : x(a), y(b) {} }; }\n"
        "int main() {\n"
        "  Waves::GeneratorSettings s;\n"
        "  if (s.seed.x != 12342 || s.seed.y != 8934) return 1;\n"
        "  s.seed = glm::ivec2(7, 9);\n"
        "  glm::ivec2 back = glm::ivec2(s.seed);\n"
        "  Waves::GeneratorSettings t = s;\n"
        "  static_assert(sizeof(Waves::GeneratorSettings) == 64, \"layout\");\n"
        "  return (back.x == 7 && back.y == 9 && t.seed == s.seed && s.seed[1] == 9) ? 0 : 2;\n"
        "}\n")
    exe = tmp_path / "seed"
    r = subprocess.run(["g++", "-std=c++17", f"-I{ROOT}/include", "-I/opt/rocm/include", "-D__HIP_PLATFORM_AMD__",
                        str(src), "-o", str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert subprocess.run([str(exe)]).returncode == 0


def test_waveapp_headless_rejects_bad_arguments():
    """The headless driver parses its script before touching a device (exit 2 = usage)."""
    import subprocess

    exe = os.path.join(ROOT, "examples", "waveapp_headless")
    assert os.path.exists(exe), "make builds examples/waveapp_headless"
    for bad in (["--bogus", "1"], ["--edit", "3:7.U_10=1"], ["--freeze", "x"], ["--n"]):
        r = subprocess.run([exe, *bad], capture_output=True, text=True, timeout=60)
        assert r.returncode == 2, (bad, r.returncode, r.stderr)


def _half_slab_restated(n, rank, ranks):
    """DESIGN.md §3 strip dealing, restated: B = 4 / 2 / 1 texels per strip at N <= 4096 / 8192 /
    16384; STRIPS = N/(2B) + 1 kept strips (u >= 0, then the Nyquist strip), ceil(STRIPS/ranks) per
    rank; a block = gab | gde | gc parts (40 B per element) + the Nyquist-row term (2N float4)."""
    b = 4 if n <= 4096 else (2 if n == 8192 else 1)
    strips = n // (2 * b) + 1
    s = -(-strips // ranks)
    strip0 = rank * s
    nstrips = max(0, min(s, strips - strip0))
    w = n // ranks
    blk = 40 * s * w * b + 2 * n * 16
    return strip0, nstrips, s, w, blk, blk * ranks


@pytest.mark.parametrize("n", [1024, 2048, 4096, 8192, 16384])
@pytest.mark.parametrize("ranks", [1, 2, 4, 8, 16])
def test_half_slab_layout_deals_every_strip_once(capi, n, ranks):
    """The strip-dealt path's geometry (host logic, no device): the ABI's layout equals the
    restatement, every kept strip is transformed by exactly one rank, and the blocks tile the
    exchange buffer."""
    from oceansimulation_amd.slab import slab_layout

    seen = []
    for r in range(ranks):
        lay = slab_layout(n, r, ranks, half=True)
        assert lay == _half_slab_restated(n, r, ranks)
        seen.extend(range(lay[0], lay[0] + lay[1]))
        assert lay[3] % 32 == 0  # whole transpose row tiles
    b = 4 if n <= 4096 else (2 if n == 8192 else 1)
    assert seen == list(range(n // (2 * b) + 1))
    full = slab_layout(n, 0, ranks, half=False)
    assert full[5] == 32 * n * (n // ranks)  # the full spectrum's 32 B per point
    # half spectrum: ~20 B per point, plus slot padding and the per-block Nyquist-row term (which
    # dominates the small blocks of small grids over 16 ranks)
    if ranks <= 8:
        assert slab_layout(n, 0, ranks)[5] < (0.7 if n >= 4096 else 0.8) * full[5]


@pytest.mark.parametrize("n,ranks", [(8192, 1), (8192, 2), (8192, 16), (16384, 8), (16384, 16)])
def test_four_step_slab_layout_deals_every_column_once(capi, n, ranks):
    """Four-step slabs (ocean_slab_layout half == 2): the N/2 regular kept columns are dealt N/(2P) per
    rank in order, only the last rank holds the Nyquist column, every block is the same size (equal
    split), and the exchange is 20 B per point (+ the 16-column pitch pad and the Nyquist-row term)."""
    from oceansimulation_amd.slab import slab_layout

    lays = [slab_layout(n, r, ranks, half=2) for r in range(ranks)]
    cols = [c for (u0, k, _, _, _, _) in lays for c in range(u0, u0 + k)]
    assert cols == list(range(n // 2))
    assert [l[2] for l in lays] == [0] * (ranks - 1) + [1]
    assert all(l[3] == n // ranks for l in lays)
    assert len({l[4] for l in lays}) == 1 and all(l[5] == l[4] * ranks for l in lays)
    per_point = lays[0][5] / (n * n / ranks)
    assert 20.0 < per_point < 20.0 * (1 + 17 / (n / (2 * ranks))) + 1.0


def test_slab_layout_rejects_bad_geometry(capi):
    from oceansimulation_amd.capi import OceanError
    from oceansimulation_amd.slab import slab_layout

    with pytest.raises(OceanError):
        slab_layout(1000, 0, 2)
    with pytest.raises(OceanError):
        slab_layout(4096, 0, 3)
    with pytest.raises(OceanError):
        slab_layout(512, 0, 2, half=True)
    assert slab_layout(512, 1, 2, half=False)[:2] == (256, 256)
    with pytest.raises(OceanError):
        slab_layout(4096, 0, 2, half=2)  # the four-step path serves 8192 / 16384 only


@pytest.mark.parametrize("n", [1024, 2048, 4096])
def test_frame_plan_pairs_column_writes_with_row_reads(capi, n):
    """ocean_frame_plan (host only): for every cascade count a launch can take and both row-pass variants,
    the field layout the column pass writes (strip width, gab/gde and gc row groups) is the one the row
    pass reads, and the h0 strips the column pass reads are the ones the seeding writes. Each launcher
    picks its kernel from the descriptor reported here (launch_half.hip), so a mode that changed one
    side's layout without the other's (round 4's fallback row pass) fails here, without a GPU."""
    import ctypes

    L = capi.lib()
    seen = set()
    for cascades in range(1, capi.OCEAN_MAX_CASCADES + 1):
        for variant in (0, 1):
            out = (ctypes.c_int32 * 8)()
            assert L.ocean_frame_plan(n, cascades, variant, out) == capi.OCEAN_OK
            cols, rows, seed_h0 = tuple(out[0:4]), tuple(out[4:7]), out[7]
            assert cols[:3] == rows, (n, cascades, variant, cols, rows)
            assert cols[3] == seed_h0, (n, cascades, variant, cols, seed_h0)
            # whole 128-B lines per store: RG * FB * 16 B (gab / gde) and RGC * FB * 8 B (gc)
            assert cols[1] * cols[0] * 16 == 128 and cols[2] * cols[0] * 8 == 128, cols
            seen.add(cols)
    # the half-strip shape exists at 2048 and 4096 (<= 2 cascades per launch)
    assert (len(seen) == 2) == (n in (2048, 4096)), seen
    bad = (ctypes.c_int32 * 8)()
    assert L.ocean_frame_plan(512, 1, 1, bad) == capi.OCEAN_ERR_INVALID  # below the half path
    assert L.ocean_frame_plan(n, 0, 1, bad) == capi.OCEAN_ERR_INVALID
    assert L.ocean_frame_plan(n, capi.OCEAN_MAX_CASCADES + 1, 1, bad) == capi.OCEAN_ERR_INVALID
    assert L.ocean_frame_plan(n, 1, 2, bad) == capi.OCEAN_ERR_INVALID
