"""Host-side logic that needs no GPU: bench workload definition, parity metrics, Python mirror."""
import importlib.util
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_bench_byte_accounting():
    b = _bench()
    assert b.frame_bytes_per_point(4096, False) == (48.0, 68.0)
    p1, p2 = b.frame_bytes_per_point(4096, True)
    kept = (2048 + 4) / 4096
    assert p1 == 16.0 * kept + 40.0 * kept and p2 == 40.0 * kept + 36.0
    assert 84.0 < p1 + p2 < 84.1  # 8 + 20 | 20 + 36 per grid point, plus the Nyquist strip
    # the whole-grid paths ocean_generator_create picks, and the four-step bytes at 8192 / 16384
    assert [b.frame_path(n) for n in (256, 1024, 4096, 8192, 16384)] == ["full", "half", "half", "four-step",
                                                                         "four-step"]
    assert b.frame_path(4096, full_spectrum=True) == "full"
    q1, q2 = b.frame_bytes_per_point(16384, "four-step")
    kept = (8192 + 1) / 16384
    assert q1 == 136.0 * kept and q2 == 40.0 * kept + 36.0 and 124.0 < q1 + q2 < 124.1
    assert b.frame_bytes_per_point(16384, "full") == (48.0, 132.0)  # + the B = 1 transpose


def test_bench_cascade_sharding_is_disjoint():
    """Every (rank, cascade) gets a distinct noise tile: seeds differ by >= 4097 > N = 4096, so
    Hash(thread + seed) windows (spectrum.compute:153) never overlap except at the +N edge index."""
    b = _bench()
    seen = set()
    for rank in range(8):
        for c in range(16):
            s = b.cascade_settings(rank, c)
            key = (s["planeSize"], s["seed"])
            assert key not in seen
            seen.add(key)
            assert s["seed"][0] >= 12342 and s["seed"][1] >= 8934
    assert b.cascade_settings(0, 0)["planeSize"] == 5.0
    assert [b.cascade_settings(0, c)["planeSize"] for c in range(3)] == [5.0, 17.0, 101.0]  # Waves.cpp:27


def test_strong_scaling_split():
    """the 8 cascades all on 1 GPU, then 8/P per GPU at P = 2, 4, 8 — disjoint and
    together the whole job whatever P; an uneven split is refused."""
    b = _bench()
    for world in (1, 2, 4, 8):
        parts = [b.rank_cascades(8, r, world) for r in range(world)]
        assert all(len(p) == 8 // world for p in parts)
        assert sorted(c for p in parts for c in p) == list(range(8))
    with pytest.raises(ValueError):
        b.rank_cascades(8, 0, 3)


def test_frame_overlap_mode_choice():
    """The strong-scaling headline overlaps frames (ocean_generator_set_frame_overlap) only at <= 2
    cascades per GPU on the blocked half path; --frame-overlap on/off overrides, never on other paths."""
    b = _bench()
    auto = b.parse([])
    assert [b.use_frame_overlap(auto, c, "half", 1024) for c in (8, 4, 2, 1)] == [False, False, True, True]
    for n in (2048, 4096):  # half strips at <= 2 cascades: serial
        assert not any(b.use_frame_overlap(auto, c, "half", n) for c in (8, 4, 2, 1))
    assert not b.use_frame_overlap(auto, 1, "full", 2048) and not b.use_frame_overlap(auto, 1, "four-step", 8192)
    assert b.use_frame_overlap(b.parse(["--frame-overlap", "on"]), 8, "half", 4096)
    assert not b.use_frame_overlap(b.parse(["--frame-overlap", "on"]), 8, "full", 4096)
    assert not b.use_frame_overlap(b.parse(["--frame-overlap", "off"]), 1, "half", 1024)


def test_lane_err_metric():
    from parity import lane_err, scalar_err

    a = np.zeros((4, 4, 4), np.float32)
    a[..., 0] = 2.0
    b = a.copy()
    b[0, 0, 0] += 0.002
    e = lane_err(b, a)
    assert abs(e[0] - 1e-3) < 1e-7 and e[1] == 0.0
    assert abs(scalar_err(b[..., 0], a[..., 0]) - 1e-3) < 1e-7


def test_python_mirror_settings_helpers():
    import oceansimulation_amd as ocean

    s = ocean.default_settings(planeSize=17.0, seed=(1, 2))
    assert s.planeSize == 17.0 and (s.seed[0], s.seed[1]) == (1, 2) and s.U_10 == 40.0
    ocean.apply_settings(s, time=2.5)
    assert s.time == 2.5


def test_bench_legs_watchdog_prints_headline_and_exits():
    """bench.py's optional legs run under a deadline: past it, rank 0 prints the headline line it
    has (with "legs_timeout") and the process exits 0, so a stuck optional leg never loses the
    measurement; legs that finish first cancel it and the caller prints."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys, time; sys.path.insert(0, %r); import bench\n"
            "out = {'metric': 'm', 'value': 1.0}\n"
            "w = bench.start_legs_watchdog(out, 0, 0.2)\n"
            "time.sleep(5)\n"
            "print('not reached')\n") % root
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert r.returncode == _bench().LEGS_TIMEOUT_RC == 3, (r.returncode, r.stderr)
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["value"] == 1.0 and "legs_timeout" in line
    code = ("import sys; sys.path.insert(0, %r); import bench\n"
            "w = bench.start_legs_watchdog({'value': 2.0}, 0, 30.0)\n"
            "print('finished', w.finish())\n") % root
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and r.stdout.strip() == "finished True", (r.stdout, r.stderr)


def _run_bench(args, timeout=240):
    import subprocess
    import sys

    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    env.pop("LOCAL_RANK", None)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          timeout=timeout, env=env, cwd=ROOT)


def test_bench_gpus_n_launches_n_ranks():
    """`bench.py --gpus 2` without a launcher starts torch.distributed.run as a child (gloo here: no
    GPU work with --plumbing-check) and rank 0's single line reports n_gpus = 2."""
    import json

    r = _run_bench(["--gpus", "2", "--plumbing-check", "--n", "1024"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.strip().startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["gpus_requested"] == 2 and line["plumbing"] is True
    assert abs(line["max_over_ranks_s"] - 0.002) < 1e-12  # the slower rank's time, not rank 0's


def test_bench_gpus_n_fails_loudly_without_n_gpus():
    """Asking for more GPUs than are visible must fail (rc 2), never report a 1-GPU number."""
    r = _run_bench(["--gpus", "2"], timeout=120)
    assert r.returncode == 2, (r.returncode, r.stdout, r.stderr[-2000:])
    assert "GPU(s) are visible" in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.strip().startswith("{")]


def test_bench_cpu_baseline_core_accounting(monkeypatch):
    b = _bench()
    monkeypatch.setenv("OMP_NUM_THREADS", "3")
    threads, machine, affinity = b.host_cores()
    assert threads == min(3, affinity) and machine == os.cpu_count()
    monkeypatch.delenv("OMP_NUM_THREADS")
    threads, _, affinity = b.host_cores()
    assert threads == affinity


def test_traffic_attribution_needs_same_device_code(tmp_path, monkeypatch):
    """roofline.traffic comes only from a PMC summary stamped with the running tree's device-code
    hash (bench.py and tools/parse_rocprof.py hash the same files the same way); a summary of other
    device code is ignored."""
    import json
    import shutil

    b = _bench()
    g = vars(_parse_rocprof())
    assert g["device_source_sha256"]() == b.device_source_sha256()
    assert g["base_name"]("void oceanfft::k_rows_half<12, 0, 2>(oceanfft::FrameParams, float*)") == "k_rows_half"
    # a fake tree: same device code, one matching and one stale summary
    root = tmp_path / "tree"
    shutil.copytree(os.path.join(ROOT, "oceansimulation_amd", "csrc"), root / "oceansimulation_amd" / "csrc",
                    ignore=shutil.ignore_patterns("build", "*.o"))
    (root / "profiles").mkdir()
    rec = {"kernels": {"k_rows_half": {"hbm_traffic_bytes": 123.0}}, "n": 4096, "cascades": 8}
    (root / "profiles" / "r09_stale_rocprof.json").write_text(json.dumps(dict(rec, device_source_sha256="0" * 64)))
    monkeypatch.setattr(b, "ROOT", str(root))
    assert b.measured_traffic("k_rows_half", 4096, 8) is None
    sha = b.device_source_sha256(str(root))
    (root / "profiles" / "r01_same_rocprof.json").write_text(json.dumps(dict(rec, device_source_sha256=sha)))
    got = b.measured_traffic("k_rows_half", 4096, 8)
    assert got["hbm_traffic_bytes"] == 123.0 and "r01_same_rocprof.json" in got["source"]


def _parse_rocprof():
    import importlib.util

    spec = importlib.util.spec_from_file_location("parse_rocprof", os.path.join(ROOT, "tools", "parse_rocprof.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _write_csv(path, header, rows):
    import csv

    path.parent.mkdir(parents=True, exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(header)
        w.writerows(rows)


def _fake_profile(tmp_path, rows_ms):
    """A gpurun_out-like directory: kernel trace + FETCH_SIZE + WRITE_SIZE CSVs in rocprofv3's columns.
    rows_ms: [(symbol, grid threads, workgroup threads, duration ms, FETCH_SIZE KB, WRITE_SIZE KB)]."""
    th = ["Kind", "Dispatch_Id", "Kernel_Name", "Start_Timestamp", "End_Timestamp", "Workgroup_Size_X",
          "Workgroup_Size_Y", "Workgroup_Size_Z", "Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z"]
    ch = ["Dispatch_Id", "Grid_Size", "Kernel_Name", "Workgroup_Size", "Counter_Name", "Counter_Value"]
    trace, fetch, write = [], [], []
    for d, (sym, grid, wg, ms, fe, wr) in enumerate(rows_ms):
        trace.append(["KERNEL_DISPATCH", d, sym, 1000, 1000 + int(ms * 1e6), wg, 1, 1, grid, 1, 1])
        fetch.append([d, grid, sym, wg, "FETCH_SIZE", fe])
        write.append([d, grid, sym, wg, "WRITE_SIZE", wr])
    _write_csv(tmp_path / "p_trace" / "t_kernel_trace.csv", th, trace)
    _write_csv(tmp_path / "p_fetch" / "f_counter_collection.csv", ch, fetch)
    _write_csv(tmp_path / "p_write" / "w_counter_collection.csv", ch, write)


def test_parse_rocprof_keys_by_geometry_and_size(tmp_path, monkeypatch):
    """tools/parse_rocprof.py: durations and counters keyed by (kernel at its size, grid, workgroup); the
    workload's algorithmic bytes only for the workload's size; "-" for kernels with no figure."""
    import json

    m = _parse_rocprof()
    rows = "void oceanfft::k_rows_half<12, 1, 2>(oceanfft::FrameParams)"
    other = "void oceanfft::k_rows_half<14, 1, 2>(oceanfft::FrameParams)"
    nyq = "void oceanfft::k_half_nyquist<12>(oceanfft::FrameParams)"
    _fake_profile(tmp_path, [(rows, 262144, 512, 1.4, 3e6, 4.5e6), (rows, 262144, 512, 1.4, 3e6, 4.5e6),
                             (other, 262144, 1024, 4.0, 1e6, 1e6), (nyq, 8192, 256, 0.01, 10, 10)])
    monkeypatch.chdir(tmp_path)
    m.main(["parse_rocprof.py", str(tmp_path), "t", "4096", "8", "p"])
    prof = json.load(open(tmp_path / "profiles" / "t_rocprof.json"))
    rec = prof["kernels"]["k_rows_half"]
    kept = (2048 + 4) / 4096
    assert rec["calls"] == 2 and rec["algorithmic_bytes"] == int((40 * kept + 36) * 4096 * 4096 * 8)
    assert rec["hbm_traffic_bytes"] == 3e6 * 2048 + 4.5e6 * 1024
    assert prof["kernels"]["k_rows_half<14>"]["algorithmic_bytes"] is None  # another size: no borrowed bytes
    assert prof["kernels"]["k_half_nyquist"]["algorithmic_bytes"] is None
    md = open(tmp_path / "profiles" / "t_rocprof.md").read()
    assert "| k_rows_half<14> | 256 x 1024 | 1 | 4.000 | - |" in md


def test_parse_rocprof_refuses_above_peak(tmp_path, monkeypatch):
    """A launch whose algorithmic rate would exceed the HBM peak covers less work than the workload the
    bytes assume (e.g. a one-cascade launch of the same persistent grid): the parser refuses it."""
    m = _parse_rocprof()
    rows = "void oceanfft::k_rows_half<12, 1, 2>(oceanfft::FrameParams)"
    _fake_profile(tmp_path, [(rows, 262144, 512, 0.18, 1, 1)])  # 8 cascades' bytes in a 1-cascade time
    monkeypatch.chdir(tmp_path)
    with pytest.raises(SystemExit, match="exceeds"):
        m.main(["parse_rocprof.py", str(tmp_path), "t", "4096", "8", "p"])


def test_xp_hp_index_model():
    """tools/xp_model.py plays k_rows_xp's (16384), k_rows_hp's and k_cols_half HX's (4096) LDS slots, in-wave
    register <-> lane bit transpositions, twiddles and output layout on the host: both must be the
    unnormalised inverse DFT (the T_in write slots must also cover every x index exactly once)."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("xp_model", os.path.join(ROOT, "tools", "xp_model.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    assert m.model_xp() < 1e-12
    assert m.model_hp() < 1e-12
    assert m.hp_bank_multiplicity() == 1  # k_rows_hp's four LDS access shapes are conflict-free
    assert m.model_hx() < 1e-12  # k_cols_half HX (measured, not kept) and its storage-row bijection


def test_cu_mask_sets_split_every_xcd():
    """A hipExtStreamCreateWithCUMask bit c is CU c / 8 of XCD c % 8, and an XCD without bits runs on
    all its CUs (profiles/r05_xcdprobe.log): the put stream's set and the RCCL projection's reserved set
    must give every XCD the same number of CUs, and the rest must be the complement."""
    b = _bench()
    dev = 256
    for k in (4, 8, 12):
        put = b.put_cu_set(k, dev)
        assert len(put) == 8 * k
        per_xcd = [sum(1 for c in put if c % 8 == x) for x in range(8)]
        assert per_xcd == [k] * 8
        rest = [c for c in range(dev) if c not in set(put)]
        assert [sum(1 for c in rest if c % 8 == x) for x in range(8)] == [dev // 8 - k] * 8
    res = b.reserved_cu_set("per_xcd", dev, 32)
    assert [sum(1 for c in res if c % 8 == x) for x in range(8)] == [4] * 8
    import pytest

    with pytest.raises(ValueError):
        b.reserved_cu_set("stride", dev, 32)


def test_fft8_index_model():
    """tools/microbench/k_cols_small.h's radix-8 Stockham schedule (first stage radix 2^(log2 N mod 3), then radix 8;
    thread i holds x[i + m N/8] and ends with X[i + m N/8]), played on the host (tools/fft8_model.py),
    equals N * ifft at every size the small-grid column pass runs (1024, 2048) and beside them."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("fft8_model", os.path.join(ROOT, "tools", "fft8_model.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    rng = np.random.default_rng(0)
    for logn in (9, 10, 11):
        n = 1 << logn
        x = rng.standard_normal(n) + 1j * rng.standard_normal(n)
        got = mod.fft8_model(x, logn)
        ref = np.fft.ifft(x) * n
        assert np.max(np.abs(got - ref)) <= 1e-9 * np.max(np.abs(ref)), logn
