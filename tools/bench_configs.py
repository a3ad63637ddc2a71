#!/usr/bin/env python3
"""Measure the BASELINE.json configs other than the bench.py headline (configs[3]) on one GPU,
with the CPU oracle timed beside them. Writes profiles/<tag>_configs.{md,json}.

  config 1: 256^2, the reference scene (3 cascades, L = 5/17/101 m), full payload
  config 2: 1024^2, one packed displacement map through FFTCalculator::EncodeIFFT
  config 3: 2048^2, one cascade, full payload
Usage: python tools/bench_configs.py [tag] [--steps K]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402

import oceansimulation_amd as ocean  # noqa: E402
from oceansimulation_amd import hip  # noqa: E402
from oceansimulation_amd.hip import DeviceBuffer  # noqa: E402
from oracle import oracle as O  # noqa: E402

HBM = 8000.0


def time_gen(n, planes, steps, warmup=3):
    fft = ocean.FFTCalculator(n)
    gen = ocean.Generator(fft, len(planes))
    for c, L in enumerate(planes):
        ocean.apply_settings(gen.GetOceanSettings(c), planeSize=L)
    gen.set_profiling(True)
    for _ in range(warmup):
        gen.CalculateOcean(1 / 60)
    gen.kernel_times()
    hip.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        gen.CalculateOcean(1 / 60)
    hip.synchronize()
    wall = (time.perf_counter() - t0) / steps
    ms, cnt = gen.kernel_times()
    kern = (ms[1] + ms[2]) / steps
    pts = n * n * len(planes)
    return {"points": pts, "wall_ms": wall * 1e3, "kernel_ms": kern,
            "points_per_s": pts / wall, "frame_GBps_algorithmic": 116 * pts / (kern * 1e-3) / 1e9}


def time_ifft(n, steps, warmup=3):
    fft = ocean.FFTCalculator(n)
    img = np.random.default_rng(0).standard_normal((n, n, 4)).astype(np.float32)
    buf = DeviceBuffer.from_array(img)
    for _ in range(warmup):
        fft.EncodeIFFT(buf.ptr)
    fft.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fft.EncodeIFFT(buf.ptr)
    fft.synchronize()
    wall = (time.perf_counter() - t0) / steps
    return {"points": n * n, "wall_ms": wall * 1e3, "points_per_s": n * n / wall,
            "GBps_algorithmic_64B": 64 * n * n / wall / 1e9}


def cpu_gen(n, planes, seconds=5.0):
    gens = [O.OracleGenerator(n, O.default_settings(planeSize=L)) for L in planes]
    for g in gens:
        g.calculate_ocean(1 / 60)
    frames, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        for g in gens:
            g.calculate_ocean(1 / 60)
        frames += 1
    el = time.perf_counter() - t0
    return {"points_per_s": n * n * len(planes) * frames / el, "frames": frames, "threads": O.get_threads()}


def cpu_ifft(n, seconds=5.0):
    img = np.random.default_rng(0).standard_normal((n, n, 4)).astype(np.float32)
    frames, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        O.encode_ifft(img)
        frames += 1
    el = time.perf_counter() - t0
    return {"points_per_s": n * n * frames / el, "frames": frames, "threads": O.get_threads()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag", nargs="?", default="r01")
    ap.add_argument("--steps", type=int, default=50)
    args = ap.parse_args()
    O.build()
    O.set_threads(min(16, os.cpu_count() or 1))
    res = {
        "config1_256_scene": {"gpu": time_gen(256, [5.0, 17.0, 101.0], args.steps), "cpu": cpu_gen(256, [5.0, 17.0, 101.0])},
        "config2_1024_encode_ifft": {"gpu": time_ifft(1024, args.steps), "cpu": cpu_ifft(1024)},
        "config3_2048_full_payload": {"gpu": time_gen(2048, [40.0], args.steps), "cpu": cpu_gen(2048, [40.0])},
    }
    lines = [f"# BASELINE configs 1-3 on one MI355X — {args.tag}", "",
             "GPU: wall time per step over the timed steps (host launch included); kernel ms from HIP events. "
             f"CPU: the oracle (fp32 radix-2 restatement of the reference), {O.get_threads()} OpenMP threads.", "",
             "| config | GPU points/s | GPU wall ms/step | GPU kernel ms | CPU points/s | GPU/CPU |",
             "|---|---|---|---|---|---|"]
    for k, v in res.items():
        g, c = v["gpu"], v["cpu"]
        lines.append(f"| {k} | {g['points_per_s']:.3e} | {g['wall_ms']:.3f} | {g.get('kernel_ms', float('nan')):.3f} | "
                     f"{c['points_per_s']:.3e} | {g['points_per_s'] / c['points_per_s']:.0f}x |")
    # gpurun only brings gpurun_out/ back from the GPU box; copy into profiles/ from there
    out_dir = os.path.join(ROOT, "gpurun_out")
    os.makedirs(out_dir, exist_ok=True)
    with open(os.path.join(out_dir, f"{args.tag}_configs.json"), "w") as f:
        json.dump(res, f, indent=1)
    with open(os.path.join(out_dir, f"{args.tag}_configs.md"), "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
