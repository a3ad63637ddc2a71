#!/usr/bin/env python3
"""GPU-vs-oracle error table for full CalculateOcean frames, including long simulated times.

Metrics (tests/parity.py): max |got - ref| / max |ref| per complex lane (worst of the 4 lanes of
the two maps), per real channel (worst of the 8 channels, and which one), and for the Jacobian - 1. Also prints the phase-precision scale eps32 * w_max * t:
the fp32 rounding of the phase w*t that the reference itself performs, which bounds how far any
two fp32 implementations (GLSL, libm, ocml, hardware v_sin) can agree at time t.
Writes gpurun_out/parity_report.md.  Usage: python tools/parity_report.py
"""
from __future__ import annotations

import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402

import numpy_ref as R  # noqa: E402
import oceansimulation_amd as ocean  # noqa: E402
from oracle import oracle as O  # noqa: E402
from parity import channel_err, lane_err, scalar_err  # noqa: E402

G = 9.81


def omega_max(n, plane, depth, g=G):
    k = math.pi * n / plane * math.sqrt(2.0)
    return math.sqrt((g * k + 0.074 / 1000.0 * k ** 3) * math.tanh(min(k * depth, 20.0)))


CHANNELS = ["h", "dh/dx", "dh/dz", "Dx", "Dz", "dDx/dx", "dDz/dz", "dDx/dz"]


def f64_frame(ref, t):
    """The oracle's fp32 h0 and prepareFFT (the reference's arithmetic) at time t, transformed in
    float64 (N^2 ifft2(ifftshift), the meaning of src/FFTCalculator.cpp:73-114), foam from those maps:
    the frame without the fp32 radix-2 rounding of the oracle's (and the reference's) FFT."""
    import copy

    s = copy.copy(ref.settings)
    s.time = t
    hp, dp = O.prepare_fft(s, ref.n, ref.h0)
    h64, d64 = R.encode_ifft(hp), R.encode_ifft(dp)
    return h64, d64, R.compute_foam(s, d64)


def run(n, planes, times):
    fft = ocean.FFTCalculator(n)
    gen = ocean.Generator(fft, len(planes))
    refs = []
    for c, L in enumerate(planes):
        ocean.apply_settings(gen.GetOceanSettings(c), planeSize=L)
        refs.append(O.OracleGenerator(n, O.default_settings(planeSize=L)))
    rows, t_prev = [], 0.0
    for t in times:
        dt = t - t_prev
        gen.CalculateOcean(dt)
        for r in refs:
            r.calculate_ocean(dt)
        t_prev = t
        for c, L in enumerate(planes):
            hm, dm = gen.height_map_host(c), gen.displacement_map_host(c)
            e = lane_err(hm, refs[c].height) + lane_err(dm, refs[c].disp)
            ec = channel_err(hm, refs[c].height) + channel_err(dm, refs[c].disp)
            ej = scalar_err(gen.jacobian_map_host(c) - 1.0, refs[c].jac - 1.0)
            depth = refs[c].settings.h
            tc = float(gen.GetOceanSettings(c).time)
            scale = 2.0 ** -23 * omega_max(n, L, depth, refs[c].settings.g) * tc
            h64, d64, j64 = f64_frame(refs[c], refs[c].settings.time)
            g64 = max(channel_err(hm, h64) + channel_err(dm, d64))
            o64 = max(channel_err(refs[c].height, h64) + channel_err(refs[c].disp, d64))
            gj64 = scalar_err(gen.jacobian_map_host(c) - 1.0, j64 - 1.0)
            rows.append((n, L, tc, max(e), ec, ej, scale, g64, o64, gj64))
            print(f"N={n} L={L:g} t={tc:g}: lane {max(e):.2e} channel {max(ec):.2e} jac {ej:.2e} | vs f64: GPU "
                  f"{g64:.2e} oracle {o64:.2e} GPU jac {gj64:.2e}", flush=True)
    return rows


def run_sampled(n, plane, dt):
    """One frame at N (e.g. 16384, too large for the whole-grid CPU oracle): sampled outputs against
    the oracle's h0 + prepareFFT and a float64 inverse DFT at the sample points (oracle.sampled_frame)."""
    fft = ocean.FFTCalculator(n)
    gen = ocean.Generator(fft, 1)
    ocean.apply_settings(gen.GetOceanSettings(0), planeSize=plane)
    gen.CalculateOcean(dt)
    s = O.default_settings(planeSize=plane)
    s.time = gen.GetOceanSettings(0).time
    xs, ys = sample_lines(n)
    h, d, j = O.sampled_frame(s, n, xs, ys, progress=True)
    gh = gen.height_map_host(0)[np.ix_(ys, xs)]
    gd = gen.displacement_map_host(0)[np.ix_(ys, xs)]
    gj = gen.jacobian_map_host(0)[np.ix_(ys, xs)]
    e = lane_err(gh, h) + lane_err(gd, d)
    ec = channel_err(gh, h) + channel_err(gd, d)
    ej = scalar_err(gj - 1.0, j - 1.0)
    print(f"N={n} L={plane:g} sampled: lane {max(e):.2e} channel {max(ec):.2e} jac {ej:.2e}", flush=True)
    # the sampled reference IS the float64 transform of the oracle's spectrum
    return [(n, plane, float(s.time), max(e), ec, ej, float("nan"), max(ec), float("nan"), ej)]


def sample_lines(n, extra=10, seed=16384):
    """Rows / columns 0, 1, N/2 - 1, N/2, N/2 + 1, N - 1 and `extra` random ones (sorted, distinct)."""
    rng = np.random.default_rng(seed)
    fixed = [0, 1, n // 2 - 1, n // 2, n // 2 + 1, n - 1]
    rest = sorted(set(rng.integers(2, n - 2, 4 * extra).tolist()) - set(fixed))[:extra]
    return np.array(sorted(fixed + rest)), np.array(sorted(fixed + rest))


def main():
    O.build()
    rows = []
    rows += run(256, [5.0, 17.0, 101.0], [1 / 60, 1.0, 60.0, 600.0, 3600.0])
    rows += run(1024, [40.0], [1.0, 600.0])
    rows += run(2048, [40.0], [1.0])
    rows += run(4096, [5.0, 251.0, 4093.0], [1 / 60, 1.0])
    rows += run(8192, [40.0], [1.0])
    rows += run_sampled(16384, 40.0, 0.25)
    rows += run_sampled(16384, 1000.0, 1.0)
    lines = ["# GPU vs CPU oracle, full frames (max |err| / max |ref|)", "",
             "Columns 4-8: GPU against the oracle (fp32 restatement of the reference, radix-2 FFT). Columns 9-11: "
             "GPU and oracle against f64 = the oracle's own fp32 h0 and prepareFFT transformed in float64 "
             "(the sampled 16384 rows: f64 at the sample points only, so the oracle column is empty). Channels: "
             + ", ".join(CHANNELS) + ".", "",
             "| N | plane m | t s | maps lane err | maps channel err (worst channel) | per channel | Jacobian err "
             "| eps32 * w_max * t | GPU vs f64 (channel) | oracle vs f64 (channel) | GPU Jacobian vs f64 |",
             "|---|---|---|---|---|---|---|---|---|---|---|"]
    for n, L, t, e, ec, ej, s, g64, o64, gj64 in rows:
        w = int(np.argmax(ec))
        per = " ".join(f"{v:.1e}" for v in ec)
        lines.append(f"| {n} | {L:g} | {t:g} | {e:.2e} | {max(ec):.2e} ({CHANNELS[w]}) | {per} | {ej:.2e} | {s:.2e} "
                     f"| {g64:.2e} | {o64:.2e} | {gj64:.2e} |")
    out = os.path.join(ROOT, "gpurun_out")
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, "parity_report.md"), "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
