#!/usr/bin/env python3
"""GPU-vs-oracle error table for full CalculateOcean frames, including long simulated times.

Metric (tests/parity.py): max |got - ref| / max |ref| per complex lane (worst of the 4 lanes of
the two maps) and for the Jacobian - 1. Also prints the phase-precision scale eps32 * w_max * t:
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

import oceansimulation_amd as ocean  # noqa: E402
from oracle import oracle as O  # noqa: E402
from parity import lane_err, scalar_err  # noqa: E402

G = 9.81


def omega_max(n, plane, depth, g=G):
    k = math.pi * n / plane * math.sqrt(2.0)
    return math.sqrt((g * k + 0.074 / 1000.0 * k ** 3) * math.tanh(min(k * depth, 20.0)))


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
            e = lane_err(gen.height_map_host(c), refs[c].height) + lane_err(gen.displacement_map_host(c), refs[c].disp)
            ej = scalar_err(gen.jacobian_map_host(c) - 1.0, refs[c].jac - 1.0)
            depth = refs[c].settings.h
            scale = 2.0 ** -23 * omega_max(n, L, depth, refs[c].settings.g) * gen.GetOceanSettings(c).time
            rows.append((n, L, float(gen.GetOceanSettings(c).time), max(e), ej, scale))
    return rows


def main():
    O.build()
    rows = []
    rows += run(256, [5.0, 17.0, 101.0], [1 / 60, 1.0, 60.0, 600.0, 3600.0])
    rows += run(1024, [40.0], [1.0, 600.0])
    rows += run(4096, [40.0], [1.0])
    lines = ["# GPU vs CPU oracle, full frames (max |err| / max |ref|)", "",
             "| N | plane m | t s | maps lane err | Jacobian err | eps32 * w_max * t |", "|---|---|---|---|---|---|"]
    for n, L, t, e, ej, s in rows:
        lines.append(f"| {n} | {L:g} | {t:g} | {e:.2e} | {ej:.2e} | {s:.2e} |")
    out = os.path.join(ROOT, "gpurun_out")
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, "parity_report.md"), "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
