#!/usr/bin/env python3
"""A/B of the whole-grid frame paths at N = 8192 / 16384 on one GPU: the four-step column pass
(ocean_generator_set_four_step(1), default) against the strip-dealt column pass + transposes, both
timed with the generator's own HIP events (ocean_generator_set_profiling), same box, interleaved;
and their maps compared (max |diff| / max |value| per lane: different factorisations of the same
transform, so not bit-identical). Usage: python tools/gen4_ab.py [frames]"""
import sys
import time

import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import oceansimulation_amd as ocean  # noqa: E402

frames = int(sys.argv[1]) if len(sys.argv) > 1 else 10
for n, C in ((8192, 2), (16384, 1)):
    fft = ocean.FFTCalculator(n)
    gens = [ocean.Generator(fft, C), ocean.Generator(fft, C)]
    gens[1].set_four_step(False)
    for g in gens:
        for c in range(C):
            ocean.apply_settings(g.GetOceanSettings(c), planeSize=[1000.0, 251.0][c % 2])
        g.CalculateOcean(0.5)
    fft.synchronize()
    for c in range(C):
        for get in ("height_map_host", "displacement_map_host"):
            a, b = getattr(gens[0], get)(c), getattr(gens[1], get)(c)
            err = [float(np.abs(a[..., k] - b[..., k]).max() / max(np.abs(b[..., k]).max(), 1e-30)) for k in range(4)]
            print(f"N={n} cascade {c} {get}: four-step vs dealt max rel diff per lane {['%.2e' % e for e in err]}")
            del a, b
    res = {0: [], 1: []}
    for rep in range(3):
        for k, g in enumerate(gens):
            g.set_profiling(True)
            g.kernel_times()
            for _ in range(frames):
                g.CalculateOcean(1.0 / 60.0)
            fft.synchronize()
            ms, cnt = g.kernel_times()
            g.set_profiling(False)
            res[k].append((ms[1] / max(cnt[1], 1), ms[2] / max(cnt[2], 1)))
    for k, name in ((0, "four-step"), (1, "dealt + transposes")):
        cols = sorted(r[0] for r in res[k])[1]
        rows = sorted(r[1] for r in res[k])[1]
        print(f"N={n} x{C} {name:20s} column phase {cols:7.3f} ms  row phase {rows:7.3f} ms  frame {cols + rows:7.3f} ms")
    for g in gens:
        g.close()
    fft.close()
