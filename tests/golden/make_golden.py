#!/usr/bin/env python3
"""Generate tests/golden/ocean_golden.npz — regression vectors for the ocean hot path.

The reference (James51332/OceanSimulation) ships no tests, fixtures or golden data, and its GLSL
path cannot run here (Vision engine absent), so these vectors come from the CPU oracle
(oracle/ocean_oracle.c, a float32 restatement of the GLSL) and are accepted only after an
independent numpy formulation (tests/numpy_ref.py) agrees with them (checks below). Parity status:
unpinned by reference outputs — see DESIGN.md §Oracle.

Cases (CalculateOcean state after the given frames; settings per src/Generator.h:14-29 and the
WaveApp cascades of src/Waves.cpp:24-35):
  n16_L{5,17,101}   N=16,  two frames: dt = 0.5 then 0.5 (time = 1.0)
  n64_L{5,17,101}   N=64,  one frame, dt = 1.0
  n256_L40          N=256, one frame, dt = 1.0 (default settings, the reference's native size)
Each case stores h0 (row-major N x N x 4), heightMap, displacementMap (N x N x 4), jacobian (N x N).
Usage: python tests/golden/make_golden.py   (rewrites the .npz and manifest.json)
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

from oracle import oracle as O  # noqa: E402
import numpy_ref as R  # noqa: E402
from parity import lane_err, scalar_err  # noqa: E402

PLANES = [5.0, 17.0, 101.0]


def cases():
    out = []
    for i, L in enumerate(PLANES):
        kw = dict(planeSize=L, boundWavelength=1, wavelengthMax=L / 2.0,
                  wavelengthMin=0.0 if i == 0 else PLANES[i - 1] / 2.0)
        out.append((f"n16_L{int(L)}", 16, kw, [0.5, 0.5]))
    for i, L in enumerate(PLANES):
        kw = dict(planeSize=L, boundWavelength=1, wavelengthMax=L / 2.0,
                  wavelengthMin=0.0 if i == 0 else PLANES[i - 1] / 2.0)
        out.append((f"n64_L{int(L)}", 64, kw, [1.0]))
    out.append(("n256_L40", 256, {}, [1.0]))
    return out


def run_case(n, kw, dts):
    g = O.OracleGenerator(n, O.default_settings(**kw))
    for dt in dts:
        g.calculate_ocean(dt)
    return g


def cross_check(name, n, g):
    """Independent numpy formulation must agree before a vector is accepted."""
    s = g.settings
    h0n = R.generate_spectrum(s, n)
    hm, dm = R.prepare_fft(s, n, g.h0)
    e_h0 = max(lane_err(h0n, g.h0))
    hm_o, dm_o = O.prepare_fft(s, n, g.h0)
    e_prep = max(lane_err(hm, hm_o) + lane_err(dm, dm_o))
    e_fft = max(lane_err(R.encode_ifft(hm_o), g.height) + lane_err(R.encode_ifft(dm_o), g.disp))
    e_jac = scalar_err(R.compute_foam(s, g.disp) - 1.0, g.jac - 1.0)
    ok = e_h0 < 1e-6 and e_prep < 1e-6 and e_fft < 1e-5 and e_jac < 1e-6
    print(f"{name}: numpy vs oracle  h0 {e_h0:.2e}  evolve {e_prep:.2e}  ifft {e_fft:.2e}  foam {e_jac:.2e}"
          f"  {'OK' if ok else 'MISMATCH'}")
    return ok, dict(h0=e_h0, evolve=e_prep, ifft=e_fft, foam=e_jac)


def main():
    O.build()
    O.set_threads(min(8, os.cpu_count() or 1))
    arrays, manifest = {}, {"source": "oracle/ocean_oracle.c (CPU restatement), cross-checked with tests/numpy_ref.py",
                            "parity": "unpinned by reference outputs (reference has no fixtures; GLSL not runnable)",
                            "cases": {}}
    all_ok = True
    for name, n, kw, dts in cases():
        g = run_case(n, kw, dts)
        ok, errs = cross_check(name, n, g)
        all_ok &= ok
        arrays[f"{name}/h0"] = g.h0
        arrays[f"{name}/height"] = g.height
        arrays[f"{name}/disp"] = g.disp
        arrays[f"{name}/jac"] = g.jac
        manifest["cases"][name] = {"n": n, "settings": kw, "timesteps": dts, "final_time": float(g.settings.time),
                                   "numpy_cross_check_max_rel_err": errs}
    if not all_ok:
        raise SystemExit("numpy cross-check failed; fixtures not written")
    np.savez_compressed(os.path.join(HERE, "ocean_golden.npz"), **arrays)
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print("wrote", os.path.join(HERE, "ocean_golden.npz"))


if __name__ == "__main__":
    main()
