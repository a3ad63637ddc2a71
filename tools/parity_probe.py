#!/usr/bin/env python3
"""Where a frame's error sits: GPU (half and full spectrum) against the float64 transform of the
oracle's spectrum (tools/parity_report.f64_frame), per channel, with the location of the worst texel
and the error restricted to rows/columns 0 and N/2. Usage: python tools/parity_probe.py [N L t]"""
import copy
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402

import numpy_ref as R  # noqa: E402
import oceansimulation_amd as ocean  # noqa: E402
from oracle import oracle as O  # noqa: E402

CH = ["h", "dh/dx", "dh/dz", "Dx", "Dz", "dDx/dx", "dDz/dz", "dDx/dz"]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    L = float(sys.argv[2]) if len(sys.argv) > 2 else 251.0
    t = float(sys.argv[3]) if len(sys.argv) > 3 else 1.0 / 60.0
    O.build()
    ref = O.OracleGenerator(n, O.default_settings(planeSize=L))
    ref.calculate_ocean(t)
    s = copy.copy(ref.settings)
    hp, dp = O.prepare_fft(s, n, ref.h0)
    f64 = np.concatenate([R.encode_ifft(hp), R.encode_ifft(dp)], -1).astype(np.float64)
    orc = np.concatenate([ref.height, ref.disp], -1).astype(np.float64)
    fft = ocean.FFTCalculator(n)
    outs = {}
    for half in (True, False):
        g = ocean.Generator(fft, 1)
        g.set_half_spectrum(half)
        ocean.apply_settings(g.GetOceanSettings(0), planeSize=L)
        g.CalculateOcean(t)
        outs["half" if half else "full"] = np.concatenate([g.height_map_host(0), g.displacement_map_host(0)], -1)
        h0 = g.initial_spectrum_host(0).astype(np.float64)
        dh0 = np.abs(h0 - ref.h0)
        print(f"{'half' if half else 'full'}: h0 max|diff| / max|h0| = {dh0.max() / np.abs(ref.h0).max():.2e} "
              f"at {np.unravel_index(np.argmax(dh0.max(-1)), dh0.shape[:2])}", flush=True)
        if half:
            gpu_h0 = g.initial_spectrum_host(0)
    # h0 texel by texel: relative error where |h0| is not negligible, and |k|^2-weighted (slope-like)
    mag = np.abs(ref.h0.astype(np.float64)).max(-1)
    rel = np.abs(gpu_h0.astype(np.float64) - ref.h0).max(-1) / np.maximum(mag, 1e-30)
    kk2 = np.add.outer((np.arange(n) - n // 2) ** 2, (np.arange(n) - n // 2) ** 2).astype(np.float64)
    for thr in (1e-2, 1e-4, 1e-6):
        m = mag > thr * mag.max()
        t = np.argmax(np.where(m, rel, 0))
        y, x = np.unravel_index(t, rel.shape)
        print(f"h0 texels with |h0| > {thr:g} max: worst relative error {rel[y, x]:.2e} at (x={x}, y={y}) "
              f"(u={x - n // 2}, v={y - n // 2}), |h0| {mag[y, x]:.2e}", flush=True)
    wk = np.abs(gpu_h0.astype(np.float64) - ref.h0).max(-1) * kk2
    print(f"h0 |k|^2-weighted: max |k|^2 |dh0| / max |k|^2 |h0| = {wk.max() / (mag * kk2).max():.2e}", flush=True)
    # the spectrum from the GPU's own h0 through the oracle's prepareFFT: splits h0 error from the rest
    hpg, dpg = O.prepare_fft(s, n, gpu_h0)
    spec_g = np.concatenate([hpg, dpg], -1).astype(np.float64)
    spec_o = np.concatenate([hp, dp], -1).astype(np.float64)
    for lane, what in ((0, "h + i dh/dx"), (4, "Dz + i dDx/dx")):
        a = spec_g[..., lane] + 1j * spec_g[..., lane + 1]
        b = spec_o[..., lane] + 1j * spec_o[..., lane + 1]
        print(f"prepareFFT(GPU h0) vs prepareFFT(oracle h0), lane '{what}': |sum dX| / |sum X| "
              f"{abs((a - b).sum()) / abs(b.sum()):.2e}", flush=True)
    outs["oracle"] = orc
    # the spectrum each output implies (forward transform in float64, the inverse of EncodeIFFT's
    # convention) against the oracle's prepareFFT spectrum: where the frame's error comes from
    spec = np.concatenate([hp, dp], -1).astype(np.float64)
    for name in ("half", "oracle"):
        a = outs[name].astype(np.float64)
        for lane, what in ((0, "h + i dh/dx"), (2, "dh/dz + i Dx"), (4, "Dz + i dDx/dx"), (6, "dDz/dz + i dDx/dz")):
            z = a[..., lane] + 1j * a[..., lane + 1]
            X = np.fft.fftshift(np.fft.fft2(z)) / (n * n)
            R0 = spec[..., lane] + 1j * spec[..., lane + 1]
            d = np.abs(X - R0)
            top = np.argsort(d.ravel())[::-1][:6]
            print(f"== spectrum of {name} lane '{what}': max|dX| / max|X| {d.max() / np.abs(R0).max():.2e}, "
                  f"|sum dX| / |sum X| {abs((X - R0).sum()) / abs(R0.sum()):.2e} (the error at the origin), "
                  f"sum|dX| / |sum X| {d.sum() / abs(R0.sum()):.2e}", flush=True)
            # the coherent part by |k| band: where sum(dX) (the origin's error) is made
            kk = np.hypot(*np.meshgrid(np.arange(n) - n // 2, np.arange(n) - n // 2))
            bands = [0, 1, 2, 4, 8, 16, 64, 256, 1024, 4096]
            parts = []
            for lo, hi in zip(bands[:-1], bands[1:]):
                m = (kk >= lo) & (kk < hi)
                parts.append(f"[{lo},{hi}) {abs((X - R0)[m].sum()) / abs(R0.sum()):.1e}")
            print("    origin error by |k| band: " + " ".join(parts), flush=True)
            for tt in top:
                j, i = np.unravel_index(tt, d.shape)
                print(f"    (u={i - n // 2}, v={j - n // 2}) |dX| {d[j, i]:.3e} |X| {abs(R0[j, i]):.3e} "
                      f"X_gpu {X[j, i]:.4e} X_ref {R0[j, i]:.4e}", flush=True)
    for name, a in outs.items():
        a = a.astype(np.float64)
        print(f"== {name} vs f64 (N={n} L={L:g} t={t:g})")
        for c in range(8):
            err = np.abs(a[..., c] - f64[..., c])
            scale = np.abs(f64[..., c]).max()
            y, x = np.unravel_index(np.argmax(err), err.shape)
            lines = {"row0": err[0].max(), "rowN2": err[n // 2].max(), "col0": err[:, 0].max(), "colN2": err[:, n // 2].max()}
            print(f"  {CH[c]:7s} max|ref| {scale:.3e}  err {err.max() / scale:.2e} at (x={x}, y={y})  "
                  + " ".join(f"{k} {v / scale:.1e}" for k, v in lines.items()) + f"  rms {np.sqrt((err ** 2).mean()) / scale:.1e}",
                  flush=True)


if __name__ == "__main__":
    main()
