import sys
sys.path[:0] = ['/root/repo', '/root/repo/tests']
import torch  # noqa
import numpy as np
import oceansimulation_amd as ocean
from oracle import oracle as O
O.build(); O.set_threads(16)
n, L = 4096, 23.0
fft = ocean.FFTCalculator(n); g = ocean.Generator(fft, 1)
ocean.apply_settings(g.GetOceanSettings(0), planeSize=L)
g.GenerateSpectrum()
a = g.initial_spectrum_host(0).astype(np.float64); r = O.generate_spectrum(O.default_settings(planeSize=L), n).astype(np.float64)
za = a[..., 0] + 1j * a[..., 1]; zr = r[..., 0] + 1j * r[..., 1]
y, x = np.meshgrid(np.arange(n), np.arange(n), indexing="ij")
k = np.hypot(x - n / 2, y - n / 2) * (2 * np.pi / L)
err = np.abs(za - zr); mag = np.abs(zr)
print("max|h0| err/max", err.max() / mag.max(), " k-weighted", (k * err).max() / (k * mag).max(), " k^2-weighted", (k*k*err).max()/(k*k*mag).max())
rel = err / np.maximum(mag, 1e-30)
for lo, hi in ((0, 1), (1, 10), (10, 50), (50, 200), (200, 500), (500, 1000)):
    m = (k >= lo) & (k < hi) & (mag > 0)
    if m.any():
        print(f"k in [{lo},{hi}): median rel {np.median(rel[m]):.2e}  p99 {np.percentile(rel[m], 99):.2e}  max {rel[m].max():.2e}  max|ref| {mag[m].max():.2e}")
i = np.argmax(k * err); print("worst k-weighted texel", np.unravel_index(i, k.shape), k.flat[i], za.flat[i], zr.flat[i])
