#!/usr/bin/env python3
"""Diagnostic (GPU box): where does a full frame's GPU-vs-oracle error come from? Compares h0,
one-frame and two-frame results, against the oracle and a float64 transform of the oracle's
packed spectra. Prints one line per check."""
import sys

sys.path[:0] = ['/root/repo', '/root/repo/tests']
import torch  # noqa: F401  (one HIP runtime, see tests/conftest.py)
import numpy as np

import oceansimulation_amd as ocean
from oracle import oracle as O
import numpy_ref as R
from parity import lane_err

O.build()
O.set_threads(16)
for n, L in ((4096, 23.0), (2048, 23.0)):
    s0 = O.default_settings(planeSize=L)
    fft = ocean.FFTCalculator(n)
    g1 = ocean.Generator(fft, 1)
    ocean.apply_settings(g1.GetOceanSettings(0), planeSize=L)
    g1.GenerateSpectrum()
    h0_gpu = g1.initial_spectrum_host(0)
    h0_ref = O.generate_spectrum(s0, n)
    print(n, L, "h0 gpu-vs-oracle", lane_err(h0_gpu, h0_ref))
    # one frame at t = 0.7666667
    t = np.float32(0.75) + np.float32(1.0 / 60.0)
    g1.CalculateOcean(float(t), update_ocean=True)
    s = O.default_settings(planeSize=L)
    s.time = float(t)
    hp, dp = O.prepare_fft(s, n, h0_ref)
    f64h, f64d = R.encode_ifft(hp), R.encode_ifft(dp)
    print(n, L, "1 frame gpu-vs-f64", lane_err(g1.height_map_host(0), f64h), lane_err(g1.displacement_map_host(0), f64d))
    g2 = ocean.Generator(fft, 1)
    ocean.apply_settings(g2.GetOceanSettings(0), planeSize=L)
    g2.CalculateOcean(0.75)
    g2.CalculateOcean(1.0 / 60.0)
    print(n, L, "2 frames gpu-vs-f64", lane_err(g2.height_map_host(0), f64h), lane_err(g2.displacement_map_host(0), f64d))
    # the packed spectra themselves: EncodeIFFT of the oracle's packed images on the GPU
    from oceansimulation_amd.hip import DeviceBuffer
    b = DeviceBuffer.from_array(np.stack([hp, dp]))
    fft.encode_ifft_batch(b.ptr, 2)
    fft.synchronize()
    e = b.to_host((2, n, n, 4))
    print(n, L, "EncodeIFFT(oracle packed) vs f64", lane_err(e[0], f64h), lane_err(e[1], f64d))
