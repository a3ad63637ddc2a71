"""oceansimulation_amd — MI355X-native (gfx950 HIP) Tessendorf ocean height-field hot path.

Drop-in for the h0 -> h(k,t) -> 2D iFFT path of James51332/OceanSimulation
(Waves::Generator / Waves::FFTCalculator). The compute lives in liboceanfft.so (C ABI,
include/oceanfft.h); this package is its ctypes binding plus a Python mirror of the reference
classes used by the tests and bench.py.
"""
from .capi import OceanError, OceanSettings, lib  # noqa: F401
from .waves import FFTCalculator, Generator, default_settings, apply_settings  # noqa: F401

__all__ = ["FFTCalculator", "Generator", "OceanSettings", "OceanError", "default_settings", "apply_settings", "lib"]
