#!/usr/bin/env python3
"""Host model of tools/microbench/k_cols_small.h's fft8_run: the radix-8 Stockham index arithmetic (a first stage
of radix R0 = 2^(log2 N mod 3) with span 1, then radix-8 stages with span p; thread i holds x[i + m T],
T = N / 8, and ends holding X[i + m T]) played on the host against N * ifft
(tests/test_host_logic.py::test_fft8_index_model)."""
import numpy as np


def _idft(x):
    r = len(x)
    n = np.arange(r)
    return np.array([np.sum(x * np.exp(2j * np.pi * n * k / r)) for k in range(r)])


def fft8_model(x, logn):
    n = 1 << logn
    t_ = n >> 3
    log_r0 = logn % 3 if logn % 3 else 3
    r0 = 1 << log_r0
    nstage = 1 + (logn - log_r0) // 3
    u_ = 8 // r0
    v = np.array([[x[i + m * t_] for m in range(8)] for i in range(t_)], dtype=complex)
    y = np.zeros(n, dtype=complex)
    for i in range(t_):
        for u in range(u_):
            w = _idft(np.array([v[i, u + t * u_] for t in range(r0)]))
            for t in range(r0):
                y[(i + u * t_) * r0 + t] = w[t]
    v = np.array([[y[i + m * t_] for m in range(8)] for i in range(t_)])
    p = r0
    for _ in range(1, nstage):
        y = np.zeros(n, dtype=complex)
        for i in range(t_):
            k = i & (p - 1)
            w = _idft(v[i] * np.exp(2j * np.pi * np.arange(8) * k * (n // (8 * p)) / n))
            j = (i // p) * 8 * p + k
            for t in range(8):
                y[j + t * p] = w[t]
        v = np.array([[y[i + m * t_] for m in range(8)] for i in range(t_)])
        p *= 8
    return y


if __name__ == "__main__":
    for logn in (9, 10, 11, 12):
        x = np.random.default_rng(logn).standard_normal(1 << logn) + 0j
        print(logn, np.max(np.abs(fft8_model(x, logn) - np.fft.ifft(x) * (1 << logn))))
