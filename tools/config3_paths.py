"""BASELINE config 3 (2048^2, full payload) on the frame paths the generator offers: the half
spectrum (production: 84 B/pt), the same with frame overlap, and the full spectrum (116 B/pt), at one
and four cascades; wall ms per frame (200 frames, medians of 5 runs) and the kernels' ms (HIP events)."""
import json
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: E402

import oceansimulation_amd as ocean  # noqa: E402


def run(n, planes, half, overlap, steps=200):
    fft = ocean.FFTCalculator(n)
    gen = ocean.Generator(fft, len(planes))
    for c, L in enumerate(planes):
        ocean.apply_settings(gen.GetOceanSettings(c), planeSize=L)
    gen.set_half_spectrum(half)
    if overlap:
        gen.set_frame_overlap(True)
    for _ in range(10):
        gen.CalculateOcean(1 / 60)
    walls = []
    for _ in range(5):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            gen.CalculateOcean(1 / 60)
        torch.cuda.synchronize()
        walls.append(1e3 * (time.perf_counter() - t0) / steps)
    gen.set_frame_overlap(False)
    gen.set_profiling(True)
    gen.kernel_times()
    for _ in range(steps):
        gen.CalculateOcean(1 / 60)
    ms, cnt = gen.kernel_times()
    b = sum(gen.frame_bytes())
    gen.close()
    fft.close()
    walls.sort()
    return {"wall_ms": walls[2], "cols_ms": ms[1] / max(cnt[1], 1), "rows_ms": ms[2] / max(cnt[2], 1), "bytes_per_pt": b}


out = {}
for planes in ([40.0], [5.0, 17.0, 101.0, 251.0]):
    key = f"{len(planes)}_cascades"
    out[key] = {"half": run(2048, planes, True, False), "half_overlap": run(2048, planes, True, True),
                "full": run(2048, planes, False, False)}
print(json.dumps(out, indent=1))
