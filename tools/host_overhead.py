"""Host cost of the frame API: per CalculateOcean call, the time to enqueue (no synchronisation)
against the wall time per frame, for 1 and 8 cascades of 4096^2 (a diagnostic for the one-cascade
share, where the GPU frame is ~0.3 ms)."""
import json
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: E402

import oceansimulation_amd as ocean  # noqa: E402
from bench import cascade_settings  # noqa: E402

out = {}
for C in (1, 8):
    fft = ocean.FFTCalculator(4096)
    gen = ocean.Generator(fft, C)
    for c in range(C):
        ocean.apply_settings(gen.GetOceanSettings(c), **cascade_settings(0, c))
    for _ in range(5):
        gen.CalculateOcean(1 / 60)
    torch.cuda.synchronize()
    steps = 200
    t0 = time.perf_counter()
    for _ in range(steps):
        gen.CalculateOcean(1 / 60)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    # the host side alone: the same calls timed one by one after a synchronize each (queue empty)
    host = []
    for _ in range(50):
        torch.cuda.synchronize()
        a = time.perf_counter()
        gen.CalculateOcean(1 / 60)
        host.append(time.perf_counter() - a)
    torch.cuda.synchronize()
    host.sort()
    out[str(C)] = {"enqueue_ms_per_frame": 1e3 * (t1 - t0) / steps, "wall_ms_per_frame": 1e3 * (t2 - t0) / steps,
                   "host_call_ms_median": 1e3 * host[len(host) // 2]}
    gen.close()
    fft.close()
print(json.dumps(out))
