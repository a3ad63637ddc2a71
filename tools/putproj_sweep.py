"""One-GPU emulation of the 8-rank one-sided slab frame (bench.py p8_put_projection) over the put
stream's CU mask: K CUs of every XCD for the put (ocean_peers_set_put_cu_mask), the rest for step 1 and
the row passes. Prints each K's pipelined rank frame and its kernels under contention."""
import json
import sys
import time

sys.path.insert(0, '.')
import torch  # noqa: E402,F401

import bench  # noqa: E402

args = bench.parse(["--slab-steps", "10"])
out = {}
for rep in range(2):
    for k in (0, 4, 6, 8, 10, 12, 16):
        t = time.time()
        r = bench._put_emulation(args, 8, calibrate=False, per_xcd=k)
        out.setdefault(str(k), []).append(r)
        print(k, rep, round(r["pipelined_rank_frame_ms"], 4), {a: round(b, 3) for a, b in r["kernels_in_pipelined_frame"].items()},
              round(time.time() - t, 1), flush=True)
print(json.dumps(out))
