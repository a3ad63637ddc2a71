import json, sys, time
sys.path.insert(0, '.')
import torch
import bench
args = bench.parse(["--slab-steps", "10"])
t = time.time()
out = bench.p8_put_projection(args, 7.30)
out["wall_s"] = time.time() - t
print(json.dumps(out, indent=1))
