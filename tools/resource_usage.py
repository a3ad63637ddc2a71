#!/usr/bin/env python3
"""Print per-kernel VGPR / AGPR / scratch / occupancy for a .hip file (hipcc -Rpass-analysis)."""
import re, subprocess, sys

src = sys.argv[1]
extra = sys.argv[2:]
cmd = ["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c", src, "-o", "/dev/null",
       "-Rpass-analysis=kernel-resource-usage"] + extra
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark:\s+(.*?)\s*\[-Rpass", line)
    if not m:
        continue
    body = m.group(1)
    if body.startswith("Function Name:"):
        name = body.split(":", 1)[1].strip()
        dem = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        dem = re.sub(r"HIP_vector_type<float, (\d)u>", r"float\1", dem)
        cur = {"name": dem.split("(")[0].replace("oceanfft::", "")}
        rows.append(cur)
    elif cur is not None and ":" in body:
        k, v = body.split(":", 1)
        cur[k.strip()] = v.strip()
for r in rows:
    print(f"{r['name']:<34} vgpr={r.get('VGPRs','?'):>4} agpr={r.get('AGPRs','?'):>3} "
          f"scratch={r.get('ScratchSize [bytes/lane]','?'):>5} occ={r.get('Occupancy [waves/SIMD]','?')}")
