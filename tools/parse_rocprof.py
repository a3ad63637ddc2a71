#!/usr/bin/env python3
"""Summarise tools/profile_gpu.sh output into profiles/<tag>_rocprof.{md,json}.

HBM traffic per launch, corrected as MI355X_MICROARCH.md §HBM prescribes for gfx950:
  read  bytes = 2 * FETCH_SIZE * 1024   (FETCH_SIZE counts 128-B requests as 64 B; unit KB)
  write bytes =     WRITE_SIZE * 1024   (exact for 16-B-per-lane streaming stores)
Algorithmic bytes per launch come from the bench config (N, cascades) and DESIGN.md's per-point
figures. Usage: tools/parse_rocprof.py <gpurun_out dir> <tag> [n] [cascades]
"""
import csv
import json
import os
import statistics
import sys

src, tag = sys.argv[1], sys.argv[2]
n = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
cascades = int(sys.argv[4]) if len(sys.argv) > 4 else 8
pts = n * n * cascades
kept = (n // 2 + 4) / n  # half-spectrum path: columns u in [0, N/2) plus the 4-wide Nyquist strip
ALGO = {"k_cols_evolve": 48 * pts, "k_rows_final": 68 * pts, "k_generate_spectrum": 16 * n * n,
        "k_generate_spectrum_pairs": 16 * n * n,
        "k_cols_half": int((16 + 40) * kept * pts), "k_rows_half": int((40 * kept + 36) * pts)}


def read_csv(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def find(sub, suffix):
    d = os.path.join(src, sub)
    for fn in os.listdir(d):
        if fn.endswith(suffix):
            return os.path.join(d, fn)
    raise FileNotFoundError(f"{d}/*{suffix}")


stats = {r["Name"]: r for r in read_csv(find("prof_trace", "kernel_stats.csv"))}
counters = {}
for sub, name in (("prof_fetch", "FETCH_SIZE"), ("prof_write", "WRITE_SIZE")):
    for r in read_csv(find(sub, "counter_collection.csv")):
        if r["Counter_Name"] == name:
            counters.setdefault(r["Kernel_Name"], {}).setdefault(name, []).append(float(r["Counter_Value"]))

out = {"tag": tag, "n": n, "cascades": cascades, "kernels": {}}
lines = [f"# rocprofv3 summary — {tag}", "",
         f"Workload: bench.py, {cascades} cascades of {n}x{n} per launch. Durations: `--kernel-trace --stats`. "
         "Traffic: separate `--pmc FETCH_SIZE` and `--pmc WRITE_SIZE` passes; read = 2 x FETCH_SIZE (gfx950 "
         "half-count correction), write = WRITE_SIZE; KB = 1024 B.", "",
         "| kernel | calls | avg ms | algorithmic GB/launch | measured HBM GB/launch (read + write) | traffic / algorithmic | achieved GB/s (algorithmic) |",
         "|---|---|---|---|---|---|---|"]
for name, st in stats.items():
    avg_ms = float(st["AverageNs"]) / 1e6
    c = counters.get(name, {})
    rd = statistics.median(c["FETCH_SIZE"]) * 1024 * 2 if "FETCH_SIZE" in c else None
    wr = statistics.median(c["WRITE_SIZE"]) * 1024 if "WRITE_SIZE" in c else None
    algo = ALGO.get(name)
    traffic = (rd + wr) if (rd is not None and wr is not None) else None
    rec = {"calls": int(st["Calls"]), "avg_ms": avg_ms, "algorithmic_bytes": algo, "hbm_read_bytes": rd,
           "hbm_write_bytes": wr, "hbm_traffic_bytes": traffic}
    if algo:
        rec["achieved_GBps_algorithmic"] = algo / (avg_ms * 1e-3) / 1e9
    out["kernels"][name] = rec
    f = lambda v: "-" if v is None else f"{v / 1e9:.3f}"
    ratio = f"{traffic / algo:.3f}" if (traffic and algo) else "-"
    ach = f"{rec['achieved_GBps_algorithmic']:.0f}" if algo else "-"
    lines.append(f"| {name} | {st['Calls']} | {avg_ms:.3f} | {f(algo)} | {f(rd)} + {f(wr)} | {ratio} | {ach} |")
os.makedirs("profiles", exist_ok=True)
with open(f"profiles/{tag}_rocprof.json", "w") as fh:
    json.dump(out, fh, indent=1)
with open(f"profiles/{tag}_rocprof.md", "w") as fh:
    fh.write("\n".join(lines) + "\n")
print("\n".join(lines))
