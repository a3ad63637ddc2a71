#!/usr/bin/env python3
"""Summarise tools/profile_gpu.sh output into profiles/<tag>_rocprof.{md,json}.

HBM traffic per launch, corrected as MI355X_MICROARCH.md §HBM prescribes for gfx950:
  read  bytes = 2 * FETCH_SIZE * 1024   (FETCH_SIZE counts 128-B requests as 64 B; unit KB)
  write bytes =     WRITE_SIZE * 1024   (exact for 16-B-per-lane streaming stores)
Algorithmic bytes per launch come from the bench config (N, cascades) and DESIGN.md's per-point
figures. Usage: tools/parse_rocprof.py <gpurun_out dir> <tag> [n] [cascades] [prefix] [frame|ifft]
"""
import csv
import hashlib
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def device_source_sha256(root=ROOT):
    """Hash of the device code the kernels are built from (csrc/*.hip, csrc/*.h, device/*.h, sorted):
    bench.py takes roofline.traffic only from a summary whose hash equals the running tree's."""
    csrc = os.path.join(root, "oceansimulation_amd", "csrc")
    files = sorted(os.path.join(csrc, f) for f in os.listdir(csrc) if f.endswith(".hip") or f.endswith(".h"))
    files += sorted(os.path.join(csrc, "device", f) for f in os.listdir(os.path.join(csrc, "device")) if f.endswith(".h"))
    h = hashlib.sha256()
    for f in files:
        with open(f, "rb") as fh:
            h.update(os.path.relpath(f, root).encode() + b"\0" + fh.read())
    return h.hexdigest()


def base_name(symbol):
    """k_rows_half from 'void oceanfft::k_rows_half<12, 0, ...>(oceanfft::FrameParams, ...)'."""
    s = symbol.split("(")[0].replace("void ", "").replace("oceanfft::", "").strip()
    return s.split("<")[0]


def size_key(symbol, logn):
    """The summary key: the base name for instantiations at the workload's log2 N (what bench.py
    looks up), else base<first template argument> (other sizes: k_rows_half<14>, k_gen4_step2<10>)."""
    s = symbol.split("(")[0].replace("void ", "").replace("oceanfft::", "").strip()
    if "<" not in s:
        return s
    first = s.split("<", 1)[1].split(",")[0].split(">")[0].strip()
    return s.split("<")[0] if first == str(logn) else f"{s.split('<')[0]}<{first}>"

src, tag = sys.argv[1], sys.argv[2]
n = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
cascades = int(sys.argv[4]) if len(sys.argv) > 4 else 8
prefix = sys.argv[5] if len(sys.argv) > 5 else "prof"  # tools/profile_gpu.sh PREFIX
mode = sys.argv[6] if len(sys.argv) > 6 else "frame"  # frame | ifft (EncodeIFFT chunks of 8 images)
pts = n * n * cascades
kept = (n // 2 + 4) / n  # half-spectrum path: columns u in [0, N/2) plus the 4-wide Nyquist strip
ALGO = {"k_cols_evolve": 48 * pts, "k_rows_final": 68 * pts, "k_generate_spectrum": 16 * n * n,
        "k_generate_spectrum_pairs": 16 * n * n,
        "k_cols_half": int((16 + 40) * kept * pts), "k_rows_half": int((40 * kept + 36) * pts),
        "k_gen4_step1": int((16 + 40) * kept * pts)}
if mode == "ifft":  # standalone EncodeIFFT at 4096: work-image chunks of 8 images, 32 B per texel per pass
    ALGO["k_cols_to_blocks"] = ALGO["k_rows_final"] = 32 * 8 * n * n


def read_csv(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def find(sub, suffix):
    d = os.path.join(src, sub)
    for fn in os.listdir(d):
        if fn.endswith(suffix):
            return os.path.join(d, fn)
    raise FileNotFoundError(f"{d}/*{suffix}")


stats = {}
for r in read_csv(find(prefix + "_trace", "kernel_stats.csv")):
    stats[r["Name"]] = r
counters = {}
for sub, name in ((prefix + "_fetch", "FETCH_SIZE"), (prefix + "_write", "WRITE_SIZE")):
    for r in read_csv(find(sub, "counter_collection.csv")):
        if r["Counter_Name"] == name:
            counters.setdefault(r["Kernel_Name"], {}).setdefault(name, []).append(float(r["Counter_Value"]))
# full symbols (no -T): aggregate per base name, keeping the symbols each base name covered
by_base = {}
logn = n.bit_length() - 1
for sym in list(stats) + list(counters):
    by_base.setdefault(size_key(sym, logn), set()).add(sym)

out = {"tag": tag, "n": n, "cascades": cascades, "device_source_sha256": device_source_sha256(), "kernels": {}}
lines = [f"# rocprofv3 summary — {tag}", "",
         f"Workload: bench.py, {cascades} cascades of {n}x{n} per launch. Durations: `--kernel-trace --stats`. "
         "Traffic: separate `--pmc FETCH_SIZE` and `--pmc WRITE_SIZE` passes; read = 2 x FETCH_SIZE (gfx950 "
         "half-count correction), write = WRITE_SIZE; KB = 1024 B.", "",
         "| kernel | calls | avg ms | algorithmic GB/launch | measured HBM GB/launch (read + write) | traffic / algorithmic | achieved GB/s (algorithmic) |",
         "|---|---|---|---|---|---|---|"]
for name in sorted(by_base):
    syms = by_base[name]
    st_list = [stats[sy] for sy in syms if sy in stats]
    if not st_list:
        continue
    calls = sum(int(st["Calls"]) for st in st_list)
    avg_ms = sum(float(st["AverageNs"]) * int(st["Calls"]) for st in st_list) / calls / 1e6
    fe = [v for sy in syms for v in counters.get(sy, {}).get("FETCH_SIZE", [])]
    wr_ = [v for sy in syms for v in counters.get(sy, {}).get("WRITE_SIZE", [])]
    rd = statistics.median(fe) * 1024 * 2 if fe else None
    wr = statistics.median(wr_) * 1024 if wr_ else None
    algo = ALGO.get(name)
    traffic = (rd + wr) if (rd is not None and wr is not None) else None
    rec = {"calls": calls, "avg_ms": avg_ms, "algorithmic_bytes": algo, "hbm_read_bytes": rd,
           "hbm_write_bytes": wr, "hbm_traffic_bytes": traffic, "symbols": sorted(syms)}
    if algo:
        rec["achieved_GBps_algorithmic"] = algo / (avg_ms * 1e-3) / 1e9
    out["kernels"][name] = rec
    f = lambda v: "-" if v is None else f"{v / 1e9:.3f}"
    ratio = f"{traffic / algo:.3f}" if (traffic and algo) else "-"
    ach = f"{rec['achieved_GBps_algorithmic']:.0f}" if algo else "-"
    lines.append(f"| {name} | {calls} | {avg_ms:.3f} | {f(algo)} | {f(rd)} + {f(wr)} | {ratio} | {ach} |")
lines += ["", f"Device source sha256: `{out['device_source_sha256']}` (bench.py uses this summary's traffic only for "
          "the same device code)."]
os.makedirs("profiles", exist_ok=True)
with open(f"profiles/{tag}_rocprof.json", "w") as fh:
    json.dump(out, fh, indent=1)
with open(f"profiles/{tag}_rocprof.md", "w") as fh:
    fh.write("\n".join(lines) + "\n")
print("\n".join(lines))
