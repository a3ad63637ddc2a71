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


HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E peak


def base_name(symbol):
    """k_rows_half from 'void oceanfft::k_rows_half<12, 0, ...>(oceanfft::FrameParams, ...)'."""
    s = symbol.split("(")[0].replace("void ", "").replace("oceanfft::", "").strip()
    return s.split("<")[0]


def first_arg(symbol):
    """The first template argument (log2 N of every frame kernel), or None."""
    s = symbol.split("(")[0]
    return s.split("<", 1)[1].split(",")[0].split(">")[0].strip() if "<" in s else None


def template_args(symbol):
    s = symbol.split("(")[0]
    return [a.strip() for a in s.split("<", 1)[1].rsplit(">", 1)[0].split(",")] if "<" in s else []


def size_key(symbol, logn):
    """The summary key: the base name for instantiations at the workload's log2 N (what bench.py
    looks up), else base<first template argument> (other sizes: k_rows_half<14>). k_gen4_step2 runs
    three launches per frame, two over 16-B field texels (second argument true: gab, gde) and one
    over gc's 8-B texels as column pairs (false), so its key carries both arguments."""
    first = first_arg(symbol)
    if base_name(symbol) == "k_rows_hp":  # 4096 only; its template arguments are the field layout
        return "k_rows_hp" if logn == 12 else "k_rows_hp<12>"
    if base_name(symbol) == "k_gen4_step2":
        args = template_args(symbol)
        return f"k_gen4_step2<{args[0]},{args[1]}>"
    return base_name(symbol) if first in (None, str(logn)) else f"{base_name(symbol)}<{first}>"


def algorithmic_bytes(key, n, cascades, mode):
    """Algorithmic HBM bytes of ONE launch of `key` at the profiled workload (DESIGN.md §4 figures,
    the same as ocean_generator_frame_bytes), or None where no figure is defined: printed "-", never
    guessed. Keyed by the size-qualified name, so another size's instantiation (k_rows_half<14> in a
    4096 profile) never borrows this workload's bytes."""
    pts = n * n * cascades
    logn = n.bit_length() - 1
    if mode == "ifft":  # standalone EncodeIFFT: work-image chunks of 8 images, 32 B per texel per pass;
        # the bench's 8192 leg (2 images per call, one launch per pass: the pre-stage column pass and its row pass)
        # the 16384 leg (2 images per call): rows in place over both images in one launch, then per
        # image and 2048-column work slab one step-1 launch (image -> slab) and one step-2 launch (slab
        # -> image), each reading and writing its 16384 x 2048 texels once (launch_ifft_fourstep)
        return {"k_cols_to_blocks": 32 * 8 * n * n, "k_rows_final": 32 * 8 * n * n,
                "k_cols_pre<13>": 32 * 2 * 8192 ** 2, "k_rows_final<13>": 32 * 2 * 8192 ** 2,
                "k_rows_ifft<14>": 32 * 2 * 16384 ** 2, "k_cols4_step1<14>": 32 * 16384 * 2048,
                "k_cols4_step2<10>": 32 * 16384 * 2048}.get(key)
    if logn in (13, 14):  # four-step whole grid: kept columns [0, N/2) + the Nyquist column
        kept = (n // 2 + 1) / n
        # step 2 (the N/16-point step) reads step 1's parts and writes the row pass's fields, one launch
        # per field: gab and gde 16 + 16 per kept texel each, gc 8 + 8 (40 + 40 in all)
        table = {"k_gen4_step1": (16 + 40) * kept, f"k_gen4_step2<{logn - 4},true>": 32 * kept,
                 f"k_gen4_step2<{logn - 4},false>": 16 * kept,
                 "k_rows_xs": 40 * kept + 36, "k_rows_half": 40 * kept + 36}
    else:
        kept = (n // 2 + 4) / n  # columns [0, N/2) plus the 4-wide Nyquist strip
        table = {"k_cols_evolve": 48, "k_rows_final": 68, "k_cols_half": (16 + 40) * kept,
                 "k_rows_half": 40 * kept + 36, "k_rows_hp": 40 * kept + 36}
    if key in ("k_generate_spectrum", "k_generate_spectrum_pairs"):
        return 16 * n * n  # one cascade's h0 per launch
    return int(table[key] * pts) if key in table else None


def main(argv):
    src, tag = argv[1], argv[2]
    n = int(argv[3]) if len(argv) > 3 else 4096
    cascades = int(argv[4]) if len(argv) > 4 else 8
    prefix = argv[5] if len(argv) > 5 else "prof"  # tools/profile_gpu.sh PREFIX
    mode = argv[6] if len(argv) > 6 else "frame"  # frame | ifft (EncodeIFFT chunks of 8 images)
    logn = n.bit_length() - 1

    def read_csv(path):
        with open(path) as f:
            return list(csv.DictReader(f))

    def find(sub, suffix):
        d = os.path.join(src, sub)
        for fn in os.listdir(d):
            if fn.endswith(suffix):
                return os.path.join(d, fn)
        raise FileNotFoundError(f"{d}/*{suffix}")

    # per dispatch: (size key, grid threads, workgroup threads) -> durations. A persistent grid has the
    # same geometry for every cascade count, so tools/profile_gpu.sh profiles bench.py --headline-only
    # (no one-cascade or re-seed legs): each key then holds the workload's launches only.
    durs = {}
    for r in read_csv(find(prefix + "_trace", "kernel_trace.csv")):
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        wg = int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]) * int(r["Workgroup_Size_Z"])
        k = (size_key(r["Kernel_Name"], logn), grid, wg)
        durs.setdefault(k, {"ns": [], "symbols": set()})
        durs[k]["ns"].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        durs[k]["symbols"].add(r["Kernel_Name"])
    counters = {}
    for sub, name in ((prefix + "_fetch", "FETCH_SIZE"), (prefix + "_write", "WRITE_SIZE")):
        for r in read_csv(find(sub, "counter_collection.csv")):
            if r["Counter_Name"] == name:
                k = (size_key(r["Kernel_Name"], logn), int(r["Grid_Size"]), int(r["Workgroup_Size"]))
                counters.setdefault(k, {}).setdefault(name, []).append(float(r["Counter_Value"]))

    out = {"tag": tag, "n": n, "cascades": cascades, "device_source_sha256": device_source_sha256(), "kernels": {},
           "by_geometry": []}
    lines = [f"# rocprofv3 summary — {tag}", "",
             f"Workload: bench.py --headline-only, {cascades} cascades of {n}x{n} per launch. Durations: "
             "`--kernel-trace --stats` (per dispatch, keyed by kernel, grid and workgroup size). Traffic: separate "
             "`--pmc FETCH_SIZE` and `--pmc WRITE_SIZE` passes; read = 2 x FETCH_SIZE (gfx950 half-count "
             "correction), write = WRITE_SIZE; KB = 1024 B. Algorithmic bytes: DESIGN.md §4 per-point figures "
             "x the points of one launch; \"-\" where no figure is defined.", "",
             "| kernel | grid x wg | calls | avg ms | algorithmic GB/launch | measured HBM GB/launch (read + write) "
             "| traffic / algorithmic | achieved GB/s (algorithmic) |",
             "|---|---|---|---|---|---|---|---|"]
    fmt = lambda v: "-" if v is None else f"{v / 1e9:.3f}"
    for k in sorted(durs):
        name, grid, wg = k
        ns = durs[k]["ns"]
        avg_ms = statistics.mean(ns) / 1e6
        fe, wr_ = counters.get(k, {}).get("FETCH_SIZE", []), counters.get(k, {}).get("WRITE_SIZE", [])
        rd = statistics.median(fe) * 1024 * 2 if fe else None
        wr = statistics.median(wr_) * 1024 if wr_ else None
        traffic = (rd + wr) if (rd is not None and wr is not None) else None
        algo = algorithmic_bytes(name, n, cascades, mode)
        achieved = algo / (avg_ms * 1e-3) / 1e9 if algo else None
        if achieved is not None and achieved > HBM_PEAK_GBS:
            raise SystemExit(f"{name} grid {grid}: {achieved:.0f} GB/s algorithmic exceeds the {HBM_PEAK_GBS:.0f} GB/s "
                             "HBM peak: the launch does not cover the workload the bytes assume (profile with "
                             "bench.py --headline-only)")
        rec = {"kernel": name, "grid_threads": grid, "workgroup_threads": wg, "calls": len(ns), "avg_ms": avg_ms,
               "algorithmic_bytes": algo, "hbm_read_bytes": rd, "hbm_write_bytes": wr, "hbm_traffic_bytes": traffic,
               "achieved_GBps_algorithmic": achieved, "symbols": sorted(durs[k]["symbols"])}
        out["by_geometry"].append(rec)
        # bench.py's lookup: the workload's kernel by name (its most-called geometry)
        if name not in out["kernels"] or out["kernels"][name]["calls"] < len(ns):
            out["kernels"][name] = rec
        ratio = f"{traffic / algo:.3f}" if (traffic and algo) else "-"
        ach = "-" if achieved is None else f"{achieved:.0f}"
        lines.append(f"| {name} | {grid // wg} x {wg} | {len(ns)} | {avg_ms:.3f} | {fmt(algo)} | {fmt(rd)} + {fmt(wr)} "
                     f"| {ratio} | {ach} |")
    lines += ["", f"Device source sha256: `{out['device_source_sha256']}` (bench.py uses this summary's traffic only for "
              "the same device code)."]
    os.makedirs("profiles", exist_ok=True)
    with open(f"profiles/{tag}_rocprof.json", "w") as fh:
        json.dump(out, fh, indent=1)
    with open(f"profiles/{tag}_rocprof.md", "w") as fh:
        fh.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv)
