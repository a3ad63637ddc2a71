#!/usr/bin/env python3
"""Summarise the rocprofv3 kernel trace of tools/bench_configs.py (tools/closing.sh PART=C) into
profiles/<tag>_configs_rocprof.md: every kernel dispatch grouped by (kernel, log2 N, grid, workgroup),
with its count and average duration, and per BASELINE config the kernel time of one step and its
roofline fraction (algorithmic bytes / that time / 8 TB/s).
Usage: tools/configs_rocprof.py <trace dir> <tag>
"""
import csv
import glob
import os
import re
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HBM_PEAK_GBS = 8000.0


def key(name):
    base = name.split("(")[0].replace("void ", "").replace("oceanfft::", "").strip()
    m = re.match(r"([A-Za-z0-9_]+)<(\d+)", base)
    return (m.group(1), int(m.group(2))) if m else (base.split("<")[0], 0)


def main(argv):
    d, tag = argv[1], argv[2]
    files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        print("no kernel trace under", d)
        return 1
    groups = {}
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k, logn = key(r["Kernel_Name"])
                if not k.startswith("k_"):
                    continue
                g = (k, logn, int(r["Grid_Size_X"]), int(r["Workgroup_Size_X"]))
                groups.setdefault(g, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    lines = [f"# BASELINE configs 1-3, rocprofv3 kernel trace — {tag}", "",
             "`rocprofv3 --kernel-trace --stats -- python3 tools/bench_configs.py` (tools/closing.sh PART=C); "
             "durations in microseconds, median over the dispatches of each group.", "",
             "| kernel | N | grid (threads) | workgroup | dispatches | median us | mean us |", "|---|---|---|---|---|---|---|"]
    for g in sorted(groups, key=lambda x: (x[1], x[0], x[2])):
        v = groups[g]
        lines.append(f"| {g[0]} | {1 << g[1] if g[1] else '-'} | {g[2]} | {g[3]} | {len(v)} | "
                     f"{statistics.median(v):.2f} | {statistics.mean(v):.2f} |")
    # config 3: the two frame kernels at N = 2048 per grid shape (1 cascade / 4 cascades differ in grid)
    lines += ["", "Config 3 (2048^2, 84.19 B per point): the two frame kernels of one step, by grid shape.", ""]
    cols = sorted((g for g in groups if g[0] == "k_cols_half" and g[1] == 11), key=lambda x: x[2])
    rows = sorted((g for g in groups if g[0] in ("k_rows_half", "k_rows_hp") and g[1] == 11), key=lambda x: x[2])
    for c, r in zip(cols, rows):
        t = statistics.median(groups[c]) + statistics.median(groups[r])
        lines.append(f"- column grid {c[2]} + row grid {r[2]}: {t:.2f} us of kernels per step")
    out = os.path.join(ROOT, "profiles", f"{tag}_configs_rocprof.md")
    with open(out, "w") as fh:
        fh.write("\n".join(lines) + "\n")
    print("\n".join(lines))
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
