#!/usr/bin/env python3
"""Summarise tools/pmc_sq.sh output (SQ issue / wait / LDS counters, three rocprofv3 --pmc passes) into
profiles/<tag>_sq.{md,json}: per kernel (keyed as tools/parse_rocprof.py keys them), the median per
dispatch of every counter and the shares of a wave's life.

MI355X_MICROARCH.md, rocprofv3 PMC slots: SQ_WAIT_ANY (wave parked on s_waitcnt / barrier),
SQ_WAIT_INST_ANY (issue stall) and SQ_ACTIVE_INST_ANY (issuing) are disjoint and add up to
SQ_WAVE_CYCLES; SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles.
SQ_LDS_BANK_CONFLICT counts the extra LDS cycles of conflicts, SQ_LDS_IDX_ACTIVE all LDS-array cycles.
Usage: tools/sq_summary.py <gpurun_out dir> <prefix> <tag> [logN]
"""
import csv
import glob
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from parse_rocprof import size_key  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(argv):
    src, prefix, tag = argv[1], argv[2], argv[3]
    logn = int(argv[4]) if len(argv) > 4 else 12
    vals = {}
    for path in sorted(glob.glob(os.path.join(src, f"{prefix}_*", "**", "*counter_collection.csv"), recursive=True)):
        with open(path) as f:
            for r in csv.DictReader(f):
                k = (size_key(r["Kernel_Name"], logn), int(r["Grid_Size"]), int(r["Workgroup_Size"]))
                vals.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    out = {"tag": tag, "kernels": []}
    lines = [f"# SQ counters — {tag}", "",
             "rocprofv3 `--pmc` in three passes (tools/pmc_sq.sh), medians per dispatch. Shares of SQ_WAVE_CYCLES "
             "(quad-cycles summed over waves): `active` = SQ_ACTIVE_INST_ANY (issuing), `wait` = SQ_WAIT_ANY (parked on "
             "s_waitcnt or a barrier), `stall` = SQ_WAIT_INST_ANY (ready but not issued); `valu`, `lds`, `vmem` = "
             "SQ_ACTIVE_INST_VALU / _LDS / _VMEM; `lds stall` = SQ_WAIT_INST_LDS. Per wave: instructions issued. "
             "`conflict` = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE.", "",
             "| kernel | grid x wg | waves | active | wait | stall | valu | lds | vmem | lds stall | VALU/wave | LDS/wave "
             "| VMEM rd/wave | VMEM wr/wave | SALU/wave | conflict |",
             "|---|---|---|---|---|---|---|---|---|---|---|---|---|---|---|---|"]
    for k in sorted(vals):
        c = {n: statistics.median(v) for n, v in vals[k].items()}
        wc = c.get("SQ_WAVE_CYCLES")
        waves = c.get("SQ_WAVES")
        if not wc or not waves:
            continue
        share = lambda n: c[n] / wc if n in c else None  # noqa: E731
        per = lambda n: c[n] / waves if n in c else None  # noqa: E731
        rec = {"kernel": k[0], "grid": k[1], "wg": k[2], "counters": c,
               "share": {n: share(n) for n in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                                               "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM",
                                               "SQ_WAIT_INST_LDS")},
               "per_wave": {n: per(n) for n in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD",
                                                "SQ_INSTS_VMEM_WR", "SQ_INSTS_SALU")},
               "lds_conflict": (c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"])
               if c.get("SQ_LDS_IDX_ACTIVE") else None}
        out["kernels"].append(rec)
        f = lambda x, d=2: "-" if x is None else f"{x:.{d}f}"  # noqa: E731
        s, p = rec["share"], rec["per_wave"]
        lines.append(f"| {k[0]} | {k[1] // k[2]} x {k[2]} | {waves:.0f} | {f(s['SQ_ACTIVE_INST_ANY'])} | "
                     f"{f(s['SQ_WAIT_ANY'])} | {f(s['SQ_WAIT_INST_ANY'])} | {f(s['SQ_ACTIVE_INST_VALU'])} | "
                     f"{f(s['SQ_ACTIVE_INST_LDS'])} | {f(s['SQ_ACTIVE_INST_VMEM'])} | {f(s['SQ_WAIT_INST_LDS'])} | "
                     f"{f(p['SQ_INSTS_VALU'], 0)} | {f(p['SQ_INSTS_LDS'], 0)} | {f(p['SQ_INSTS_VMEM_RD'], 0)} | "
                     f"{f(p['SQ_INSTS_VMEM_WR'], 0)} | {f(p['SQ_INSTS_SALU'], 0)} | {f(rec['lds_conflict'], 3)} |")
    with open(os.path.join(ROOT, "profiles", f"{tag}_sq.md"), "w") as fh:
        fh.write("\n".join(lines) + "\n")
    with open(os.path.join(ROOT, "profiles", f"{tag}_sq.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv)
