#!/usr/bin/env python3
"""BASELINE.json configs 1-3 on one GPU with the CPU oracle beside them: bench.py's `configs` leg run on
its own (so rocprofv3 can trace exactly these launches, tools/closing.sh PART=C). Writes
gpurun_out/<tag>_configs.{json,md}.

Usage: python tools/bench_configs.py [tag] [--steps K]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag", nargs="?", default="r06")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--cpu-seconds", type=float, default=2.0)
    args = ap.parse_args()
    res = bench.configs_leg(steps=args.steps, cpu_seconds=args.cpu_seconds)
    lines = [f"# BASELINE configs 1-3 on one MI355X — {args.tag}", "",
             "GPU: wall ms per step over the timed steps (host launch included); kernel ms from HIP events "
             "around every launch; frac = algorithmic bytes / kernel time / 8 TB/s. CPU: the oracle (fp32 "
             f"restatement of the reference), {res['cpu_threads']} OpenMP threads.", "",
             "| config | GPU points/s | wall ms | kernel ms | column / row ms | B/pt | frac (kernel) | frac (overlapped wall) "
             "| CPU points/s | GPU/CPU |", "|---|---|---|---|---|---|---|---|---|---|"]
    for k, v in res.items():
        if not isinstance(v, dict) or "gpu" not in v:
            continue
        g, c = v["gpu"], v["cpu"]
        split = f"{g['column_pass_ms']:.4f} / {g['row_pass_ms']:.4f}" if "column_pass_ms" in g else "-"
        ov = f"{g['frame_overlap']['frac_hbm_peak_wall']:.3f}" if "frame_overlap" in g else "-"
        bpp = g.get("frame_hbm_bytes_per_point", g.get("bytes_per_texel"))
        lines.append(f"| {k} | {g['points_per_s']:.3e} | {g['wall_ms_per_step']:.4f} | {g['kernel_ms_per_step']:.4f} | "
                     f"{split} | {bpp:.0f} | {g['frac_hbm_peak']:.3f} | {ov} | {c['points_per_s']:.3e} | "
                     f"{v['gpu_over_cpu']:.0f}x |")
    out_dir = os.path.join(ROOT, "gpurun_out")
    os.makedirs(out_dir, exist_ok=True)
    with open(os.path.join(out_dir, f"{args.tag}_configs.json"), "w") as f:
        json.dump(res, f, indent=1)
    with open(os.path.join(out_dir, f"{args.tag}_configs.md"), "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines), flush=True)


if __name__ == "__main__":
    main()
