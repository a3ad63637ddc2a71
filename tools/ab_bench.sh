#!/bin/bash
# Same-box A/B of two library builds through bench.py: ab_old/ (a copy of the package + bench.py from
# an earlier commit) against the tree's own, alternating, each run under its own time limit.
#   AB_ARGS  bench.py arguments (default: the headline and the one-cascade leg only)
set -u
ARGS=${AB_ARGS:-"--steps 50 --warmup 5 --no-slab --no-ifft --no-surface --no-reseed --no-cpu-baseline"}
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in old new; do
    if [ $v = old ]; then d=ab_old; else d=.; fi
    (cd $d && timeout -k 10 300 python bench.py $ARGS) > gpurun_out/ab_${v}_$r.log 2>&1 || { echo "$v run $r failed"; exit 1; }
    python3 - "$v" "$r" gpurun_out/ab_${v}_$r.log <<'PY'
import json, sys
line = [l for l in open(sys.argv[3]) if l.startswith("{")][-1]
d = json.loads(line)
k = d["kernels"]
extra = ""
il = d.get("ifft_only_large") or {}
for n_, v_ in sorted(il.items()):
    extra += f"  ifft {n_} {v_['ms_per_call']:.3f} ms"
if "slab" in d:
    extra += f"  16384 frame {d['slab']['ms_per_frame']:.3f} ms"
print(f"{sys.argv[1]} run {sys.argv[2]}: frame {d['ms_per_step']:.4f} ms  cols {k['column_pass_k_cols_half']['avg_ms']:.4f}  "
      f"rows {k['row_pass_k_rows_hp']['avg_ms']:.4f}  one cascade {d['strong_scaling']['one_cascade_ms']:.4f} ms{extra}", flush=True)
PY
  done
done
