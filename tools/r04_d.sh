#!/bin/bash
# Round 4, session D: the 8-rank projection with XCD-balanced CU masks (which logical CU numbering?).
set -u
export PYTHONUNBUFFERED=1
tools/gpu_step.sh r04d_slab 600 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-ifft --no-surface --no-reseed \
  --slab-reserve-cus 32 --slab-mask-layouts xcd,stride || exit 1
echo "r04d done"
