#!/bin/bash
# Round 4, session C: k_rows_hp with the conflict-free LDS layout against k_rows_half (halfbench hp),
# its SQ counters, and the slab leg with both 8-rank projections (unmasked, CU-masked streams).
set -u
export PYTHONUNBUFFERED=1
tools/gpu_step.sh r04c_halfbench_hp 150 tools/microbench/halfbench 12 8 hp || exit 1
tools/gpu_step.sh r04c_slab 500 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-ifft --no-surface --no-reseed || exit 1
PREFIX=r04c_sq_4k KERNEL_REGEX="k_rows_hp|k_cols_half" tools/pmc_sq.sh || exit 1
echo "r04c done"
