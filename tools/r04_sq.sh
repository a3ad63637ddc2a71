#!/bin/bash
# Round 4: SQ issue/wait/LDS counters for the 4096 frame passes (headline) and the 16384 passes.
set -u
PREFIX=r04_sq_4k tools/pmc_sq.sh || exit 1
PREFIX=r04_sq_16k KERNEL_REGEX="k_rows_xs|k_gen4" \
  BENCH_ARGS="--n 16384 --cascades 1 --steps 5 --warmup 2 --headline-only --no-profile" tools/pmc_sq.sh || exit 1
echo "sq done"
