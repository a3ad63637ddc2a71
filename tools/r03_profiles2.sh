#!/bin/bash
# rocprofv3 collections of the 16384^2 whole grid (four-step path) and the EncodeIFFT legs.
set -u
PREFIX=r03_16k BENCH_ARGS="--n 16384 --cascades 1 --steps 10 --warmup 2 --headline-only" tools/profile_gpu.sh || exit 1
PREFIX=r03_ifft BENCH_ARGS="--steps 3 --warmup 1 --no-slab --no-surface --no-reseed --no-cpu-baseline" \
  KERNEL_REGEX="k_cols_to_blocks|k_rows_final|k_cols|k_rows_ifft|k_cols4" tools/profile_gpu.sh || exit 1
echo "profiles done"
