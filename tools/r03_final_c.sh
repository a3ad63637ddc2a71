#!/bin/bash
# Round-3 closing profiles of the last session's build (8192 pre-stage and 4096 one-row EncodeIFFT, frame
# overlap changed the device-code sha): rocprofv3 trace + separate FETCH_SIZE / WRITE_SIZE passes of the
# headline, the 16384^2 whole grid and the EncodeIFFT legs.
set -u
PREFIX=r03h tools/profile_gpu.sh || exit 1
PREFIX=r03h_16k BENCH_ARGS="--n 16384 --cascades 1 --steps 10 --warmup 2 --headline-only" tools/profile_gpu.sh || exit 1
PREFIX=r03h_ifft BENCH_ARGS="--steps 3 --warmup 1 --no-slab --no-surface --no-reseed --no-cpu-baseline" \
  KERNEL_REGEX="k_cols_to_blocks|k_cols_pre|k_rows_final|k_cols|k_rows_ifft|k_cols4" tools/profile_gpu.sh || exit 1
echo "part C done"
