#!/bin/bash
# Round-3 closing measurement on one GPU box: smoke, the default bench line, and the rocprofv3
# collections (trace + separate FETCH_SIZE / WRITE_SIZE passes) of the headline, the 16384^2 whole
# grid and the EncodeIFFT legs. Each step has its own time limit; the first failure ends the script.
set -u
mkdir -p gpurun_out
tools/gpu_step.sh smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
tools/gpu_step.sh bench 900 python -u bench.py || exit 1
PREFIX=r03 tools/profile_gpu.sh || exit 1
PREFIX=r03_16k BENCH_ARGS="--n 16384 --cascades 1 --steps 10 --warmup 2 --headline-only" tools/profile_gpu.sh || exit 1
PREFIX=r03_ifft BENCH_ARGS="--steps 3 --warmup 1 --no-slab --no-surface --no-reseed --no-cpu-baseline" \
  KERNEL_REGEX="k_cols_to_blocks|k_rows_final|k_cols|k_rows_ifft|k_cols4" tools/profile_gpu.sh || exit 1
echo "closing measurements done"
