#!/bin/bash
# Round-5 closing measurement. Part A: smoke, the GPU suite, the default bench line, the 4-rank
# --shared-gpu rehearsal (one-sided exchange across processes, self-verifying legs). Part B: rocprofv3
# collections (trace + separate FETCH_SIZE / WRITE_SIZE passes) of the headline, the 16384^2 whole grid
# and the EncodeIFFT legs, and the parity report. TAG (default r05f) prefixes every output.
set -u
T=${TAG:-r05f}
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
if [ "${PART:-A}" = A ]; then
  tools/gpu_step.sh ${T}_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
  tools/gpu_step.sh ${T}_suite 700 python -u -m pytest tests/ -m gpu -v --timeout 300 --timeout-method thread || exit 1
  tools/gpu_step.sh ${T}_bench 500 python -u bench.py || exit 1
  echo "r05 part A done"
else
  PREFIX=${T} tools/profile_gpu.sh || exit 1
  PREFIX=${T}_16k BENCH_ARGS="--n 16384 --cascades 1 --steps 10 --warmup 2 --headline-only" tools/profile_gpu.sh || exit 1
  PREFIX=${T}_ifft BENCH_ARGS="--steps 3 --warmup 1 --no-slab --no-surface --no-reseed --no-cpu-baseline" \
    KERNEL_REGEX="k_cols_to_blocks|k_cols_pre|k_rows_final|k_cols|k_rows_ifft|k_cols4" tools/profile_gpu.sh || exit 1
  tools/gpu_step.sh ${T}_parity 400 python -u tools/parity_report.py || exit 1
  echo "r05 part B done"
fi
