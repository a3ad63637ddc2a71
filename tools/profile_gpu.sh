#!/bin/bash
# rocprofv3 collection for the bench workload (run on the GPU box from the repo root):
#   1. kernel trace + stats (durations)          -> gpurun_out/${PREFIX:-prof}_trace
#   2. PMC FETCH_SIZE only (own pass)            -> gpurun_out/prof_fetch
#   3. PMC WRITE_SIZE only (own pass)            -> gpurun_out/prof_write
# Counters are never combined with tracing domains (pool rule), and each step has its own limit.
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
ARGS=${BENCH_ARGS:-"--steps 20 --warmup 3 --headline-only"}
KRE=${KERNEL_REGEX:-"k_cols_evolve|k_rows_final|k_rows_ifft|k_rows_half|k_rows_hp|k_rows_xs|k_cols|k_gen4|k_generate_spectrum|k_half_nyquist"}
P=${PREFIX:-prof}  # output directories gpurun_out/${P}_trace, _fetch, _write
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${P}_trace -o trace --output-format csv \
  -- python3 bench.py $ARGS > gpurun_out/${P}_trace.log 2>&1 || { echo "trace pass failed rc=$?"; tail -20 gpurun_out/${P}_trace.log; exit 1; }
echo "trace pass ok"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRE" -d gpurun_out/${P}_fetch -o fetch \
  --output-format csv -- python3 bench.py $ARGS --no-profile > gpurun_out/${P}_fetch.log 2>&1 || { echo "fetch pass failed rc=$?"; tail -20 gpurun_out/${P}_fetch.log; exit 1; }
echo "fetch pass ok"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRE" -d gpurun_out/${P}_write -o write \
  --output-format csv -- python3 bench.py $ARGS --no-profile > gpurun_out/${P}_write.log 2>&1 || { echo "write pass failed rc=$?"; tail -20 gpurun_out/${P}_write.log; exit 1; }
echo "write pass ok"
find gpurun_out/${P}_trace gpurun_out/${P}_fetch gpurun_out/${P}_write -name "*.csv" | head -20
