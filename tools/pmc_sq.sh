#!/bin/bash
# SQ counter passes (issue/wait breakdown, LDS) over the bench's frame workload, one rocprofv3 run per
# counter set (counters never combined with tracing domains); each pass has its own time limit.
#   KERNEL_REGEX  kernels to count (default: the frame passes)
#   BENCH_ARGS    bench.py arguments
#   PREFIX        output prefix (default pmc_sq)
#   CMD           program + arguments to profile instead of bench.py (e.g. a microbench binary)
# Output: gpurun_out/<prefix>_<k>/ (csv); summarise with tools/sq_summary.py.
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
ARGS=${BENCH_ARGS:-"--steps 5 --warmup 2 --no-cpu-baseline --no-slab --no-ifft --no-surface --no-reseed --no-profile"}
KRE=${KERNEL_REGEX:-"k_rows_half|k_rows_hp|k_cols_half"}
P=${PREFIX:-pmc_sq}
SETS=(
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
  "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_INSTS_SALU"
  "SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE GRBM_COUNT"
)
mkdir -p gpurun_out
k=0
for s in "${SETS[@]}"; do
  timeout -s KILL 150 rocprofv3 --pmc $s --kernel-include-regex "$KRE" -d gpurun_out/${P}_$k -o sq \
    --output-format csv -- ${CMD:-python3 bench.py $ARGS} > gpurun_out/${P}_$k.log 2>&1 || { echo "pass $k failed rc=$?"; tail -5 gpurun_out/${P}_$k.log; exit 1; }
  echo "pass $k ok"
  k=$((k + 1))
done
