#!/bin/bash
# SQ counters of tools/microbench/sqcontrol (the streaming controls), the three counter sets of
# tools/pmc_sq.sh, one rocprofv3 run per set; summarise with tools/sq_summary.py <dir> <prefix> <tag>.
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
P=${PREFIX:-sqctl}
SETS=(
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
  "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_INSTS_SALU"
  "SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE GRBM_COUNT"
)
mkdir -p gpurun_out
timeout -k 10 60 ./tools/microbench/sqcontrol > gpurun_out/${P}_time.log 2>&1 || { echo "timing failed"; exit 1; }
k=0
for s in "${SETS[@]}"; do
  timeout -s KILL 90 rocprofv3 --pmc $s --kernel-include-regex "k_stream" -d gpurun_out/${P}_$k -o sq \
    --output-format csv -- ./tools/microbench/sqcontrol > gpurun_out/${P}_$k.log 2>&1 || { echo "pass $k failed rc=$?"; exit 1; }
  echo "pass $k ok"
  k=$((k + 1))
done
