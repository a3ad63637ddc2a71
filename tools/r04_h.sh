#!/bin/bash
# Round 4, session H: pass 1 with the LDS-staged h0 prefetch (halfbench lpf, 8 and 1 cascades), and the
# 16384 row pass with a streaming T_in (rm16bench).
set -u
tools/gpu_step.sh r04h_halfbench_lpf_8 200 tools/microbench/halfbench 12 8 lpf || exit 1
tools/gpu_step.sh r04h_halfbench_lpf_1 200 tools/microbench/halfbench 12 1 lpf || exit 1
tools/gpu_step.sh r04h_rm16bench 200 tools/microbench/rm16bench || exit 1
echo "r04h done"
