#!/bin/bash
# Round 4, session I: k_rows_hp with a streaming T_in (halfbench hp).
set -u
tools/gpu_step.sh r04i_halfbench_hp 200 tools/microbench/halfbench 12 8 hp || exit 1
echo "r04i done"
