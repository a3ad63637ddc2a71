#!/bin/bash
# Round 4, session F: pass-1 round 2 on float2 and the cross-item h0 prefetch (halfbench r2f), 8 and 1 cascades.
set -u
tools/gpu_step.sh r04f_halfbench_r2f_8 200 tools/microbench/halfbench 12 8 r2f || exit 1
tools/gpu_step.sh r04f_halfbench_r2f_1 200 tools/microbench/halfbench 12 1 r2f || exit 1
echo "r04f done"
