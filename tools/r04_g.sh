#!/bin/bash
# Round 4, session G: the 16384 row pass with a streaming T_in (rm16bench).
set -u
tools/gpu_step.sh r04g_rm16bench 200 tools/microbench/rm16bench || exit 1
echo "r04g done"
