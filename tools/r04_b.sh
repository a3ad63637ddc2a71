#!/bin/bash
# Round 4, second GPU session: production validation of the k_rows_hp build (smoke, GPU suite, bench,
# rocprof traffic), then the one-cascade column-pass A/B (halfbench 12 1: half-strip items at two
# workgroups per CU against production).
set -u
TAG=r04b tools/r04_final.sh || exit 1
tools/gpu_step.sh r04b_halfbench_c1 200 tools/microbench/halfbench 12 1 quick || exit 1
echo "r04b done"
