#!/bin/bash
# Round 4, first GPU session: the new path-switch test + the native RCCL tests, the standalone RCCL
# large send/recv check (ROCm's and torch's librccl), the slab leg with the honest 8-rank projection,
# then the SQ counters of the 4096 and 16384 frame passes.
set -u
export PYTHONUNBUFFERED=1
tools/gpu_step.sh r04a_rm16bench 150 tools/microbench/rm16bench || exit 1
tools/gpu_step.sh r04a_halfbench_hp 150 tools/microbench/halfbench 12 8 hp || exit 1
tools/gpu_step.sh r04a_ifft4bench_mall 150 tools/microbench/ifft4bench mall || exit 1
tools/gpu_step.sh r04a_tests 300 python -u -m pytest tests/test_gpu_configs.py -x -v --timeout 240 --timeout-method thread \
  -k "path_switch or native_rccl" || exit 1
tools/gpu_step.sh r04a_rccl_rocm 200 tools/rccl_repro/rccl_big_sendrecv_rocm; rc1=$?
[ $rc1 -le 1 ] || exit 1
tools/gpu_step.sh r04a_rccl_torch 200 tools/rccl_repro/rccl_big_sendrecv_torch; rc2=$?
[ $rc2 -le 1 ] || exit 1
tools/gpu_step.sh r04a_slab 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-ifft --no-surface --no-reseed || exit 1
tools/r04_sq.sh || exit 1
echo "r04a done"
