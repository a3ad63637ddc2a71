#!/bin/bash
# The closing measurement of a build, parameterised (replaces the per-round r0N_*.sh drivers).
#   PART=A: smoke, the GPU suite, the default bench line.
#   PART=B: rocprofv3 collections (trace + separate FETCH_SIZE / WRITE_SIZE passes) of the headline, the
#           16384^2 whole grid and the EncodeIFFT legs, and the parity report.
#   PART=C: rocprofv3 trace of BASELINE configs 1-3 (tools/bench_configs.py under the profiler).
# TAG prefixes every output under gpurun_out/ (copy what is judged into profiles/). Every GPU step runs
# under its own time limit (tools/gpu_step.sh, tools/profile_gpu.sh) and the first failure ends the call.
set -u
T=${TAG:?set TAG, e.g. TAG=r06a}
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
case "${PART:-A}" in
A)
  tools/gpu_step.sh ${T}_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
  tools/gpu_step.sh ${T}_suite 700 python -u -m pytest tests/ -m gpu -v --timeout 300 --timeout-method thread || exit 1
  tools/gpu_step.sh ${T}_bench 600 python -u bench.py || exit 1
  ;;
B)
  PREFIX=${T} tools/profile_gpu.sh || exit 1
  PREFIX=${T}_16k BENCH_ARGS="--n 16384 --cascades 1 --steps 10 --warmup 2 --headline-only" tools/profile_gpu.sh || exit 1
  PREFIX=${T}_ifft BENCH_ARGS="--steps 3 --warmup 1 --no-slab --no-surface --no-reseed --no-cpu-baseline --no-configs" \
    KERNEL_REGEX="k_cols_to_blocks|k_cols_pre|k_rows_final|k_cols|k_rows_ifft|k_cols4" tools/profile_gpu.sh || exit 1
  tools/gpu_step.sh ${T}_parity 400 python -u tools/parity_report.py || exit 1
  ;;
C)
  cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_configs_trace -o trace --output-format csv \
    -- python3 tools/bench_configs.py ${T} --steps 50 > gpurun_out/${T}_configs_trace.log 2>&1 || exit 1
  ;;
esac
echo "closing ${T} part ${PART:-A} done"
