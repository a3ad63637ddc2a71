#!/bin/bash
# Round-3 final measurement, part A: smoke, the GPU suite, the default bench line.
set -u
mkdir -p gpurun_out
tools/gpu_step.sh f_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
tools/gpu_step.sh f_suite 600 python -u -m pytest tests/ -m gpu -v --timeout 300 --timeout-method thread || exit 1
tools/gpu_step.sh f_bench 600 python -u bench.py || exit 1
echo "part A done"
