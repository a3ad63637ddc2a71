#!/bin/bash
# PMC write/read bytes of the 8192^2 EncodeIFFT column-pass variants in tools/microbench/ifft4bench
# (one rocprofv3 pass per counter, never combined with tracing), then a kernel trace for durations.
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
for c in WRITE_SIZE FETCH_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --kernel-include-regex "k_cols" -d gpurun_out/ifft4_$c -o p \
    --output-format csv -- tools/microbench/ifft4bench > gpurun_out/ifft4_$c.log 2>&1 || { echo "pass $c failed"; exit 1; }
  echo "pass $c ok"
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/ifft4_trace -o t --output-format csv \
  -- tools/microbench/ifft4bench > gpurun_out/ifft4_trace.log 2>&1 || { echo "trace failed"; exit 1; }
echo "trace ok"
