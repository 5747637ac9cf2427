#!/bin/bash
# Kernel trace of the steady-state bench with the located fallback forced.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
mkdir -p gpurun_out/locate_trace
TMV_LOCATE_MIN=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/locate_trace -o run -- \
  python -u bench.py --steps 256 --warmup 32 --no-extras --no-cpu-baseline > gpurun_out/locate_trace/bench.log 2>&1 \
  || { tail -20 gpurun_out/locate_trace/bench.log; exit 1; }
ls gpurun_out/locate_trace
