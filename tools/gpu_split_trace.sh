#!/bin/bash
# Kernel trace of the driver-shaped bench with the split launch (one launch of 20).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
mkdir -p gpurun_out/split_trace
TMV_SPLIT_MIN=40000 timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/split_trace -o run --output-format csv -- \
  python -u bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline --plan 20 > gpurun_out/split_trace/bench.log 2>&1 \
  || { tail -20 gpurun_out/split_trace/bench.log; exit 1; }
find gpurun_out/split_trace -name "*kernel_trace.csv" | head
