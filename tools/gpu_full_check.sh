#!/bin/bash
# Whole GPU suite, then the driver-shaped bench (x2) and the steady state.
set -o pipefail
out=gpurun_out/full
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $out/tests.log 2>&1 \
  || { tail -40 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for args in "--steps 20" "--steps 20" "--steps 1536"; do
  timeout -k 10 200 python -u bench.py $args --warmup 5 --no-extras --no-cpu-baseline > $out/b.log 2>&1 || { tail -5 $out/b.log; exit 1; }
  grep '^{' $out/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$args', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step']*d['steps'],3), 'ms', d['config']['launch_sizes'][:4])"
done
