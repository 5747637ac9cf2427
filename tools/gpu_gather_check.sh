#!/bin/bash
# Coalesced gather: parity (multi-batch launches) + driver-shaped bench, then
# the end-to-end host-path timing.
set -o pipefail
out=gpurun_out/gather
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_batch_equation.py tests/test_gpu_host_pipeline.py > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for rep in 1 2; do
  timeout -k 10 150 python -u bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline > $out/s20_$rep.log 2>&1 || { tail -5 $out/s20_$rep.log; exit 1; }
  grep '^{' $out/s20_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('s20', d['value']/1e6, d['ms_per_step']*20)"
done
./tools/gpu_e2e_timing.sh > $out/e2e.txt 2>&1 || { tail -20 $out/e2e.txt; exit 1; }
tail -45 $out/e2e.txt
