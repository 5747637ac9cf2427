#!/bin/bash
# Mixed-batch GPU tests, then C5 (1M mixed, device-resident) with the two
# kinds' pipelines on two streams vs one (TMV_MIXED_TWO).
set -o pipefail
out=gpurun_out/c5
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_batch_equation.py \
  tests/test_gpu_sr25519.py tests/test_gpu_configs.py > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for rep in 1 2; do
  for v in 0 1; do
    echo -n "TMV_MIXED_TWO=$v: "
    TMV_MIXED_TWO=$v timeout -k 10 300 python -u tools/bench_configs.py --only 5 --c5-methods "batch m=64,per-entry" > $out/c5_$v.log 2>&1 || { tail -20 $out/c5_$v.log; exit 1; }
    grep '^{' $out/c5_$v.log | python -c "import json,sys; [print(json.loads(l)['config'][-12:], json.loads(l)['ms'], json.loads(l)['verifies_per_s'], json.loads(l)['same_vector']) for l in sys.stdin]" | tr '\n' ' '; echo
  done
done
