#!/bin/bash
# GPU check of the sub-group bisection: batch-equation tests, the full GPU
# suite, then the C2 bench with and without k_msm_subcheck (under gpurun).
OUT=gpurun_out/subcheck
mkdir -p $OUT
run() {
  local name=$1; shift
  timeout -k 10 "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  [ $rc -ne 0 ] && { tail -30 $OUT/$name.log; exit $rc; }
  return 0
}
run beq 300 python -u -m pytest tests/test_gpu_batch_equation.py -x -v --timeout 120 --timeout-method thread
run gpu 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run bench_on 300 python bench.py
TMV_SUBCHECK=0 run bench_off 300 python bench.py
run bench_on2 300 python bench.py
for f in bench_on bench_off bench_on2; do python3 -c "import json,sys; d=json.loads(open('$OUT/$f.log').read().strip().splitlines()[-1]); print('$f', d['value'], d['batch_latency_ms'], d['roofline']['launch_avg_ms'])"; done
