#!/bin/bash
# batch-equation tests, then the C2 bench at 32 / 64 batches per launch (under gpurun).
OUT=gpurun_out/perlaunch
mkdir -p $OUT
run() {
  local name=$1; shift
  timeout -k 10 "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  [ $rc -ne 0 ] && { tail -30 $OUT/$name.log; exit $rc; }
  return 0
}
run beq 300 python -u -m pytest tests/test_gpu_batch_equation.py -x -q --timeout 120 --timeout-method thread
run b32 300 python bench.py --no-cpu-baseline
run b64 300 python bench.py --no-cpu-baseline --per-launch 64
run b64i8 300 python bench.py --no-cpu-baseline --per-launch 64 --inflight 8
run b32i8 300 python bench.py --no-cpu-baseline --inflight 8
for f in b32 b64 b64i8 b32i8; do python3 -c "import json,sys; d=json.loads(open('$OUT/$f.log').read().strip().splitlines()[-1]); print('$f', d['value'], d['roofline']['launch_avg_ms'])"; done
