#!/bin/bash
# Full GPU suite, then the C2 bench (batch equation) and the per-entry bench (under gpurun).
OUT=gpurun_out/${1:-quick}
mkdir -p $OUT
run() {
  local name=$1; shift
  timeout -k 10 "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  [ $rc -ne 0 ] && { tail -30 $OUT/$name.log; exit $rc; }
  return 0
}
run gpu 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run bench 300 python bench.py --no-cpu-baseline
run bench_pe 300 python bench.py --no-cpu-baseline --method per-entry
run bench2 300 python bench.py --no-cpu-baseline
for f in bench bench_pe bench2; do python3 -c "import json,sys; d=json.loads(open('$OUT/$f.log').read().strip().splitlines()[-1]); print('$f', d['value'], d['batch_latency_ms'], d['roofline']['launch_avg_ms'])"; done
