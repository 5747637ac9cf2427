#!/bin/bash
# Sub-group bisection A/B on C5 (1M mixed, one launch) and the C2 bench with
# 8 launches in flight (under gpurun).
OUT=gpurun_out/subcheck2
mkdir -p $OUT
run() {
  local name=$1; shift
  timeout -k 10 "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  [ $rc -ne 0 ] && { tail -30 $OUT/$name.log; exit $rc; }
  return 0
}
run c5_on 300 python tools/bench_configs.py --only 5
TMV_SUBCHECK=0 run c5_off 300 python tools/bench_configs.py --only 5
run b8_on 300 python bench.py --inflight 8 --no-cpu-baseline
TMV_SUBCHECK=0 run b8_off 300 python bench.py --inflight 8 --no-cpu-baseline
for f in b8_on b8_off; do python3 -c "import json,sys; d=json.loads(open('$OUT/$f.log').read().strip().splitlines()[-1]); print('$f', d['value'], d['batch_latency_ms'], d['roofline']['launch_avg_ms'])"; done
grep -h "C5\|M/s" $OUT/c5_on.log $OUT/c5_off.log | head -20
