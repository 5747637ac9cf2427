#!/bin/bash
# C2 bench over group size / window with and without the sub-group check (under gpurun).
OUT=gpurun_out/msweep
mkdir -p $OUT
run() {
  local name=$1; shift
  timeout -k 10 "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  [ $rc -ne 0 ] && { tail -30 $OUT/$name.log; exit $rc; }
  return 0
}
B="python bench.py --no-cpu-baseline --steps 192"
run m6 300 $B
TMV_SUBCHECK=1 run m6s 300 $B
TMV_SUBCHECK=1 run m7c5s 300 $B --group-log2 7 --window 5
TMV_SUBCHECK=1 run m7c6s 300 $B --group-log2 7 --window 6
TMV_SUBCHECK=0 run m7c6 300 $B --group-log2 7 --window 6
TMV_SUBCHECK=1 run m8c6s 300 $B --group-log2 8 --window 6
TMV_SUBCHECK=1 run m5c5s 300 $B --group-log2 5 --window 5
for f in m6 m6s m7c5s m7c6s m7c6 m8c6s m5c5s; do python3 -c "import json,sys; d=json.loads(open('$OUT/$f.log').read().strip().splitlines()[-1]); print('$f', d['value'], d['batch_latency_ms'])"; done
