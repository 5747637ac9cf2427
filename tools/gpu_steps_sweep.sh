#!/bin/bash
# C2 bench rate against the number of timed steps (tail of the 4 in-flight
# launches), with and without the sub-group check (under gpurun).
OUT=gpurun_out/steps
mkdir -p $OUT
run() {
  local name=$1; shift
  timeout -k 10 "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  [ $rc -ne 0 ] && { tail -30 $OUT/$name.log; exit $rc; }
  return 0
}
B="python bench.py --no-cpu-baseline"
run s384 300 $B --steps 384
run s1536 300 $B --steps 1536
run s3072 300 $B --steps 3072
TMV_SUBCHECK=1 run s3072sub 300 $B --steps 3072
run s3072i8 300 $B --steps 3072 --inflight 8
run s3072p16 300 $B --steps 3072 --per-launch 16
for f in s384 s1536 s3072 s3072sub s3072i8 s3072p16; do python3 -c "import json,sys; d=json.loads(open('$OUT/$f.log').read().strip().splitlines()[-1]); print('$f', d['value'], d['roofline']['launch_avg_ms'])"; done
