#!/bin/bash
# A/B of one environment knob on the C2 bench (batch equation and per entry),
# with the batch-equation / ed25519 GPU tests under the knob first (under gpurun).
#   bash tools/gpu_ab_env.sh NAME VALUE
K=$1; V=$2
OUT=gpurun_out/ab_$K
mkdir -p $OUT
run() {
  local name=$1; shift
  timeout -k 10 "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  [ $rc -ne 0 ] && { tail -30 $OUT/$name.log; exit $rc; }
  return 0
}
B="python bench.py --no-cpu-baseline --steps 3072"
env $K=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_batch_equation.py tests/test_gpu_ed25519.py tests/test_gpu_sr25519.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo tests failed; tail -30 $OUT/tests.log; exit 1; }
run off1 300 $B
export $K=$V
run on1 300 $B
run on_pe 300 $B --method per-entry
unset $K
run off2 300 $B
run off_pe 300 $B --method per-entry
export $K=$V
run on2 300 $B
for f in off1 on1 off2 on2 off_pe on_pe; do python3 -c "import json,sys; d=json.loads(open('$OUT/$f.log').read().strip().splitlines()[-1]); print('$f', d['value'], d['batch_latency_ms'], d['roofline']['launch_avg_ms'])"; done
