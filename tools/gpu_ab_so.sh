#!/bin/bash
# A/B of several builds of libtmgpu.so in one GPU call:
#   bash tools/gpu_ab_so.sh old new [more ...]
# runs the batch-equation / ed25519 GPU tests on every build
# (tendermint_amd/_build/ab_<name>.so, copied over libtmgpu.so in turn), then
# the C2 bench (--steps 20, the driver's shape) REPS times per build,
# interleaved; leaves the last named build in place.
set -o pipefail
B=tendermint_amd/_build
OUT=gpurun_out/ab
mkdir -p $OUT
REPS=${AB_REPS:-3}
[ $# -ge 2 ] || { echo "usage: $0 name1 name2 [...]"; exit 2; }
for v in "$@"; do
  cp $B/ab_$v.so $B/libtmgpu.so
  timeout -k 10 300 python -u -m pytest tests/test_gpu_batch_equation.py tests/test_gpu_ed25519.py -x -q \
    -k "not kernel_timing" --timeout 120 --timeout-method thread > $OUT/tests_$v.log 2>&1 \
    || { echo "tests failed on $v"; tail -30 $OUT/tests_$v.log; exit 1; }
  echo "tests ok on $v: $(tail -1 $OUT/tests_$v.log)"
done
run() {
  timeout -k 10 200 python -u bench.py --steps ${AB_STEPS:-20} --warmup 5 --no-extras --no-cpu-baseline \
    > $OUT/bench.log 2>&1 || { tail -5 $OUT/bench.log; exit 1; }
  grep '^{' $OUT/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,2), 'M/s', d['ms_per_step'], 'ms/step')"
}
for rep in $(seq $REPS); do
  for v in "$@"; do
    cp $B/ab_$v.so $B/libtmgpu.so
    echo "$v rep$rep: $(run)"
  done
done
