#!/bin/bash
# A/B of environment settings on the C2 bench (under gpurun):
#   bash tools/gpu_ab.sh "TMV_X=1" "TMV_X=2 TMV_Y=3" ...
# Each setting first runs the batch-equation GPU tests, then every setting
# (and the default, "-") runs the bench twice, interleaved.
set -o pipefail
OUT=gpurun_out/ab
mkdir -p $OUT
STEPS=${AB_STEPS:-20}
for cfg in "$@"; do
  env $cfg timeout -k 10 300 python -u -m pytest tests/test_gpu_batch_equation.py tests/test_gpu_ed25519.py -x -q \
    -k "not kernel_timing" --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed under $cfg"; tail -30 $OUT/tests.log; exit 1; }
  echo "tests ok under $cfg: $(tail -1 $OUT/tests.log)"
done
for rep in 1 2; do
  for cfg in "-" "$@"; do
    e=""; [ "$cfg" != "-" ] && e="$cfg"
    env $e timeout -k 10 200 python -u bench.py --steps $STEPS --warmup 5 --no-cpu-baseline --no-extras > $OUT/b.log 2>&1 \
      || { echo "bench failed under $cfg"; tail -20 $OUT/b.log; exit 1; }
    echo "$cfg rep$rep: $(grep '^{' $OUT/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
  done
done
