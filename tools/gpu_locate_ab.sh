#!/bin/bash
# Located fallback: exactness with it forced on every batch-equation launch,
# then the bench with it off / default / forced.
set -o pipefail
out=gpurun_out/locate
mkdir -p $out
TMV_LOCATE_MIN=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_batch_equation.py tests/test_gpu_configs.py tests/test_gpu_fuzz.py tests/test_gpu_sr25519.py \
  > $out/tests_forced.log 2>&1 || { tail -40 $out/tests_forced.log; exit 1; }
tail -1 $out/tests_forced.log
run() {  # name, env, args
  local name=$1 envs=$2; shift 2
  env $envs timeout -k 10 200 python -u bench.py --warmup 5 --no-extras --no-cpu-baseline "$@" \
    > $out/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $out/$name.log; exit 1; }
  grep '^{' $out/$name.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('%-14s' % '$name', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step']*d['steps'],3), 'ms')"
}
for rep in 1 2; do
  run s20_off_$rep "TMV_LOCATE_MIN=0" --steps 20
  run s20_on_$rep "TMV_LOCATE_MIN=1" --steps 20
done
run s1536_off "TMV_LOCATE_MIN=0" --steps 1536
run s1536_on "TMV_LOCATE_MIN=1" --steps 1536
run s1536_off2 "TMV_LOCATE_MIN=0" --steps 1536
run s1536_on2 "TMV_LOCATE_MIN=1" --steps 1536
