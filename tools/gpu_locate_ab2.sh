#!/bin/bash
# Located fallback at its default gate (>= 150k entries per launch) vs off:
# steady-state C2 bench (3 pairs) and C5 (1M mixed, one launch).
set -o pipefail
out=gpurun_out/locate2
mkdir -p $out
run() {  # name, env, args
  local name=$1 envs=$2; shift 2
  env $envs timeout -k 10 200 python -u bench.py --warmup 5 --no-extras --no-cpu-baseline "$@" \
    > $out/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $out/$name.log; exit 1; }
  grep '^{' $out/$name.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('%-14s' % '$name', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step']*d['steps'],3), 'ms')"
}
for rep in 1 2 3; do
  run s1536_off_$rep "TMV_LOCATE_MIN=0" --steps 1536
  run s1536_def_$rep "" --steps 1536
done
for v in 0 150000; do
  TMV_LOCATE_MIN=$v timeout -k 10 300 python -u tools/bench_configs.py --only 5 > $out/c5_$v.log 2>&1 || { tail -5 $out/c5_$v.log; exit 1; }
  echo "C5 locate_min=$v"; grep -i "c5" $out/c5_$v.log | tail -4
done
