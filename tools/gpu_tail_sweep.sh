#!/bin/bash
# Driver-shaped bench (--steps 20) under launch plans and tail-kernel priority.
# Each run is one process; prints one compact line per run.
set -o pipefail
out=gpurun_out/tail_sweep
mkdir -p $out
run() {  # name, env, args
  local name=$1 envs=$2; shift 2
  env $envs timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline "$@" \
    > $out/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $out/$name.log; exit 1; }
  python - $out/$name.log $name <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith('{')][-1]; d=json.loads(l)
print("%-22s value=%7.2f M/s ms=%.3f sizes=%s" % (sys.argv[2], d["value"]/1e6, d["ms_per_step"]*d["steps"], d["config"].get("launch_sizes")))
PY
}
for rep in 1 2; do
  run base_$rep "TMV_TAIL_PRIO=1"
  run noprio_$rep "TMV_TAIL_PRIO=0"
  run p6_14_$rep "TMV_TAIL_PRIO=1" --plan 6,14
  run p14_6_$rep "TMV_TAIL_PRIO=1" --plan 14,6
  run p4_16_$rep "TMV_TAIL_PRIO=1" --plan 4,16
  run p4_6_10_$rep "TMV_TAIL_PRIO=1" --plan 4,6,10
  run p20_$rep "TMV_TAIL_PRIO=1" --plan 20
done
