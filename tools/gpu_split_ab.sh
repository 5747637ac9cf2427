#!/bin/bash
# Split batch-equation launches (two concurrent halves, one tail) vs one
# stream: parity tests, then the driver-shaped bench and the steady state.
set -o pipefail
out=gpurun_out/split
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_batch_equation.py tests/test_gpu_configs.py tests/test_gpu_fuzz.py > $out/tests.log 2>&1 \
  || { tail -30 $out/tests.log; exit 1; }
tail -3 $out/tests.log
run() {  # name, env, args
  local name=$1 envs=$2; shift 2
  env $envs timeout -k 10 150 python -u bench.py --warmup 5 --no-extras --no-cpu-baseline "$@" \
    > $out/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $out/$name.log; exit 1; }
  python - $out/$name.log $name <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith('{')][-1]; d=json.loads(l)
print("%-18s value=%7.2f M/s ms=%.3f sizes=%s" % (sys.argv[2], d["value"]/1e6, d["ms_per_step"]*d["steps"], d["config"].get("launch_sizes")[:4]))
PY
}
for rep in 1 2; do
  run s20_nosplit_$rep "TMV_SPLIT_MIN=0" --steps 20
  run s20_split_p10_$rep "TMV_SPLIT_MIN=40000" --steps 20
  run s20_split_p20_$rep "TMV_SPLIT_MIN=40000" --steps 20 --plan 20
done
run s1536_nosplit "TMV_SPLIT_MIN=0" --steps 1536
run s1536_split "TMV_SPLIT_MIN=40000" --steps 1536
