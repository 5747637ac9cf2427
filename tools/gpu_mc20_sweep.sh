#!/bin/bash
# Group size / window at the driver's --steps 20 and at steady state.
set -o pipefail
out=gpurun_out/mc20
mkdir -p $out
run() {  # name, args
  local name=$1; shift
  timeout -k 10 150 python -u bench.py --warmup 5 --no-extras --no-cpu-baseline "$@" \
    > $out/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $out/$name.log; exit 1; }
  python - $out/$name.log $name <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith('{')][-1]; d=json.loads(l)
print("%-16s value=%7.2f M/s ms=%.3f sizes=%s" % (sys.argv[2], d["value"]/1e6, d["ms_per_step"]*d["steps"], d["config"].get("launch_sizes")[:3]))
PY
}
for rep in 1 2; do
  for mc in "6 5" "5 5" "5 4" "6 4"; do
    set -- $mc
    run s20_m$1_c$2_$rep --steps 20 --group-log2 $1 --window $2
  done
done
for mc in "6 5" "5 5" "5 4"; do
  set -- $mc
  run s768_m$1_c$2 --steps 768 --group-log2 $1 --window $2
done
