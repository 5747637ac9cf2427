#!/bin/bash
# A/B of environment settings for bench.py (under gpurun), interleaved:
#   bash tools/gpu_ab_env.sh "" "TMV_MSM_CHUNK=32" ...   ("" = defaults)
set -o pipefail
mkdir -p gpurun_out/ab
for rep in $(seq ${AB_REPS:-2}); do
  for a in "$@"; do
    env $a timeout -k 10 200 python -u bench.py --steps ${AB_STEPS:-20} --warmup 5 --no-cpu-baseline --no-extras \
      > gpurun_out/ab/b.log 2>&1 || { echo "bench failed: $a"; tail -20 gpurun_out/ab/b.log; exit 1; }
    echo "[$a] rep$rep: $(grep '^{' gpurun_out/ab/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,2), 'M/s', d['ms_per_step'])")"
  done
done
