#!/bin/bash
# A/B of bench.py argument sets (under gpurun), interleaved, twice:
#   bash tools/gpu_ab_args.sh "--batches-per-step 32" "--batches-per-step 64"
set -o pipefail
mkdir -p gpurun_out/ab
for rep in 1 2; do
  for a in "$@"; do
    timeout -k 10 200 python -u bench.py --steps ${AB_STEPS:-20} --warmup 5 --no-cpu-baseline --no-extras $a > gpurun_out/ab/b.log 2>&1 \
      || { echo "bench failed: $a"; tail -20 gpurun_out/ab/b.log; exit 1; }
    echo "$a rep$rep: $(grep '^{' gpurun_out/ab/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
  done
done
