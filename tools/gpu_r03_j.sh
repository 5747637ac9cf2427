#!/bin/bash
# Round-3 GPU call J: C3 / C4 native host-layer phase times, each config in
# its own process, unsliced and sliced (TMV_HOST_SLICE = 0 / 512 / 300).
set -o pipefail
OUT=gpurun_out/r03j
mkdir -p $OUT
for cfg in 3 4; do
  for sl in 0 512 300; do
    TMV_HOST_SLICE=$sl TMV_HOST_TIMING=1 timeout -k 10 200 python -u tools/bench_configs.py --only $cfg --native-only \
      > $OUT/c${cfg}_s$sl.log 2> $OUT/c${cfg}_s${sl}_timing.log || exit 1
  done
done
