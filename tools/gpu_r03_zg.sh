#!/bin/bash
# Round-3 GPU call ZG: end to end with two callers (2.56 M per call), each
# call's parts on two streams (lane + helper, default) or on the lane's
# stream only (TMV_STREAM_TWO=0: a call then uses two streams, two calls
# four -- the box's hardware queue count); interleaved twice.
set -o pipefail
out=gpurun_out/r03zg
mkdir -p $out
for rep in 1 2; do
  for cfg in "TMV_STREAM_TWO=1" "TMV_STREAM_TWO=0"; do
    echo "cfg=$cfg" >> $out/ab.txt
    env $cfg TMV_E2E_NB=256 TMV_E2E_CALLERS=2 timeout -k 10 300 python -u tools/e2e_probe.py >> $out/ab.txt 2>&1 || { tail -5 $out/ab.txt; exit 1; }
  done
done
