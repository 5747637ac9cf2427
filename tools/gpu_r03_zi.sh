#!/bin/bash
# Round-3 GPU call ZI: part sizes of a 2.56 M streamed call (one pipeline,
# chunks of 4 M), interleaved twice.
set -o pipefail
out=gpurun_out/r03zi
mkdir -p $out
for rep in 1 2; do
  for cfg in "TMV_STREAM_PART=131072" "TMV_STREAM_PART=262144" "TMV_STREAM_PART=524288" "TMV_STREAM_PART=65536" "TMV_STREAM_FIRST=131072"; do
    echo "cfg=$cfg" >> $out/ab.txt
    env $cfg TMV_E2E_NB=256 timeout -k 10 300 python -u tools/e2e_probe.py >> $out/ab.txt 2>&1 || { tail -5 $out/ab.txt; exit 1; }
  done
done
