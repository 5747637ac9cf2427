#!/bin/bash
# Round-3 GPU call P: streamed host batches -- part sizes and first-part
# size A/B on the 640k-signature end-to-end probe.
set -o pipefail
OUT=gpurun_out/r03p
mkdir -p $OUT
for rep in 1 2; do
  for cfg in "" "TMV_STREAM_PART=131072" "TMV_STREAM_PART=262144" "TMV_STREAM_FIRST=16384" "TMV_STREAM_FIRST=65536 TMV_STREAM_PART=131072"; do
    env $cfg timeout -k 10 200 python -u tools/e2e_probe.py > $OUT/p.log 2>&1 || { tail -5 $OUT/p.log; exit 1; }
    echo "[$cfg] rep$rep: $(tail -1 $OUT/p.log)" >> $OUT/e2e_parts.txt
  done
done
