#!/bin/bash
# Round-3 GPU call S: C3 / C4 native, pooled host layer vs the build before
# it, interleaved three times.
set -o pipefail
OUT=gpurun_out/r03s
mkdir -p $OUT
B=tendermint_amd/_build
for rep in 1 2 3; do
  for v in prepool pool; do
    cp $B/ab_$v.so $B/libtmgpu.so
    timeout -k 10 300 python -u tools/bench_configs.py --only 3,4 --native-only > $OUT/c.log 2>&1 || { tail -5 $OUT/c.log; exit 1; }
    echo "$v rep$rep: $(grep config $OUT/c.log | python -c 'import json,sys; print([json.loads(l)[k] for l in sys.stdin for k in json.loads(l) if k.startswith("native_") and k.endswith("_per_s")])')" >> $OUT/ab.txt
  done
done
