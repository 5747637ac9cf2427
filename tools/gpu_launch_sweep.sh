#!/bin/bash
# C2 bench over batches per launch and launches in flight (under gpurun).
OUT=gpurun_out/lsweep
mkdir -p $OUT
B="python bench.py --no-cpu-baseline --steps 3072"
for cfg in "32 4" "16 4" "48 4" "64 4" "32 3" "32 6" "24 6" "16 8"; do
  set -- $cfg
  timeout -k 10 300 $B --per-launch $1 --inflight $2 > $OUT/p$1_i$2.log 2>&1 || { echo "p$1 i$2 failed"; tail -20 $OUT/p$1_i$2.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/p$1_i$2.log').read().strip().splitlines()[-1]); print('per-launch $1 inflight $2', d['value'])"
done
