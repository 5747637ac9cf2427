#!/bin/bash
# C2 bench over group size (2^m) and window bits c (under gpurun).
OUT=gpurun_out/mcsweep
mkdir -p $OUT
B="python bench.py --no-cpu-baseline --steps 3072"
for cfg in "6 5" "5 4" "5 5" "7 5" "7 6" "6 4" "6 6"; do
  set -- $cfg
  timeout -k 10 300 $B --group-log2 $1 --window $2 > $OUT/m$1_c$2.log 2>&1 || { echo "m$1 c$2 failed"; tail -20 $OUT/m$1_c$2.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/m$1_c$2.log').read().strip().splitlines()[-1]); print('m_log2 $1 c $2', d['value'])"
done
