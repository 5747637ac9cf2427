#!/bin/bash
# Kernel-time profile of the key-merged form on 1M keyed signatures, per
# group size (csv kernel traces under gpurun_out/prof_km/).
set -e
cd "$(dirname "$0")/.."
ROOT=$PWD
mkdir -p gpurun_out/prof_km
cd /tmp && export TMPDIR=/tmp
for g in ${KM_GROUPS:-8 9 10}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_km" -o km_g$g -- \
    python3 "$ROOT/tools/km_bench.py" --n 1000000 --keys 2000 --reps 3 --methods key_merged --group-log2 $g \
    > "$ROOT/gpurun_out/prof_km/km_g$g.log" 2>&1
done
