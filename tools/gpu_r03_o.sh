#!/bin/bash
# Round-3 GPU call O: group / window sweep now that the running sums read
# whole buckets (cheaper buckets favour larger windows), and 32-entry
# accumulation chunks (fewer chunk edges to join).
set -o pipefail
OUT=gpurun_out/r03o
mkdir -p $OUT
bash tools/gpu_ab_args.sh "" "--window 7" "--group-log2 8 --window 7" "--group-log2 8 --window 6" > $OUT/ab_group_window.txt 2>&1 &&
bash tools/gpu_ab_env.sh "" "TMV_MSM_CHUNK=32" > $OUT/ab_chunk.txt 2>&1
