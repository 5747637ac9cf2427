#!/bin/bash
# Round-3 GPU call K: paired Niels points A/B (sortlds = LDS-staged sort,
# pair = + (+P, -P) slots), then the C3 / C4 host-phase runs (call J).
set -o pipefail
mkdir -p gpurun_out/r03k
bash tools/gpu_prof_ab.sh sortlds pair > gpurun_out/r03k/prof.txt 2>&1 || exit 1
AB_REPS=3 bash tools/gpu_ab_so.sh sortlds pair > gpurun_out/r03k/ab.txt 2>&1
rc=$?; echo "ab rc=$rc" >> gpurun_out/r03k/ab.txt; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_r03_j.sh
