#!/bin/bash
# Round-3 GPU call U: register budgets -- k_msm_wpart for 3 waves / SIMD
# (168 VGPRs, 2 spilled), k_msm_accum for 4 (128 VGPRs, 26 spilled).
set -o pipefail
mkdir -p gpurun_out/r03u
AB_REPS=3 bash tools/gpu_ab_so.sh base w3 a4 > gpurun_out/r03u/ab.txt 2>&1
rc=$?; echo "ab rc=$rc" >> gpurun_out/r03u/ab.txt; exit $rc
