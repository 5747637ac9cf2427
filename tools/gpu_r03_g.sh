#!/bin/bash
# Round-3 GPU call G: compact k_msm_join -- per-kernel profile (one launch at
# a time) of head / join2 / wjoin2, then the interleaved bench A/B.
set -o pipefail
mkdir -p gpurun_out/r03g
bash tools/gpu_prof_ab.sh head join2 wjoin2 > gpurun_out/r03g/prof.txt 2>&1 || exit 1
AB_REPS=3 bash tools/gpu_ab_so.sh head join2 wjoin2 > gpurun_out/r03g/ab.txt 2>&1
rc=$?; echo "ab rc=$rc" >> gpurun_out/r03g/ab.txt; exit $rc
