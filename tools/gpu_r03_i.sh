#!/bin/bash
# Round-3 GPU call I: LDS-staged k_msm_sort scatter -- per-kernel profile and
# bench A/B against the committed build (join); then C5 1M mixed with groups
# of 64 / 128 on the committed build.
set -o pipefail
mkdir -p gpurun_out/r03i
bash tools/gpu_prof_ab.sh join sortlds pair > gpurun_out/r03i/prof.txt 2>&1 || exit 1
AB_REPS=3 bash tools/gpu_ab_so.sh join sortlds pair > gpurun_out/r03i/ab.txt 2>&1
rc=$?; echo "ab rc=$rc" >> gpurun_out/r03i/ab.txt; [ $rc -eq 0 ] || exit $rc
cp tendermint_amd/_build/ab_join.so tendermint_amd/_build/libtmgpu.so
timeout -k 10 300 python -u tools/bench_configs.py --only 5 --c5-methods "batch m=64,batch m=128,per-entry" > gpurun_out/r03i/configs_c5.log 2>&1
