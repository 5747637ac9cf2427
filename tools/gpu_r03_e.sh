#!/bin/bash
# Round-3 GPU call E: bucket-layout / in-wave join A/B (HEAD, i-major + join,
# w-major + join), GPU batch-equation tests on each build first.
set -o pipefail
mkdir -p gpurun_out/r03e
AB_REPS=3 bash tools/gpu_ab_so.sh head join wjoin > gpurun_out/r03e/ab.txt 2>&1
rc=$?; echo "ab rc=$rc" >> gpurun_out/r03e/ab.txt; exit $rc
