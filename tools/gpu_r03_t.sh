#!/bin/bash
# Round-3 GPU call T: sub-group checks for the groups the located search
# cannot name -- batch-equation / ed25519 / sr25519 / config GPU tests, then
# the C2 bench with and without (TMV_LOC_SUBCHECK=0), interleaved.
set -o pipefail
OUT=gpurun_out/r03t
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_batch_equation.py tests/test_gpu_ed25519.py tests/test_gpu_configs.py tests/test_gpu_host_pipeline.py > $OUT/tests.log 2>&1 &&
AB_REPS=3 bash tools/gpu_ab_env.sh "" "TMV_LOC_SUBCHECK=0" > $OUT/ab.txt 2>&1
