#!/bin/bash
# Round-3 GPU call R: pooled host-layer conversions -- commit / light / chain
# GPU tests (at-size C3 / C4 included), then C1 / C3 / C4 native twice.
set -o pipefail
OUT=gpurun_out/r03r
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu \
  tests/test_commit_verify.py tests/test_gpu_light.py tests/test_gpu_chains.py tests/test_vote_set.py \
  tests/test_gpu_configs.py tests/test_gpu_c3_at_size.py tests/test_gpu_c4_at_size.py > $OUT/tests.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_configs.py --only 1,3,4 --native-only > $OUT/configs1.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_configs.py --only 3,4 --native-only > $OUT/configs2.log 2>&1
