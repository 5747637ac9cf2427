#!/bin/bash
# Round-3 GPU call Q: mixed launches with per-kind group sizes (ed25519 half
# 128 + located fallback, sr25519 half 64) -- the mixed / sr25519 GPU tests,
# C5 per method; then the streamed-part A/B of the end-to-end probe.
set -o pipefail
OUT=gpurun_out/r03q
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_batch_equation.py tests/test_gpu_configs.py tests/test_gpu_ed25519.py > $OUT/tests.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_configs.py --only 5 --c5-methods "batch m=64,batch default,per-entry" > $OUT/c5.log 2>&1 &&
bash tools/gpu_r03_p.sh
