#!/bin/bash
# One GPU call: the GPU suite (minus the at-size modules), the at-size C3 / C4
# tests, then C1/C3/C4 of tools/bench_configs.py at BASELINE sizes.
set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests \
  --deselect tests/test_gpu_c3_at_size.py --deselect tests/test_gpu_c4_at_size.py > gpurun_out/r03/gpu_tests.log 2>&1 &&
timeout -k 10 900 python -u -m pytest -s -x -v --timeout 400 --timeout-method thread \
  tests/test_gpu_c3_at_size.py tests/test_gpu_c4_at_size.py > gpurun_out/r03/atsize.log 2>&1 &&
timeout -k 10 400 python -u tools/bench_configs.py --only 1,3,4 > gpurun_out/r03/configs_c1_c3_c4.log 2>&1
