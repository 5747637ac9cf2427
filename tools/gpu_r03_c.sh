#!/bin/bash
# Round-3 GPU call C: H2D copy rates, the host-pipeline tests, secondary
# configs at BASELINE sizes (host phase times for C3 / C4), the round profile
# (tools/profile_r03.sh), the driver's bench command, then the whole suite.
set -o pipefail
OUT=gpurun_out/r03c
mkdir -p $OUT
timeout -k 10 60 ./tools/h2dbench 128 > $OUT/h2dbench.json 2>&1 &&
HSA_ENABLE_SDMA=0 timeout -k 10 200 python -u tools/e2e_probe.py > $OUT/e2e_nosdma.log 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_host_pipeline.py > $OUT/host_pipeline.log 2>&1 &&
TMV_HOST_TIMING=1 timeout -k 10 400 python -u tools/bench_configs.py --only 1,3,4 > $OUT/configs_c1_c3_c4.log 2> $OUT/configs_host_timing.log &&
timeout -k 10 300 python -u tools/bench_configs.py --only 5 --c5-methods "batch m=64,batch m=128,per-entry" > $OUT/configs_c5.log 2>&1 &&
bash tools/profile_r03.sh r03 > $OUT/profile.log 2>&1 &&
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_s20.json 2> $OUT/bench_s20.err &&
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread -m gpu tests > $OUT/gpu_tests.log 2>&1
