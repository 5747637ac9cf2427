#!/bin/bash
# Round-3 GPU call L: whole GPU suite on the current build, smoke, the
# driver's bench command, C1 / C3 / C4 (driver + native) with host phase
# times, C3 / C4 native again.
set -o pipefail
OUT=gpurun_out/r03l
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests > $OUT/gpu_tests.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_s20.json 2> $OUT/bench_s20.err &&
TMV_HOST_TIMING=1 timeout -k 10 400 python -u tools/bench_configs.py --only 1,3,4 > $OUT/configs_c1_c3_c4.log 2> $OUT/configs_host_timing.log &&
timeout -k 10 300 python -u tools/bench_configs.py --only 3,4 --native-only > $OUT/configs_c3_c4_native.log 2>&1
