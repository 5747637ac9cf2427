#!/bin/bash
# Round-3 final check on one box: whole GPU suite, smoke, the driver's bench
# command, BASELINE configs 1 / 3 / 4 / 5.
set -o pipefail
OUT=gpurun_out/r03final
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests > $OUT/gpu_tests.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_s20.json 2> $OUT/bench_s20.err &&
timeout -k 10 400 python -u tools/bench_configs.py --only 1,3,4,5 --native-only --c5-methods "batch default,per-entry" > $OUT/configs.log 2>&1
