#!/bin/bash
# Round-3 GPU call N: two-launch key-table build -- the key-cache / commit /
# light GPU tests, C1 / C3 / C4 native with a kernel trace of C3; H2D copy
# rates (tools/h2dbench); the driver's bench command (with the sustained
# extra).
set -o pipefail
OUT=gpurun_out/r03n
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_keycache.py tests/test_gpu_key_merged.py tests/test_commit_verify.py tests/test_gpu_light.py \
  tests/test_gpu_configs.py tests/test_gpu_c3_at_size.py > $OUT/tests.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_configs.py --only 1,3,4 --native-only > $OUT/configs.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c3 -o c3 -- \
  python3 tools/bench_configs.py --only 3 --native-only > $OUT/c3.log 2>&1 &&
timeout -k 10 60 ./tools/h2dbench 128 > $OUT/h2dbench.json 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_s20.json 2> $OUT/bench_s20.err
