#!/bin/bash
# Round-3 GPU call Z: chain drivers with windows in flight (chains.in_order):
# the chain GPU tests (C3 / C4 at size included) and bench_configs C3 / C4.
set -o pipefail
out=gpurun_out/r03z
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_chains.py tests/test_gpu_c3_at_size.py tests/test_gpu_c4_at_size.py tests/test_gpu_valset_hash.py \
  > $out/tests.txt 2>&1 || { tail -20 $out/tests.txt; exit 1; }
tail -3 $out/tests.txt
timeout -k 10 600 python -u tools/bench_configs.py --only 3,4 > $out/configs.log 2>&1 || { tail -20 $out/configs.log; exit 1; }
cat $out/configs.log
