#!/bin/bash
# Round-3 GPU call ZC: per-call lane claims (device lock not held while a
# call waits for the device) -- concurrency tests, host-path GPU tests, and
# the C3 / C4 windows-in-flight loops.
set -o pipefail
out=gpurun_out/r03zc
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_concurrent_calls.py > $out/tests_conc.txt 2>&1 || { tail -30 $out/tests_conc.txt; exit 1; }
tail -3 $out/tests_conc.txt
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_commit_verify.py tests/test_gpu_host_pipeline.py tests/test_gpu_chains.py tests/test_gpu_keycache.py \
  > $out/tests_host.txt 2>&1 || { tail -30 $out/tests_host.txt; exit 1; }
tail -3 $out/tests_host.txt
timeout -k 10 600 python -u tools/c34_pipeline.py --modes seq,thr2,thr3,seq,thr2,thr3 > $out/pipe.txt 2>&1 || { tail -20 $out/pipe.txt; exit 1; }
cat $out/pipe.txt
