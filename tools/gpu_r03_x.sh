#!/bin/bash
# Round-3 GPU call X: streamed host batches in chunks of up to 4 M entries
# (one pipeline per 2.56 M call) -- host-pipeline GPU tests, e2e probe at
# 0.64 / 2.56 / 5.12 M per call, and the driver's bench command.
set -o pipefail
out=gpurun_out/r03x
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_host_pipeline.py tests/test_gpu_batch_equation.py > $out/tests.txt 2>&1 || { tail -20 $out/tests.txt; exit 1; }
tail -3 $out/tests.txt
for nb in 64 256 512; do
  TMV_E2E_NB=$nb timeout -k 10 300 python -u tools/e2e_probe.py >> $out/probe.txt 2>&1 || exit 1
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $out/bench_s20.json 2> $out/bench_s20.err || exit 1
