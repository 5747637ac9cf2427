#!/bin/bash
# Round-3 GPU call V: end-to-end probe size -- one host-resident call of 64,
# 128 or 256 C2 batches (0.64 / 1.28 / 2.56 M signatures) against the same
# batches in one resident launch.
set -o pipefail
mkdir -p gpurun_out/r03v
for ke in 64 256 128; do
  TMV_BENCH_SUSTAIN_S=0 TMV_BENCH_E2E_BATCHES=$ke timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 \
    > gpurun_out/r03v/bench_e2e$ke.json 2> gpurun_out/r03v/bench_e2e$ke.err || exit $?
done
