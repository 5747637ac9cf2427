#!/bin/bash
# Round-3 GPU call ZF: the bench with the two-caller end-to-end extra.
set -o pipefail
out=gpurun_out/r03zf
mkdir -p $out
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $out/bench_s20.json 2> $out/bench_s20.err || { tail -20 $out/bench_s20.err; exit 1; }
