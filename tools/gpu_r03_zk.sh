#!/bin/bash
# Round-3 GPU call ZK: one more box -- the driver's bench command and the
# secondary configs (C3 / C4 native with windows in flight).
set -o pipefail
out=gpurun_out/r03zk
mkdir -p $out
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $out/bench_s20.json 2> $out/bench_s20.err || { tail -20 $out/bench_s20.err; exit 1; }
timeout -k 10 400 python -u tools/bench_configs.py --only 1,3,4,5 --native-only --c5-methods "batch default" > $out/configs.log 2>&1 || { tail -20 $out/configs.log; exit 1; }
