#!/bin/bash
# Round-3 GPU call D: the driver's bench command, then the round profile
# (tools/profile_r03.sh: kernel traces of the bench alone / in flight, PMC
# passes at the bench's launch size, FETCH_SIZE calibration).
set -o pipefail
OUT=gpurun_out/r03d
mkdir -p $OUT
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_s20.json 2> $OUT/bench_s20.err &&
bash tools/profile_r03.sh r03 > $OUT/profile.log 2>&1
