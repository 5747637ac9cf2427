#!/bin/bash
# Round-3 GPU call M: the round profile of the current build
# (tools/profile_r03.sh r03b), then kernel traces of the C3 / C4 native
# loops (which kernels the commit / light paths spend their GPU time in).
set -o pipefail
OUT=gpurun_out/r03m
mkdir -p $OUT
bash tools/profile_r03.sh r03b > $OUT/profile.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c3 -o c3 -- \
  python3 tools/bench_configs.py --only 3 --native-only > $OUT/c3.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c4 -o c4 -- \
  python3 tools/bench_configs.py --only 4 --native-only > $OUT/c4.log 2>&1
