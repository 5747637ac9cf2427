#!/bin/bash
# Kernel trace + stats of the bench workload (run under gpurun).
#   bash tools/prof_bench.sh <tag> [bench args...]
T=${1:-bench}; shift
OUT=gpurun_out/prof_$T
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o $T -- python3 bench.py --no-cpu-baseline "$@" > $OUT/bench.log 2>&1
