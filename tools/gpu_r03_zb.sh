#!/bin/bash
# Round-3 GPU call ZB: C5 (1M mixed, batch default) kernel stats.
set -o pipefail
out=gpurun_out/r03zb
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/c5 -o c5 -- python3 tools/bench_configs.py --only 5 --c5-methods "batch default" > $out/c5.log 2>&1 || { tail -20 $out/c5.log; exit 1; }
tail -3 $out/c5.log
