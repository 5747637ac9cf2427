#!/bin/bash
# Per-kernel durations of several builds (one launch at a time):
#   bash tools/gpu_prof_ab.sh name1 name2 ...   (tendermint_amd/_build/ab_<name>.so)
# rocprofv3 --kernel-trace --stats of bench.py --inflight 1 per build, into
# gpurun_out/profab/<name>/; leaves the last named build in place.
set -o pipefail
B=tendermint_amd/_build
OUT=gpurun_out/profab
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in "$@"; do
  cp $B/ab_$v.so $B/libtmgpu.so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$v -o k -- \
    python3 bench.py --steps 10 --warmup 3 --inflight 1 --no-cpu-baseline --no-extras > $OUT/$v.log 2>&1 \
    || { echo "profile failed on $v"; tail -5 $OUT/$v.log; exit 1; }
  echo "$v: $(grep '^{' $OUT/$v.log | tail -1 | cut -c1-120)"
done
