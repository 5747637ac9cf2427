#!/bin/bash
# Round-2 GPU call A: full GPU suite, then bench step-semantics sweep, then
# the PMC counter list.  Stops at the first failing step.
OUT=gpurun_out/r02_a
mkdir -p $OUT
step() {
  local name=$1 limit=$2; shift 2
  timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a $OUT/steps.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step bench_driver 300 python bench.py --steps 20 --warmup 5
for pl in "20 1" "10 2" "5 4" "3 4" "2 4"; do
  set -- $pl
  step bench_s20_p$1_f$2 300 python bench.py --steps 20 --warmup 5 --per-launch $1 --inflight $2 --no-extras --no-cpu-baseline
done
step bench_s1536 300 python bench.py --steps 1536 --warmup 64 --no-cpu-baseline
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 5 60 rocprofv3 --list-avail > $OUT/rocprof_avail.txt 2>&1; echo "avail rc=$?" >> $OUT/steps.txt
echo done >> $OUT/steps.txt
