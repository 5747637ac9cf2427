#!/bin/bash
# Profiles the bench workload on the GPU box (run under gpurun).
#   kernel trace + stats of the default bench, then PMC passes (one counter
#   group per pass, no tracing domains mixed with --pmc).  Outputs under
#   gpurun_out/prof_<tag>/.  Stops at the first timeout / crash.
R=${1:-r01}
OUT=gpurun_out/prof_$R
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() {
  local name=$1; shift
  timeout -k 10 300 "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  case $rc in 124|137|134|139) echo "stopping after $name"; exit $rc;; esac
  return 0
}
B="python3 tools/pmc_driver.py --launches 4"
run trace rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench -- python3 bench.py
run fetch rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- $B
run write rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- $B
run valu rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES --output-format csv -d $OUT/valu -o valu -- $B
run busy rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_VALU_MUL_I32 --output-format csv -d $OUT/busy -o busy -- $B
echo done
