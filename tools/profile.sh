#!/bin/bash
# Round profile (run under gpurun; tag = first argument): kernel trace + stats of the driver's
# bench command, then PMC passes over tools/pmc_driver.py (one counter group
# per pass, nothing else traced).  Outputs under gpurun_out/prof_<tag>/.
# Stops at the first timeout / crash.
R=${1:-r02}
OUT=gpurun_out/prof_$R
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() {
  local name=$1 limit=$2; shift 2
  timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a $OUT/steps.txt
  case $rc in 0) ;; *) echo "stopping after $name"; exit $rc;; esac
}
B="python3 tools/pmc_driver.py --launches 4"
run trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline
run trace_ss 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_ss -o bench -- python3 bench.py --steps 48 --warmup 8 --no-cpu-baseline --no-extras
run fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- $B
run write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- $B
run valu 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES --output-format csv -d $OUT/valu -o valu -- $B
run busy 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 --output-format csv -d $OUT/busy -o busy -- $B
echo done | tee -a $OUT/steps.txt
