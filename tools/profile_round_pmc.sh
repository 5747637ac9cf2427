#!/bin/bash
# Round profile (round 3 on; round 4 reran it unchanged) (under gpurun; tag = first argument).  Outputs under
# gpurun_out/prof_<tag>/; stops at the first timeout / crash.
#   trace_alone  kernel trace + stats of bench.py --inflight 1 (one launch at
#                a time: every dispatch's duration is the kernel's own, the
#                roofline's dominant-kernel figure)
#   trace        the same of the driver's bench command (4 launches in flight)
#   fetch/write/valu/busy  PMC passes over tools/pmc_driver.py at the bench's
#                launch size (256 C2 batches = 2.56M signatures per launch)
#   fetchcal     FETCH_SIZE of tools/fetchbench (known byte counts: the
#                gfx950 correction per access pattern)
R=${1:-r04}
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
B="python3 tools/pmc_driver.py --launches 2 --per-launch 256"
run trace_alone 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_alone -o bench -- python3 bench.py --steps 20 --warmup 5 --inflight 1 --no-cpu-baseline --no-extras
run trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras
run fetch 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- $B
run write 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- $B
run valu 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES --output-format csv -d $OUT/valu -o valu -- $B
run busy 180 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 --output-format csv -d $OUT/busy -o busy -- $B
run fetchcal 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetchcal -o fetchcal -- ./tools/fetchbench
echo done | tee -a $OUT/steps.txt
