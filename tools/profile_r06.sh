#!/bin/bash
# Round-6 profile (under gpurun; tag = first argument): the round-4 passes of
# tools/profile_round_pmc.sh plus single launches of the 125k shard and of the
# bench's 2.56M size (tools/launch_alone.py --stats: groups, failing groups,
# fallback entries) under a kernel trace and an SQ_INSTS_VALU_INT64 PMC pass,
# the inputs of tools/kernel_fracs.py.  Outputs under gpurun_out/prof_<tag>/;
# stops at the first timeout / crash.  Second argument "alone": only the two
# single-launch passes (kernel_fracs.py / pmc_launch.py inputs).
R=${1:-r06}
OUT=gpurun_out/prof_$R
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() {
  local name=$1 limit=$2; shift 2
  timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a $OUT/steps.txt
  case $rc in 0) ;; *) echo "stopping after $name"; tail -20 $OUT/$name.log; exit $rc;; esac
}
A="python3 tools/launch_alone.py --n 125000,2560000 --stats"
B="python3 tools/pmc_driver.py --launches 2 --per-launch 256"
run alone_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/alone_trace -o alone -- $A --reps 6
run alone_pmc 300 rocprofv3 --pmc SQ_INSTS_VALU_INT64 SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d $OUT/alone_pmc -o alone -- $A --reps 3 --warmup 1
[ "$2" = alone ] && { echo done | tee -a $OUT/steps.txt; exit 0; }
run trace_alone 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_alone -o bench -- python3 bench.py --steps 20 --warmup 5 --inflight 1 --no-cpu-baseline --no-extras
run fetch 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- $B
run write 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- $B
run valu 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES --output-format csv -d $OUT/valu -o valu -- $B
run busy 180 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 --output-format csv -d $OUT/busy -o busy -- $B
run fetchcal 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetchcal -o fetchcal -- ./tools/fetchbench
echo done | tee -a $OUT/steps.txt
