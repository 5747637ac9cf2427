#!/bin/bash
OUT=gpurun_out/subprof
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export TMV_SUBCHECK=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench -- python3 bench.py --no-cpu-baseline --steps 128 > $OUT/trace.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES --output-format csv -d $OUT/valu -o valu -- python3 tools/pmc_driver.py --launches 4 > $OUT/valu.log 2>&1 || exit 1
echo done
