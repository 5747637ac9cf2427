#!/bin/bash
# Round-3 GPU call B: field-arithmetic A/B on the current tree (HEAD field /
# asm multiply-adds / empty-asm barrier), then the whole GPU suite (at-size
# C3 / C4 included) on the barrier build.
set -o pipefail
B=tendermint_amd/_build
OUT=gpurun_out/r03b
mkdir -p $OUT
AB_REPS=3 bash tools/gpu_ab_so.sh old asm barrier > $OUT/ab_field.txt 2>&1
rc=$?
echo "ab rc=$rc" >> $OUT/ab_field.txt
[ $rc -le 1 ] || exit $rc
pick=old
grep -q "^tests ok on barrier" $OUT/ab_field.txt && pick=barrier
cp $B/ab_$pick.so $B/libtmgpu.so
echo "suite on: $pick" > $OUT/gpu_tests.log
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread -m gpu tests >> $OUT/gpu_tests.log 2>&1
