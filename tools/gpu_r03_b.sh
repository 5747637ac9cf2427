#!/bin/bash
# Round-3 GPU call B: field-arithmetic A/B (HEAD field / asm multiply-adds /
# empty-asm barrier), end-to-end probe with and without pinning the caller's
# pages, then the whole GPU suite (at-size C3 / C4 included) on the working
# tree's build (ab_cur.so).
set -o pipefail
B=tendermint_amd/_build
OUT=gpurun_out/r03b
mkdir -p $OUT
AB_REPS=3 bash tools/gpu_ab_so.sh old asm barrier > $OUT/ab_field.txt 2>&1
rc=$?
echo "ab rc=$rc" >> $OUT/ab_field.txt
[ $rc -le 1 ] || exit $rc
cp $B/ab_cur.so $B/libtmgpu.so
for r in 1 0 1 0; do
  TMV_REGISTER=$r TMV_HOST_TIMING=1 timeout -k 10 300 python -u tools/e2e_probe.py > $OUT/e2e_reg$r.log 2>&1 \
    || { tail -5 $OUT/e2e_reg$r.log; exit 1; }
  tail -1 $OUT/e2e_reg$r.log >> $OUT/e2e.txt
done
echo "suite on: cur" > $OUT/gpu_tests.log
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread -m gpu tests >> $OUT/gpu_tests.log 2>&1
