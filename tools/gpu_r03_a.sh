#!/bin/bash
# Round-3 GPU call A: field-arithmetic A/B (HEAD field vs biased single-chain
# columns: empty-asm barrier / asm multiply-adds), then the GPU suite, the
# at-size C3 / C4 tests and the C1/C3/C4 configs on the build that passed.
set -o pipefail
B=tendermint_amd/_build
OUT=gpurun_out/r03
mkdir -p $OUT
AB_REPS=3 bash tools/gpu_ab_so.sh old barrier asm > $OUT/ab_field.txt 2>&1
rc=$?
echo "ab rc=$rc" >> $OUT/ab_field.txt
[ $rc -le 1 ] || exit $rc   # only a failed assertion / bench check continues
pick=old
grep -q "^tests ok on barrier" $OUT/ab_field.txt && pick=barrier
cp $B/ab_$pick.so $B/libtmgpu.so
echo "suite on: $pick" > $OUT/gpu_tests.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests \
  --deselect tests/test_gpu_c3_at_size.py --deselect tests/test_gpu_c4_at_size.py >> $OUT/gpu_tests.log 2>&1 &&
timeout -k 10 900 python -u -m pytest -s -x -v --timeout 400 --timeout-method thread \
  tests/test_gpu_c3_at_size.py tests/test_gpu_c4_at_size.py > $OUT/atsize.log 2>&1 &&
timeout -k 10 400 python -u tools/bench_configs.py --only 1,3,4 > $OUT/configs_c1_c3_c4.log 2>&1
