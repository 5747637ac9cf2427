#!/bin/bash
# Round-3 GPU call ZD: A/B of the lane claims on one box -- ab_old.so (device
# lock held for a whole host-buffer call) vs ab_new.so (held only while a
# call stages and launches), C3 / C4 native loops one window at a time and
# with 2 / 3 windows in flight, interleaved; leaves ab_new in place.
set -o pipefail
B=tendermint_amd/_build
out=gpurun_out/r03zd
mkdir -p $out
for rep in 1 2 3; do
  for v in old new; do
    cp $B/ab_$v.so $B/libtmgpu.so
    echo "== $v rep$rep" >> $out/ab.txt
    timeout -k 10 300 python -u tools/c34_pipeline.py --modes seq,thr2,thr3 >> $out/ab.txt 2>&1 || { tail -5 $out/ab.txt; exit 1; }
  done
done
cp $B/ab_new.so $B/libtmgpu.so
