#!/bin/bash
# Round-3 GPU call ZJ: window sizes x windows in flight for the C3 / C4
# native loops (C3 500 / 1000 headers, C4 300 / 600 / 1200 blocks).
set -o pipefail
out=gpurun_out/r03zj
mkdir -p $out
for w in "500 300" "1000 600" "2000 1200" "1000 600"; do
  set -- $w
  echo "== c3 window $1, c4 window $2" >> $out/win.txt
  timeout -k 10 300 python -u tools/c34_pipeline.py --c3-window $1 --c4-window $2 --modes seq,thr2,thr3,thr4 >> $out/win.txt 2>&1 || { tail -5 $out/win.txt; exit 1; }
done
