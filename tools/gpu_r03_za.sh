#!/bin/bash
# Round-3 GPU call ZA: the Python chain drivers at depth 1 / 2, with and
# without gc.freeze() (tools/c34_pipeline.py --python).
set -o pipefail
out=gpurun_out/r03za
mkdir -p $out
timeout -k 10 900 python -u tools/c34_pipeline.py --python --modes seq,thr2 > $out/pipe.txt 2>&1 || { tail -20 $out/pipe.txt; exit 1; }
