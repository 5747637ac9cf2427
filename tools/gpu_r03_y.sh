#!/bin/bash
# Round-3 GPU call Y: C3 / C4 native loops with the caller pipelining windows.
set -o pipefail
out=gpurun_out/r03y
mkdir -p $out
timeout -k 10 900 python -u tools/c34_pipeline.py --modes seq,thr2,thr3,whole,seq,thr2 > $out/pipe.txt 2>&1 || { tail -20 $out/pipe.txt; exit 1; }
