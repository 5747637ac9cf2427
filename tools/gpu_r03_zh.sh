#!/bin/bash
# Round-3 GPU call ZH: two streamed callers under the engine's phase timer,
# and the same with TMV_REGISTER=0 (staging copies instead of pinned pages).
set -o pipefail
out=gpurun_out/r03zh
mkdir -p $out
TMV_HOST_TIMING=1 TMV_E2E_NB=256 TMV_E2E_CALLERS=2 timeout -k 10 300 python -u tools/e2e_probe.py > $out/timing.log 2>&1 || { tail -5 $out/timing.log; exit 1; }
TMV_REGISTER=0 TMV_E2E_NB=256 TMV_E2E_CALLERS=2 timeout -k 10 300 python -u tools/e2e_probe.py > $out/noreg.log 2>&1 || { tail -5 $out/noreg.log; exit 1; }
