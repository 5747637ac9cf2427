#!/bin/bash
timeout -k 10 60 ./tools/fieldbench.bin 1048576 > gpurun_out/fieldbench_v2.json 2>&1 || exit 1
# End-to-end host-buffer path: per-stage host timing and lane/chunk A/B.
set -o pipefail
out=gpurun_out/e2e_t
mkdir -p $out
TMV_HOST_TIMING=1 timeout -k 10 200 python tools/e2e_probe.py > $out/timing.log 2>&1 || { tail -5 $out/timing.log; exit 1; }
tail -40 $out/timing.log
for cfg in "4 40000" "4 80000" "4 131072" "3 65536" "2 262144"; do
  set -- $cfg
  TMV_HOST_LANES=$1 TMV_HOST_CHUNK=$2 timeout -k 10 120 python tools/e2e_probe.py 2>/dev/null | tail -1 || exit 1
done
