#!/bin/bash
# Round-3 GPU call W: end-to-end host-buffer path at 2.56 M signatures per
# call -- per-stage host timing, then chunk / part / pinning knobs.
set -o pipefail
out=gpurun_out/r03w
mkdir -p $out
TMV_E2E_NB=256 TMV_HOST_TIMING=1 timeout -k 10 300 python -u tools/e2e_probe.py > $out/timing.log 2>&1 || { tail -5 $out/timing.log; exit 1; }
for cfg in "" "TMV_STREAM_CHUNK=4194304" "TMV_STREAM_CHUNK=1048576" "TMV_STREAM_PART=262144" "TMV_REGISTER=0" "TMV_HOST_LANES=3" ""; do
  echo "cfg=$cfg" >> $out/ab.txt
  env $cfg TMV_E2E_NB=256 timeout -k 10 200 python -u tools/e2e_probe.py >> $out/ab.txt 2>&1 || exit 1
done
