# A/B of the host-buffer pipeline knobs (lanes x chunk) on the bench's 320k
# C2 call and on 1M keyed signatures (development tool; GPU box).
set -e
out=gpurun_out/e2e_sweep2.log; : > $out
for cfg in "2 262144" "3 262144" "4 131072" "4 262144" "4 196608"; do
  set -- $cfg
  echo "lanes=$1 chunk=$2" >> $out
  TMV_HOST_LANES=$1 TMV_HOST_CHUNK=$2 timeout -k 10 100 python tools/e2e_probe.py 2>/dev/null | grep e2e >> $out
  TMV_HOST_LANES=$1 TMV_HOST_CHUNK=$2 timeout -k 10 200 python tools/km_bench.py 2>/dev/null | grep verifies >> $out
done
