#!/bin/bash
# Round-3 GPU call ZE: launches in flight in the bench's timed region
# (--inflight 2 / 3 / 4 / 6 / 8), interleaved twice.
set -o pipefail
out=gpurun_out/r03ze
mkdir -p $out
for rep in 1 2; do
  for f in 4 2 3 6 8; do
    timeout -k 10 200 python -u bench.py --steps 20 --warmup 8 --inflight $f --no-extras --no-cpu-baseline > $out/b.json 2> $out/b.err || { tail -5 $out/b.err; exit 1; }
    python -c "import json; d=json.load(open('$out/b.json')); print('inflight $f rep$rep', round(d['value']/1e6,2), d['ms_per_step'])" >> $out/ab.txt
  done
done
cat $out/ab.txt
