#!/bin/bash
# A/B two builds of libtmgpu.so in one GPU call (tendermint_amd/_build/ab_old.so
# vs ab_new.so, copied over libtmgpu.so in turn); restores ab_new.so.
set -o pipefail
B=tendermint_amd/_build
run() {
  timeout -k 10 200 python -u bench.py "$@" --warmup 5 --no-extras --no-cpu-baseline > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
  grep '^{' gpurun_out/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,2), 'M/s', round(d['ms_per_step']*d['steps'],3), 'ms')"
}
for rep in 1 2 3; do
  for v in old new; do
    cp $B/ab_$v.so $B/libtmgpu.so
    echo -n "$v s20: "; run --steps 20
  done
done
for v in old new; do
  cp $B/ab_$v.so $B/libtmgpu.so
  echo -n "$v s48: "; run --steps 48
done
cp $B/ab_new.so $B/libtmgpu.so
