#!/bin/bash
# Rehearsal of bench.py's --gpus N path on a one-GPU box: two ranks (both on
# GPU 0, gloo for the validity all-gather instead of RCCL, which refuses two
# ranks on one device), real kernels, extras on rank 0.
set -o pipefail
mkdir -p gpurun_out/n2
TMV_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 8 --warmup 4 --no-cpu-baseline \
  > gpurun_out/n2/bench.log 2>&1 || { tail -30 gpurun_out/n2/bench.log; exit 1; }
grep '^{' gpurun_out/n2/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('n_gpus','value','steps','ms_per_step')}, d['config']['parallelism'])"
