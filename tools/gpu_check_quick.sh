#!/bin/bash
# Batch-equation / host-pipeline GPU tests, then the driver-shaped bench line.
set -o pipefail
out=gpurun_out/quick
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_batch_equation.py \
  tests/test_gpu_ed25519.py tests/test_gpu_host_pipeline.py tests/test_gpu_key_merged.py tests/test_gpu_sr25519.py \
  > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
grep '^{' $out/bench.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']
print({k: d.get(k) for k in ('value','launch_alone_ms','batch_latency_ms','end_to_end_verifies_per_s','end_to_end_vs_same_call_kernels','verify_commit_150_p50_ms')})
print('frac', r['frac'], 'executed_frac', r.get('executed_frac'))
print(json.dumps(r.get('dominant_kernel')))"
