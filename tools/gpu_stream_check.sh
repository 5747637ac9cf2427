#!/bin/bash
# Streamed host path: GPU tests of the host pipeline, then an e2e sweep of the
# part sizes (tools/e2e_probe.py, one process per setting) and the bench line.
set -o pipefail
out=gpurun_out/stream
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_host_pipeline.py > $out/tests.log 2>&1 \
  || { tail -40 $out/tests.log; exit 1; }
TMV_STREAM_MODE=prep timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_host_pipeline.py > $out/tests_prep.log 2>&1 \
  || { tail -40 $out/tests_prep.log; exit 1; }
tail -1 $out/tests_prep.log
tail -1 $out/tests.log
for cfg in "TMV_STREAM=0" "TMV_STREAM_TWO=0" "TMV_STREAM_TWO=1" "TMV_STREAM_FIRST=16384 TMV_STREAM_PART=65536" "TMV_STREAM_FIRST=16384 TMV_STREAM_PART=32768" "TMV_STREAM_FIRST=32768 TMV_STREAM_PART=65536" "TMV_STREAM_TWO=0" "TMV_STREAM_TWO=1"; do
  echo -n "$cfg: "
  env $cfg timeout -k 10 120 python -u tools/e2e_probe.py 2>&1 | tail -1 || exit 1
done | tee $out/sweep.txt
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
grep '^{' $out/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ('value','launch_alone_ms','end_to_end_verifies_per_s','end_to_end_vs_same_call_kernels','end_to_end_h2d_GBps','verify_commit_150_p50_ms')}); print(d['roofline'].get('dominant_kernel'), d['roofline'].get('executed_frac'))"
