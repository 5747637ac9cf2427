#!/bin/bash
# Round-end style check: whole GPU suite, smoke(), the driver-shaped bench and the default bench.
set -o pipefail
out=gpurun_out/round
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $out/tests.log 2>&1 \
  || { tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $out/bench_s20.log 2>&1 || { tail -20 $out/bench_s20.log; exit 1; }
grep '^{' $out/bench_s20.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('s20', d['value'], d['roofline']['frac'], d['cpu_baseline']['value'] if d['cpu_baseline'] else None, d.get('verify_commit_150_p50_ms'))"
timeout -k 10 400 python -u bench.py > $out/bench_default.log 2>&1 || { tail -20 $out/bench_default.log; exit 1; }
grep '^{' $out/bench_default.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('default', d['steps'], d['value'], d['roofline']['frac'], d.get('batch_latency_ms'), d.get('end_to_end_verifies_per_s'), d.get('end_to_end_vs_same_call_kernels'))"
