set -e
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_accum.log 2>&1
timeout -k 10 300 python bench.py --steps 384 --warmup 16 > gpurun_out/bench_accum.log 2>&1
bash tools/e2e_sweep.sh
