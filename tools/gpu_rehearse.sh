#!/bin/bash
# SCALE-run rehearsal on a one-GPU box: bench.py --gpus N under
# torch.distributed.run with every rank on GPU 0 (gloo for the gathers: RCCL
# refuses two ranks on one device), real kernels, the driver's step counts.
# Times the whole command (the driver allows 600 s) and keeps the JSON line,
# whose run_timing carries the setup time and device memory (max over ranks).
#   bash tools/gpu_rehearse.sh N [BATCHES_PER_STEP] [RESIDENT]  -> gpurun_out/rehearse_nN/
set -o pipefail
N=${1:-8}
K=${2:-32}
R=${3:-16}
out=gpurun_out/rehearse_n$N
mkdir -p "$out"
t0=$(date +%s.%N)
TMV_BENCH_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" \
  --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus "$N" --steps 20 --warmup 5 \
  --batches-per-step "$K" --resident "$R" > "$out/bench.log" 2>&1
rc=$?
t1=$(date +%s.%N)
wall=$(python3 -c "print(round($t1 - $t0, 1))")
echo "rc=$rc wall_s=$wall n=$N batches_per_step=$K resident=$R" | tee "$out/summary.txt"
[ $rc -eq 0 ] || { tail -40 "$out/bench.log"; exit $rc; }
grep '^{' "$out/bench.log" > "$out/bench.json"
python3 - "$out/bench.json" >> "$out/summary.txt" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("n_gpus", d["n_gpus"], "parallelism", d["config"]["parallelism"])
print("value (all ranks on ONE GPU: not a measurement)", d["value"], "ms_per_step", d["ms_per_step"])
print("run_timing", json.dumps(d.get("run_timing")))
for leg in ("strong_1m", "strong_1m_mixed"):
    s = d.get(leg)
    if s:
        print(leg, "shards", s["shard_per_rank"], "kernel_only_ms", s["kernel_only"]["ms"], "end_to_end_ms",
              s["end_to_end"]["ms"], "exact", s["exact_vector_on_every_rank"])
EOF
cat "$out/summary.txt"
