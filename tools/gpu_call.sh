#!/bin/bash
# One parameterised GPU call (replaces round 3's one-script-per-call
# gpu_r03_*.sh launchers).  Run on the box as
#   gpurun -- bash tools/gpu_call.sh NAME STEP [STEP ...]
# Every step runs under its own time limit, writes under gpurun_out/NAME/,
# and the call stops at the first step that fails (no GPU step after a
# failure, a fault or a time limit).  Steps (ARGS after the first ':'):
#   tests[:ARGS]        python -m pytest -m gpu ARGS (default: tests)
#   smoke               __graft_entry__.smoke()
#   bench[:ARGS]        bench.py ARGS                     -> bench_K.json
#   alone[:ARGS]        tools/launch_alone.py ARGS        -> alone_K.jsonl
#   trace[:ARGS]        rocprofv3 --kernel-trace --stats of tools/launch_alone.py ARGS -> trace_K/
#   tracebench[:ARGS]   rocprofv3 --kernel-trace --stats of bench.py ARGS     -> tracebench_K/
#   tracepy:SCRIPT ARGS rocprofv3 --kernel-trace --stats of python3 SCRIPT ARGS -> tracepy_K/
#   tracecp:SCRIPT ARGS the same with --memory-copy-trace (host-buffer timelines) -> tracecp_K/
#   configs[:ARGS]      tools/bench_configs.py ARGS       -> configs_K.log
#   py[:ARGS]           python -u ARGS                    -> py_K.log
#   bin:PATH [ARGS]     a built tool binary (e.g. tools/affine_bench) -> bin_K.log
# Optional per-step limit: STEP@SECONDS (default 600).  Optional per-step
# environment: [K=V,K2=V2]STEP (e.g. [TMV_MSM_PARTS=2]alone:--n 125000, or
# [TMV_LIB_PATH=tendermint_amd/_build/ab_x.so]alone:... for an A/B build).
set -o pipefail
name=$1; shift
out=gpurun_out/$name
mkdir -p "$out"
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
k=0
for step in "$@"; do
  k=$((k + 1))
  lim=600
  if [[ "$step" == *@* ]]; then lim=${step##*@}; step=${step%@*}; fi
  envs=""
  if [[ "$step" == \[* ]]; then envs=${step%%]*}; envs=${envs#[}; step=${step#*]}; fi
  kind=${step%%:*}
  args=""
  [[ "$step" == *:* ]] && args=${step#*:}
  echo "[gpu_call] step $k: ${envs:+[$envs] }$kind $args (limit ${lim}s)"
  saved_env=()
  IFS=',' read -ra kvs <<< "$envs"
  for kv in "${kvs[@]}"; do [ -n "$kv" ] && { saved_env+=("${kv%%=*}"); export "$kv"; }; done
  case $kind in
    tests)
      timeout -k 10 "$lim" python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu ${args:-tests} \
        > "$out/tests_$k.log" 2>&1; rc=$?; tail -5 "$out/tests_$k.log";;
    smoke)
      timeout -k 10 "$lim" python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke_$k.log" 2>&1; rc=$?
      cat "$out/smoke_$k.log";;
    bench)
      timeout -k 10 "$lim" python -u bench.py $args > "$out/bench_$k.json" 2> "$out/bench_$k.err"; rc=$?
      tail -c 600 "$out/bench_$k.json";;
    alone)
      timeout -k 10 "$lim" python -u tools/launch_alone.py $args > "$out/alone_$k.jsonl" 2> "$out/alone_$k.err"; rc=$?
      cat "$out/alone_$k.jsonl";;
    trace)
      timeout -k 10 "$lim" rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace_$k" -o run -- \
        python3 -u tools/launch_alone.py $args > "$out/trace_$k.log" 2>&1; rc=$?
      grep '^{' "$out/trace_$k.log";;
    tracebench)
      timeout -k 10 "$lim" rocprofv3 --kernel-trace --stats --output-format csv -d "$out/tracebench_$k" -o run -- \
        python3 -u bench.py $args > "$out/tracebench_$k.log" 2>&1; rc=$?
      grep '^{' "$out/tracebench_$k.log" | tail -c 400;;
    tracepy)
      timeout -k 10 "$lim" rocprofv3 --kernel-trace --stats --output-format csv -d "$out/tracepy_$k" -o run -- \
        python3 -u $args > "$out/tracepy_$k.log" 2>&1; rc=$?
      grep '^{' "$out/tracepy_$k.log" | tail -c 600;;
    tracecp)
      timeout -k 10 "$lim" rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv \
        -d "$out/tracecp_$k" -o run -- python3 -u $args > "$out/tracecp_$k.log" 2>&1; rc=$?
      grep '^{' "$out/tracecp_$k.log" | tail -c 600;;
    configs)
      timeout -k 10 "$lim" python -u tools/bench_configs.py $args > "$out/configs_$k.log" 2>&1; rc=$?
      cat "$out/configs_$k.log" | grep '^{';;
    py)
      timeout -k 10 "$lim" python -u $args > "$out/py_$k.log" 2>&1; rc=$?; tail -20 "$out/py_$k.log";;
    bin)
      timeout -k 10 "$lim" $args > "$out/bin_$k.log" 2>&1; rc=$?; tail -20 "$out/bin_$k.log";;
    *)
      echo "unknown step $kind"; exit 2;;
  esac
  for v in "${saved_env[@]}"; do unset "$v"; done
  if [ $rc -ne 0 ]; then echo "[gpu_call] step $k ($kind) failed rc=$rc"; exit $rc; fi
done
echo "[gpu_call] all $k steps ok"
