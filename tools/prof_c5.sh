cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/prof_c5
timeout -k 10 300 python3 $R/tools/bench_configs.py --only 5 > $R/gpurun_out/c5.log 2>&1 || exit 1
for m in "per-entry" "batch m=64"; do
  tag=$(echo $m | tr -d ' =')
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c5 -o c5_$tag -- python3 $R/tools/bench_configs.py --only 5 --c5-methods "$m" > $R/gpurun_out/prof_c5/$tag.log 2>&1 || exit 1
done
