cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_msm1 -o c2 -- python3 tools/msm_sweep.py --n 10000 --kind c2 --configs b:6:0:1 --steps 10 > gpurun_out/prof_msm1.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_msm2 -o h1m -- python3 tools/msm_sweep.py --n 1000000 --kind honest --configs b:10:0:1 --steps 10 > gpurun_out/prof_msm2.log 2>&1
