#!/bin/bash
# Build A/B variants of libtmgpu.so from the working tree, in parallel, each
# in its own object directory:  tools/build_ab.sh name="-DFLAG=1" name2="" ...
# -> tendermint_amd/_build/ab_<name>.so (input of tools/gpu_ab_so.sh).  Every
# variant is built with -DTMV_AB, so it also reads the A/B switches of
# tendermint_amd/csrc/knobs.h (TMV_KERNEL, TMV_MSM_CHUNK, ...), which the
# product library ignores.
set -e
cd "$(dirname "$0")/.."
pids=()
for nv in "$@"; do
  name=${nv%%=*}; flags=${nv#*=}
  ( make -s -j3 -C tendermint_amd/csrc OUT=../_build_ab_$name EXTRA="-DTMV_AB $flags" > /tmp/build_ab_$name.log 2>&1 &&
    cp tendermint_amd/_build_ab_$name/libtmgpu.so tendermint_amd/_build/ab_$name.so && echo "built ab_$name.so" ) &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=1; done
exit $rc
