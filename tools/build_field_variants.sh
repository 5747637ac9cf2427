#!/bin/bash
# Builds tendermint_amd/_build/ab_<name>.so for each field-arithmetic header
# given as name=path (e.g. old=/tmp/curve_old.h), restoring the working
# tree's curve25519.h and libtmgpu.so afterwards (A/B input for gpu_ab_so.sh).
set -e
H=tendermint_amd/csrc/curve25519.h
cp $H /tmp/curve_keep.h
for nv in "$@"; do
  name=${nv%%=*}; path=${nv#*=}
  cp "$path" $H
  make -s -B -C tendermint_amd/csrc 2>&1 | grep -v "loop not unrolled\|warnings generated\|^ *[0-9]* |\|^ *| *\^" || true
  cp tendermint_amd/_build/libtmgpu.so tendermint_amd/_build/ab_$name.so
  echo "built ab_$name.so"
done
cp /tmp/curve_keep.h $H
make -s -B -C tendermint_amd/csrc 2>&1 | grep -i " error" || true
