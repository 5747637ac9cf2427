#!/bin/bash
# Test build of libtmgpu.so with -DTMV_CHECKS (device-side join / bucket
# counters, tmv_internal_checks) -> tendermint_amd/_build_checks/libtmgpu.so,
# loaded by tests/test_gpu_checks.py through TMV_LIB_PATH in a subprocess.
# __graft_entry__.build() runs this too, so the library ships to the GPU box.
set -e
cd "$(dirname "$0")/.."
make -s -j8 -C tendermint_amd/csrc OUT=../_build_checks EXTRA="-DTMV_CHECKS"
