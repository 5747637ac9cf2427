#!/usr/bin/env python3
"""Host-layer timing of tmv_verify_commits on the CPU (no GPU): the product's
tm_host_abi.cpp linked against the test double of the engine
(tests/native/commit_check.cpp, libcommitcheck.so) with hashing skipped, on
C4-shaped windows (blocksync: light + full check per block).  Prints the
phase times (TMV_HOST_TIMING) and the wall time per window.

  TMV_HOST_TIMING=1 python tools/host_layer_timing.py [--blocks 1200]
"""
import argparse
import ctypes
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
from tendermint_amd import host as H  # noqa: E402
from tendermint_amd.testing import factory as Fa  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--blocks", type=int, default=602)
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()
L = ctypes.CDLL(os.path.join(REPO, "oracle", "_build", "libcommitcheck.so"))
L.commitcheck_verify_commits.argtypes = [ctypes.POINTER(H.CCommitJob), ctypes.c_uint32,
                                         ctypes.POINTER(ctypes.c_int32), ctypes.c_char_p, ctypes.c_size_t]
ctypes.c_int.in_dll(L, "g_skip_hash").value = 1
vals, blocks = Fa.make_block_chain(a.blocks, 175)
jobs = []
for i in range(1, len(blocks) - 1):
    f = blocks[i]
    jobs.append(H.CommitJob(H.MODE_LIGHT, "test_chain_id", vals, f.block_id, f.height, blocks[i + 1].last_commit))
    jobs.append(H.CommitJob(H.MODE_FULL, "test_chain_id", vals, blocks[i - 1].block_id, f.height - 1, f.last_commit))
pj = H.PreparedJobs(jobs)
ts = []
for _ in range(a.reps):
    t = time.perf_counter()
    L.commitcheck_verify_commits(pj.arr, pj.n, pj.results, pj.errs, pj.stride)
    ts.append(time.perf_counter() - t)
print(f"{len(jobs)} jobs, {len(blocks) - 2} blocks: best {min(ts) * 1e3:.2f} ms per window", flush=True)
