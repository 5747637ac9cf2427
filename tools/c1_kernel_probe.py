#!/usr/bin/env python3
"""Median wall time of the C1-sized key-cached call (150 commit signatures,
tmv_verify_batch_ex with TMV_FLAG_KEY_CACHE: the fused latency kernel) and
of the full VerifyCommit call, for A/B of builds (development tool)."""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from tendermint_amd import _native as N  # noqa: E402
from tendermint_amd import host as H  # noqa: E402
from tendermint_amd.testing.factory import make_c1_commit, make_commit_batch  # noqa: E402

ctx = N.Context(1)
b = make_commit_batch(150)
for _ in range(5):
    ctx.verify_batch_ex(N.TMV_KIND_ED25519, N.TMV_FLAG_KEY_CACHE, b.pk, b.sig, b.msg, b.off)
ts = []
for _ in range(400):
    t = time.perf_counter()
    ok, st = ctx.verify_batch_ex(N.TMV_KIND_ED25519, N.TMV_FLAG_KEY_CACHE, b.pk, b.sig, b.msg, b.off)
    ts.append((time.perf_counter() - t) * 1e3)
vals, bid, commit = make_c1_commit(150)
call = H.PreparedCommitCall(ctx, H.MODE_FULL, "test_chain_id", vals, bid, 3, commit)
call()
tc = []
for _ in range(400):
    t = time.perf_counter()
    err = call()
    tc.append((time.perf_counter() - t) * 1e3)
print(json.dumps({"batch150_p50_ms": round(statistics.median(ts), 4), "all_valid": bool(ok),
                  "verify_commit_p50_ms": round(statistics.median(tc), 4), "commit_err": err is not None}))
