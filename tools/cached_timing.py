"""Timing of the key-cached path on validator-style workloads (development
tool): V distinct validator keys, N signatures, host-buffer API (PCIe
included) and the C1 VerifyCommit latency."""
import json, os, sys, time, statistics
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np
from tendermint_amd import _native as N, host as H
from tendermint_amd.testing.factory import Batch, make_commit_batch, make_c1_commit

ctx = N.Context(1)
for vals, n in [(150, 150), (175, 175 * 100), (175, 175 * 1000), (100, 100 * 2000)]:
    base = make_commit_batch(vals, seed=3)
    b = base.tile(n)
    for flags in (0, N.TMV_FLAG_KEY_CACHE):
        ctx.verify_batch_ex(N.TMV_KIND_ED25519, flags, b.pk, b.sig, b.msg, b.off)  # warm (builds keys)
        ts = []
        for _ in range(5):
            t = time.perf_counter()
            ok, st = ctx.verify_batch_ex(N.TMV_KIND_ED25519, flags, b.pk, b.sig, b.msg, b.off)
            ts.append(time.perf_counter() - t)
            assert ok
        m = statistics.median(ts)
        print(json.dumps({"validators": vals, "n": n, "cache": bool(flags), "ms": round(m * 1e3, 3),
                          "verifies_per_s_e2e": round(n / m)}))
vals, bid, commit = make_c1_commit(150)
call = H.PreparedCommitCall(ctx, H.MODE_FULL, "test_chain_id", vals, bid, 3, commit)
assert call() is None
lat = []
for _ in range(300):
    t = time.perf_counter(); assert call() is None; lat.append((time.perf_counter() - t) * 1e3)
lat.sort()
print(json.dumps({"verify_commit_150_p50_ms": round(lat[150], 4), "p99": round(lat[296], 4)}))
print(json.dumps(ctx.key_cache_stats()))
