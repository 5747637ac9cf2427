#!/usr/bin/env python3
"""Key-cached large batches (commit traffic: few keys, many signatures)
through the host-buffer API: key-merged batch equation vs the key-cached
per-entry path vs the uncached batch equation.

  python tools/km_bench.py [--n 1000000] [--keys 2000] [--reps 5]
Prints one JSON line per method: median wall time per call (host staging +
H2D + kernels + D2H) and verifies/s.  Kernel-only time: run under
rocprofv3 --kernel-trace --stats.
"""
import argparse
import json
import os
import statistics
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from tendermint_amd import _native as N  # noqa: E402
from tendermint_amd.testing.factory import make_commit_batch  # noqa: E402

METHODS = {
    "key_merged": N.TMV_FLAG_KEY_CACHE | N.TMV_FLAG_BATCH_EQUATION,
    "cached_per_entry": N.TMV_FLAG_KEY_CACHE | N.TMV_FLAG_PER_ENTRY,
    "batch_equation": N.TMV_FLAG_BATCH_EQUATION,
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--keys", type=int, default=2000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--methods", default="key_merged,cached_per_entry,batch_equation")
    ap.add_argument("--group-log2", type=int, default=0, help="batch-equation group size (0 = engine default)")
    a = ap.parse_args()
    b = make_commit_batch(a.keys).tile(a.n)  # key i signs entry i mod keys
    ctx = N.Context(1)
    if a.group_log2:
        ctx.set_batch_options(group_log2=a.group_log2)
    for name in a.methods.split(","):
        flags = METHODS[name]
        ok, st = ctx.verify_batch_ex(N.TMV_KIND_ED25519, flags, b.pk, b.sig, b.msg, b.off)  # warm (key builds)
        assert ok, name
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            ok, st = ctx.verify_batch_ex(N.TMV_KIND_ED25519, flags, b.pk, b.sig, b.msg, b.off)
            ts.append(time.perf_counter() - t0)
            assert ok, name
        med = statistics.median(ts)
        print(json.dumps({"method": name, "n": a.n, "keys": a.keys, "call_ms": round(med * 1e3, 3),
                          "verifies_per_s_end_to_end": round(a.n / med)}), flush=True)


if __name__ == "__main__":
    main()
