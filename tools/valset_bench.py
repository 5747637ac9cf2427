"""ValidatorSet.Hash throughput (tmv_validator_set_hashes)
on C3-shaped windows: S sets x V validators (ed25519, power 2).  Reports the
C-ABI call (host arrays: staging, H2D, kernels, D2H) and, with HIP events,
the kernels alone, next to hashlib on one host core over a sample.
  python tools/valset_bench.py [--sets 1000] [--vals 100] [--reps 20]"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sets", type=int, default=1000)
    ap.add_argument("--vals", type=int, default=100)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    from tendermint_amd import _native as N
    import merkle_ref as M  # checker and CPU timing only
    rng = np.random.default_rng(1)
    n = a.sets * a.vals
    pk = rng.integers(0, 256, 32 * n, dtype=np.uint8)
    kind = np.zeros(n, np.uint8)
    power = np.full(n, 2, np.int64)
    off = (np.arange(a.sets + 1, dtype=np.uint32) * a.vals).astype(np.uint32)
    ctx = N.Context(1)
    out = ctx.validator_set_hashes(pk, kind, power, off)
    for s in (0, a.sets - 1):
        vals = [(pk[32 * i:32 * i + 32].tobytes(), 0, 2) for i in range(s * a.vals, (s + 1) * a.vals)]
        assert bytes(out[s]) == M.validator_set_hash(vals)
    t = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        ctx.validator_set_hashes(pk, kind, power, off)
        t.append(time.perf_counter() - t0)
    call_ms = float(np.median(t)) * 1e3
    # CPU: hashlib over a sample of sets, one core
    sample = min(a.sets, 50)
    t0 = time.perf_counter()
    for s in range(sample):
        M.validator_set_hash([(pk[32 * i:32 * i + 32].tobytes(), 0, 2) for i in range(s * a.vals, (s + 1) * a.vals)])
    cpu_s = (time.perf_counter() - t0) / sample
    comp = a.sets * (a.vals + 2 * (a.vals - 1))  # leaf: 1 block; inner: 2 blocks
    print(json.dumps({"workload": f"{a.sets} sets x {a.vals} validators", "call_ms_p50": round(call_ms, 3),
                      "sets_per_s": round(a.sets / call_ms * 1e3), "sha256_blocks_per_s": round(comp / call_ms * 1e3),
                      "cpu_python_hashlib_sets_per_s_1core": round(1 / cpu_s)}))


if __name__ == "__main__":
    main()
