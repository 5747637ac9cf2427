"""End-to-end (host buffers: pinned staging + PCIe + kernels + D2H) rate of
the bench's 640k-signature C2 call (64 batches; TMV_E2E_NB) under the current TMV_* environment
(development tool).  The batch is generated once and cached in /tmp, so a
shell loop can A/B runtime knobs in separate processes:

  for l in 2 4; do TMV_HOST_LANES=$l python tools/e2e_probe.py; done
"""
import json, os, statistics, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from concurrent.futures import ProcessPoolExecutor
import numpy as np

CACHE = "/tmp/tmv_e2e_c2x64.npz"
NB = 64
# TMV_E2E_NB: batches per call (the 64 distinct batches repeated)
NBC = int(os.environ.get("TMV_E2E_NB", "64"))


def _c2(seed):
    from tendermint_amd.testing.factory import make_c2_batch
    b = make_c2_batch(10_000, seed=seed)
    return b.pk, b.sig, b.msg, b.off


def main():
    if not os.path.exists(CACHE):
        with ProcessPoolExecutor(8) as ex:
            parts = list(ex.map(_c2, [0xED25519 + j for j in range(NB)]))
        from tendermint_amd.testing.factory import Batch
        hb = Batch.concat([Batch(pk, sig, msg, off) for pk, sig, msg, off in parts])
        np.savez(CACHE, pk=hb.pk, sig=hb.sig, msg=hb.msg, off=hb.off)
    z = np.load(CACHE)
    pk, sig, msg, off = z["pk"], z["sig"], z["msg"], z["off"]
    if NBC != NB:
        from tendermint_amd.testing.factory import Batch
        one = Batch(pk, sig, msg, off)
        hb = Batch.concat([one] * (NBC // NB))
        pk, sig, msg, off = hb.pk, hb.sig, hb.msg, hb.off
    from tendermint_amd import _native as N
    # TMV_E2E_TORCH_STREAMS=K: K torch streams, each used once, before the
    # engine's lanes create theirs (bench.py's order: its in-flight streams
    # first) -- do they share the device's hardware queues with the lanes?
    ks = int(os.environ.get("TMV_E2E_TORCH_STREAMS", "0"))
    keep = []
    if ks:
        import torch
        for _ in range(ks):
            st = torch.cuda.Stream()
            with torch.cuda.stream(st):
                keep.append(torch.ones(1024, device="cuda") * 2)
            keep.append(st)
        torch.cuda.synchronize()
    ctx = N.Context(1)
    flags = N.TMV_FLAG_BATCH_EQUATION
    n = len(off) - 1
    ts, calls_ns = [], []
    for i in range(9):
        t, t_ns = time.perf_counter(), time.monotonic_ns()
        ok, st = ctx.verify_batch_ex(N.TMV_KIND_ED25519, flags, pk, sig, msg, off)
        ts.append(time.perf_counter() - t)
        calls_ns.append([t_ns, time.monotonic_ns()])
        assert int((st == 1).sum()) == (len(off) - 1) // 10_000 * 9950
    m = statistics.median(ts[2:])
    env = {k: v for k, v in os.environ.items() if k.startswith("TMV_")}
    h2d = pk.nbytes + sig.nbytes + msg.nbytes + off.nbytes
    line = {"env": env, "n": n, "median_ms": round(m * 1e3, 3), "e2e_verifies_per_s": round(n / m),
            "h2d_GBps": round(h2d / m / 1e9, 2), "calls_monotonic_ns": calls_ns}
    # TMV_E2E_CALLERS=C: C threads, each calling 4 times on its own copy of
    # the batch (each call claims its own lanes)
    callers = int(os.environ.get("TMV_E2E_CALLERS", "1"))
    if callers > 1:
        from concurrent.futures import ThreadPoolExecutor
        copies = [(pk, sig, msg, off)] + [(pk.copy(), sig.copy(), msg.copy(), off.copy()) for _ in range(callers - 1)]

        def caller(b, calls=4):
            for _ in range(calls):
                _, st = ctx.verify_batch_ex(N.TMV_KIND_ED25519, flags, *b)
                assert int((st == 1).sum()) == n // 10_000 * 9950

        with ThreadPoolExecutor(callers) as ex:
            list(ex.map(lambda b: caller(b, 1), copies))
            t = time.perf_counter()
            list(ex.map(caller, copies))
            dt = time.perf_counter() - t
        line.update({"callers": callers, "callers_verifies_per_s": round(4 * callers * n / dt),
                     "callers_h2d_GBps": round(4 * callers * h2d / dt / 1e9, 2)})
    line["metrics"] = ctx.metrics()
    print(json.dumps(line))


if __name__ == "__main__":
    main()
