#!/usr/bin/env python3
"""C5-shaped mixed ed25519 + sr25519 batch (a 20k base tiled to --n) end to
end from host buffers (tmv_verify_mixed_batch_ex: staging / the caller's
pages DMA'd, kernels, D2H) and kernel-only (device-resident inputs), median
of --reps, under the current TMV_* environment (A/B: run it in separate
processes, e.g. TMV_MIXED_STREAM=0).  The statuses are checked against the C
oracle once (checker role).  One JSON line.

  python tools/mixed_e2e.py --n 1000000 --reps 7
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
sys.path.insert(0, os.path.join(REPO, "oracle"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--group-log2", type=int, default=0, help="batch-equation group size 2^k (0: the library's)")
    ap.add_argument("--window-bits", type=int, default=0, help="window bits c (0: the library's)")
    a = ap.parse_args()
    from tendermint_amd.testing.factory import make_mixed_batch
    import oracle_c as C  # checker only
    kind, base = make_mixed_batch(20_000, seed=0xC5)
    ed, sr = np.flatnonzero(kind == 0), np.flatnonzero(kind == 1)
    want1 = np.zeros(base.n, np.int8)
    be, bs = base.take(ed), base.take(sr)
    want1[ed] = C.ed25519_verify_packed(be.pk, be.sig, be.msg, be.off, threads=16)[1]
    want1[sr] = C.sr25519_status_packed(bs.pk, bs.sig, bs.msg, bs.off, threads=16)
    idx = np.arange(a.n) % base.n
    hb = base.take(idx)
    kinds = np.ascontiguousarray(kind[idx])
    want = want1[idx]
    import torch
    from tendermint_amd import _native as N
    dev = torch.device("cuda", 0)
    keep = []
    for _ in range(int(os.environ.get("TMV_E2E_TORCH_STREAMS", "0"))):  # see tools/e2e_probe.py
        st = torch.cuda.Stream(dev)
        with torch.cuda.stream(st):
            keep.append(torch.ones(1024, device=dev) * 2)
        keep.append(st)
    torch.cuda.synchronize(dev)
    ctx = N.Context(1)
    if a.group_log2 or a.window_bits:
        ctx.set_batch_options(group_log2=a.group_log2, window_bits=a.window_bits)
    flags = N.TMV_FLAG_BATCH_EQUATION
    e2e, calls_ns = [], []
    for r in range(a.reps + 2):
        t0, t0_ns = time.perf_counter(), time.monotonic_ns()
        _, st = ctx.verify_mixed_batch_ex(flags, kinds, hb.pk, hb.sig, hb.msg, hb.off)
        t1 = time.perf_counter()
        calls_ns.append([t0_ns, time.monotonic_ns()])
        if r == 0:
            bad = np.flatnonzero(np.asarray(st, np.int8) != want)
            assert not len(bad), f"end to end: entries {bad[:8]} differ from the oracle"
        if r >= 2:
            e2e.append((t1 - t0) * 1e3)
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)  # noqa: E731
    d = [t(kinds), t(hb.pk), t(hb.sig), t(hb.msg), t(hb.off.view(np.int32))]
    out = torch.zeros(a.n, dtype=torch.int8, device=dev)
    s = torch.cuda.Stream(dev)
    ker = []
    for r in range(a.reps + 2):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        ctx.verify_batch_device_ex(0, N.TMV_KIND_MIXED, flags, d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(),
                                   d[3].data_ptr(), d[4].data_ptr(), a.n, out.data_ptr(), s.cuda_stream)
        e1.record(s)
        torch.cuda.synchronize(dev)
        if r == 0:
            assert np.array_equal(out.cpu().numpy(), want), "kernel path differs from the oracle"
        if r >= 2:
            ker.append(e0.elapsed_time(e1))
    em, km = statistics.median(e2e), statistics.median(ker)
    print(json.dumps({"n": a.n, "env": {k: v for k, v in os.environ.items() if k.startswith("TMV_")},
                      "group_log2": a.group_log2, "window_bits": a.window_bits,
                      "end_to_end_ms": round(em, 3), "end_to_end_verifies_per_s": round(a.n / em * 1e3, 1),
                      "kernel_only_ms": round(km, 3), "kernel_only_verifies_per_s": round(a.n / km * 1e3, 1),
                      "e2e_reps_ms": [round(x, 3) for x in e2e], "exact_vs_oracle": True,
                      "calls_monotonic_ns": calls_ns}), flush=True)


if __name__ == "__main__":
    main()
