#!/usr/bin/env python3
"""Probe: does a per-entry slice on a second stream, started late, fill the
latency-bound tail of a lone batch-equation launch?

A 125k launch (the 8-GPU shard of the 1M north-star batch) is ~1.0 ms of
throughput kernels and ~0.6 ms of chains that leave most SIMDs idle
(running sums, Horner, fallback).  Here the batch equation verifies entries
[0, n - X) on stream 1 while stream 2 sleeps D us (torch.cuda._sleep, one
wave) and then verifies [n - X, n) per entry.  Prints one JSON line per
(X, D): the joint span (HIP events), next to the two parts alone.

  python tools/tail_fill_probe.py --n 125000 --x 0,16000,24000,32000 --delay-us 0,300,500,700
"""
import argparse
import json
import os
import statistics
import sys
from concurrent.futures import ProcessPoolExecutor

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from tendermint_amd.testing.factory import Batch, C2_VALID_KINDS, make_c2_batch  # noqa: E402


def _c2(seed):
    return make_c2_batch(10_000, seed=seed)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=125_000)
    ap.add_argument("--x", default="0,16000,24000,32000")
    ap.add_argument("--delay-us", default="0,300,500,700")
    ap.add_argument("--reps", type=int, default=9)
    a = ap.parse_args()
    with ProcessPoolExecutor(8) as ex:
        base = list(ex.map(_c2, [0xED25519 + j for j in range(13)]))
    import torch
    from tendermint_amd import _native as N
    dev = torch.device("cuda", 0)
    ctx = N.Context(1)
    n = a.n
    hb = Batch.concat([base[j % len(base)] for j in range(-(-n // 10_000))]).take(np.arange(n))
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)  # noqa: E731
    pk, sig, msg, off = t(hb.pk), t(hb.sig), t(hb.msg), t(hb.off.view(np.int32))
    want = torch.tensor([k in C2_VALID_KINDS for k in hb.kinds], dtype=torch.int8, device=dev)
    out = torch.zeros(n, dtype=torch.int8, device=dev)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    def part(lo, hi, flags, st):
        ctx.verify_batch_device_ex(0, N.TMV_KIND_ED25519, flags, 0, pk.data_ptr() + 32 * lo, sig.data_ptr() + 64 * lo,
                                   msg.data_ptr(), off.data_ptr() + 4 * lo, hi - lo, out.data_ptr() + lo,
                                   st.cuda_stream)

    # _sleep(cycles) calibration: one wave spinning
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(s2):
        torch.cuda._sleep(1000)
        torch.cuda.synchronize()
        e0.record(s2)
        torch.cuda._sleep(1_000_000)
        e1.record(s2)
    torch.cuda.synchronize()
    cyc_per_us = 1_000_000 / (e0.elapsed_time(e1) * 1e3)
    print(json.dumps({"sleep_cycles_per_us": round(cyc_per_us, 2)}), flush=True)

    def timed(fn):
        lat = []
        for r in range(2 + a.reps):
            out.zero_()
            torch.cuda.synchronize()
            b0, b1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            b0.record(s1)
            s2.wait_event(b0)
            fn()
            s1.wait_stream(s2)
            b1.record(s1)
            torch.cuda.synchronize()
            if r >= 2:
                lat.append(b0.elapsed_time(b1))
        return round(statistics.median(lat), 4), round(min(lat), 4)

    B, P = N.TMV_FLAG_BATCH_EQUATION, N.TMV_FLAG_PER_ENTRY
    for x in [int(v) for v in a.x.split(",")]:
        lo = n - x
        res = {"n": n, "x": x}
        res["batch_part_alone"] = timed(lambda: part(0, lo, B, s1))
        if x:
            res["per_entry_part_alone"] = timed(lambda: part(lo, n, P, s2))
        for d in [int(v) for v in a.delay_us.split(",")]:
            if not x and d:
                continue

            def both():
                part(0, lo, B, s1)
                if x:
                    with torch.cuda.stream(s2):
                        if d:
                            torch.cuda._sleep(int(d * cyc_per_us))
                    part(lo, n, P, s2)
            res[f"joint_d{d}"] = timed(both)
            res[f"exact_d{d}"] = bool(torch.equal(out, want))
        print(json.dumps(res), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
