#!/usr/bin/env python3
"""Throughput / latency sweep of the batch equation vs per-entry
verification on device-resident batches (one MI355X).

  python tools/msm_sweep.py [--n 10000] [--kind c2|honest] [--tile N]
Prints one JSON line per configuration: method, group_log2, window, inflight,
verifies/s over the timed launches and the single-launch latency.
"""
import argparse
import json
import os
import statistics
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from tendermint_amd import _native as N  # noqa: E402
from tendermint_amd.testing.factory import make_c2_batch, make_commit_batch  # noqa: E402


def run(ctx, d, n, flags, F, steps, kind=N.TMV_KIND_ED25519):
    dev = d["pk"].device
    outs = [torch.zeros(n, dtype=torch.int8, device=dev) for _ in range(F)]
    streams = [torch.cuda.Stream(dev) for _ in range(F)]

    def launch(i):
        ctx.verify_batch_device_ex(0, kind, flags, 0, d["pk"].data_ptr(), d["sig"].data_ptr(), d["msg"].data_ptr(),
                                   d["off"].data_ptr(), n, outs[i % F].data_ptr(), streams[i % F].cuda_stream)
    for i in range(2 * F):
        launch(i)
    torch.cuda.synchronize()
    # latency: one at a time
    lat = []
    for _ in range(5):
        t0 = time.perf_counter()
        launch(0)
        torch.cuda.synchronize()
        lat.append(time.perf_counter() - t0)
    t0 = time.perf_counter()
    for i in range(steps):
        launch(i)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    return n * steps / el, statistics.median(lat) * 1e3, int((outs[0] == 1).sum().item())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10_000)
    ap.add_argument("--kind", default="c2")
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--configs", default="pe:0:0:1,pe:0:0:8,b:6:0:1,b:6:0:8,b:5:0:8,b:7:0:8,b:8:0:8,b:10:0:8")
    args = ap.parse_args()
    base = make_c2_batch(10_000) if args.kind == "c2" else make_commit_batch(2000)
    b = base.tile(args.n) if args.n != base.n else base
    dev = torch.device("cuda:0")
    d = {"pk": torch.from_numpy(b.pk).to(dev), "sig": torch.from_numpy(b.sig).to(dev),
         "msg": torch.from_numpy(b.msg).to(dev), "off": torch.from_numpy(b.off.view(np.int32)).to(dev)}
    ctx = N.Context(1)
    for cfg in args.configs.split(","):
        meth, mlog, c, F = cfg.split(":")
        mlog, c, F = int(mlog), int(c), int(F)
        ctx.set_batch_options(group_log2=mlog, window_bits=c)
        flags = N.TMV_FLAG_BATCH_EQUATION if meth == "b" else N.TMV_FLAG_PER_ENTRY
        steps = max(F, args.steps if args.n <= 20000 else max(F, args.steps // 10))
        rate, lat_ms, valid = run(ctx, d, b.n, flags, F, steps)
        print(json.dumps({"n": b.n, "kind": args.kind, "method": meth, "group_log2": mlog, "window": c,
                          "inflight": F, "verifies_per_s": round(rate), "latency_ms": round(lat_ms, 3),
                          "valid": valid}), flush=True)


if __name__ == "__main__":
    main()
