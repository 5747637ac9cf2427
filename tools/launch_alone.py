#!/usr/bin/env python3
"""One C2-shaped launch of n signatures alone on the GPU, repeated (device-
resident inputs, one launch at a time, HIP events), for rocprofv3 kernel
traces of a single launch's critical path (the 1/N
shard of the 1M north-star batch is a 125k launch at 8 GPUs).

  python tools/launch_alone.py --n 125000,250000,500000,1000000 --reps 10
Prints one JSON line per size: median / min ms and verifies/s.
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
    ap.add_argument("--n", default="125000")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--distinct", type=int, default=16, help="distinct C2 batches, tiled")
    ap.add_argument("--method", default="batch", choices=["batch", "per-entry", "auto"])
    ap.add_argument("--group-log2", type=int, default=0, help="batch-equation group size 2^k (0: the library's choice)")
    ap.add_argument("--window-bits", type=int, default=0, help="batch-equation window bits c (0: the library's choice)")
    ap.add_argument("--stats", action="store_true", help="also count the launch's groups / failing groups / fallback "
                                                         "entries (one extra host-buffer call)")
    ap.add_argument("--kind", default="ed25519", choices=["ed25519", "mixed", "mixed-ed", "mixed-sr"],
                    help="mixed-ed / mixed-sr: one kind's entries of the C5 base alone (pure-kind launch)")
    a = ap.parse_args()
    sizes = [int(x) for x in a.n.split(",")]
    with ProcessPoolExecutor(8) as ex:
        base = list(ex.map(_c2, [0xED25519 + j for j in range(a.distinct)]))
    kind_arr = None
    if a.kind == "mixed":
        from tendermint_amd.testing.factory import make_mixed_batch
        kind_arr, mb = make_mixed_batch(20_000)
        base = [mb]
    elif a.kind in ("mixed-ed", "mixed-sr"):
        from tendermint_amd.testing.factory import make_mixed_batch
        karr, mb = make_mixed_batch(20_000)
        base = [mb.take(np.flatnonzero(karr == (1 if a.kind == "mixed-sr" else 0)))]
    import torch
    from tendermint_amd import _native as N
    dev = torch.device("cuda", 0)
    ctx = N.Context(1)
    if a.group_log2 or a.window_bits:
        ctx.set_batch_options(group_log2=a.group_log2, window_bits=a.window_bits)
    flags = {"batch": N.TMV_FLAG_BATCH_EQUATION, "per-entry": N.TMV_FLAG_PER_ENTRY, "auto": 0}[a.method]
    st = torch.cuda.Stream(dev)
    for n in sizes:
        per = base[0].n
        hb = Batch.concat([base[j % len(base)] for j in range(-(-n // per))]).take(np.arange(n))
        t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)  # noqa: E731
        d = [t(hb.pk), t(hb.sig), t(hb.msg), t(hb.off.view(np.int32))]
        dk = t(np.tile(kind_arr, -(-n // len(kind_arr)))[:n]) if kind_arr is not None else None
        out = torch.zeros(n, dtype=torch.int8, device=dev)
        kk = (N.TMV_KIND_MIXED if dk is not None
              else N.TMV_KIND_SR25519 if a.kind == "mixed-sr" else N.TMV_KIND_ED25519)
        lat = []
        for r in range(a.warmup + a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            ctx.verify_batch_device_ex(0, kk, flags, dk.data_ptr() if dk is not None else 0, d[0].data_ptr(),
                                       d[1].data_ptr(), d[2].data_ptr(), d[3].data_ptr(), n, out.data_ptr(),
                                       st.cuda_stream)
            e1.record(st)
            torch.cuda.synchronize(dev)
            if r >= a.warmup:
                lat.append(e0.elapsed_time(e1))
        line = {"n": n, "method": a.method, "kind": a.kind, "ms_median": round(statistics.median(lat), 4),
                "ms_min": round(min(lat), 4), "verifies_per_s": round(n / statistics.median(lat) * 1e3, 1)}
        if a.kind == "ed25519":
            want = np.array([k in C2_VALID_KINDS for k in hb.kinds], np.int8)
            line["exact"] = bool(np.array_equal(out.cpu().numpy(), want))
        if a.stats and kk == N.TMV_KIND_ED25519 and a.method == "batch":
            # the same batch once through the host C-ABI with group verdicts
            # counted (the device-pointer calls keep no statistics): groups,
            # failing groups, entries verified one by one
            ctx.set_batch_options(group_log2=a.group_log2, window_bits=a.window_bits, stats=True)
            g0, m0 = ctx.batch_stats(), ctx.metrics()
            ctx.verify_batch_ex(N.TMV_KIND_ED25519, flags, hb.pk, hb.sig, hb.msg, hb.off)
            g1, m1 = ctx.batch_stats(), ctx.metrics()
            ctx.set_batch_options(group_log2=a.group_log2, window_bits=a.window_bits)
            line["groups"] = g1["groups"] - g0["groups"]
            line["groups_failed"] = g1["failed"] - g0["failed"]
            line["fallback_signatures"] = m1["fallback_signatures"] - m0["fallback_signatures"]
            line["located_groups"] = m1["located_groups"] - m0["located_groups"]
        print(json.dumps(line), flush=True)
        del d, out
    ctx.close()


if __name__ == "__main__":
    main()
