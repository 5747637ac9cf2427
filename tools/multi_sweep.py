#!/usr/bin/env python3
"""Sweep of multi-batch launches (tmv_verify_batches_device) on one MI355X:
batches per launch K, launches in flight F, method and group size, over 8
distinct C2 batches reused cyclically.  One JSON line per configuration.

  python tools/multi_sweep.py --configs b:6:8:2,b:6:16:2,pe:0:8:2 [--repeat 3]
config = method(b|pe):group_log2:K:F[:window]
"""
import argparse
import json
import os
import statistics
import sys
import time
from concurrent.futures import ProcessPoolExecutor

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from tendermint_amd import _native as N  # noqa: E402
from tendermint_amd.testing.factory import make_c2_batch  # noqa: E402


def _gen(seed):
    return make_c2_batch(10_000, seed=seed)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="pe:0:8:2,b:6:8:2,b:6:16:2,b:6:32:2,b:6:16:4,b:5:16:2,b:7:16:2")
    ap.add_argument("--launches", type=int, default=12)
    ap.add_argument("--repeat", type=int, default=3)
    args = ap.parse_args()
    with ProcessPoolExecutor(8) as ex:
        batches = list(ex.map(_gen, [0xED25519 + j for j in range(8)]))
    dev = torch.device("cuda:0")
    d_in = [(torch.from_numpy(b.pk).to(dev), torch.from_numpy(b.sig).to(dev), torch.from_numpy(b.msg).to(dev),
             torch.from_numpy(b.off.view(np.int32)).to(dev), int(b.off[-1] - b.off[0]), b.n) for b in batches]
    ctx = N.Context(1)
    for cfg in args.configs.split(","):
        parts = cfg.split(":")
        meth, mlog, K, F = parts[0], int(parts[1]), int(parts[2]), int(parts[3])
        win = int(parts[4]) if len(parts) > 4 else 0
        ctx.set_batch_options(group_log2=mlog, window_bits=win)
        flags = N.TMV_FLAG_BATCH_EQUATION if meth == "b" else N.TMV_FLAG_PER_ENTRY
        outs = [[torch.zeros(10_000, dtype=torch.int8, device=dev) for _ in range(K)] for _ in range(F)]
        refs = [[N.BatchRef(d_in[j % 8][0].data_ptr(), d_in[j % 8][1].data_ptr(), d_in[j % 8][2].data_ptr(),
                            d_in[j % 8][3].data_ptr(), d_in[j % 8][5], d_in[j % 8][4], outs[f][j].data_ptr())
                 for j in range(K)] for f in range(F)]
        streams = [torch.cuda.Stream(dev) for _ in range(F)]

        def launch(i):
            ctx.verify_batches_device(0, N.TMV_KIND_ED25519, flags, refs[i % F], streams[i % F].cuda_stream)
        for i in range(2 * F):
            launch(i)
        torch.cuda.synchronize()
        rates = []
        for _ in range(args.repeat):
            t0 = time.perf_counter()
            for i in range(args.launches):
                launch(i)
            torch.cuda.synchronize()
            rates.append(10_000 * K * args.launches / (time.perf_counter() - t0))
        ok = all(int((o == 1).sum().item()) == 9950 for row in outs for o in row)
        print(json.dumps({"method": meth, "group_log2": mlog, "window": win, "K": K, "F": F,
                          "verifies_per_s": round(statistics.median(rates)), "spread": round(max(rates) / min(rates), 3),
                          "valid_ok": ok}), flush=True)


if __name__ == "__main__":
    main()
