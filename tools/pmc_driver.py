#!/usr/bin/env python3
"""Minimal driver for PMC passes: only the bench's launches (32 C2 batches
per tmv_verify_batches_device call, batch equation), nothing else, so every
profiled dispatch belongs to one.  `--launches N` timed-equivalent launches
after 2 warm-up launches.  Used by tools/profile_round.sh."""
import argparse
import os
import sys
from concurrent.futures import ProcessPoolExecutor

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from tendermint_amd.testing.factory import make_c2_batch  # noqa: E402


def _gen(seed):
    return make_c2_batch(10_000, seed=seed)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--launches", type=int, default=4)
    ap.add_argument("--per-launch", type=int, default=32)
    ap.add_argument("--method", choices=["batch", "per-entry"], default="batch")
    a = ap.parse_args()
    with ProcessPoolExecutor(8) as ex:
        batches = list(ex.map(_gen, [0xED25519 + j for j in range(8)]))
    import torch
    from tendermint_amd import _native as N
    dev = torch.device("cuda:0")
    d_in = [(torch.from_numpy(b.pk).to(dev), torch.from_numpy(b.sig).to(dev), torch.from_numpy(b.msg).to(dev),
             torch.from_numpy(b.off.view(np.int32)).to(dev), int(b.off[-1] - b.off[0])) for b in batches]
    K = a.per_launch
    out = torch.zeros(K * 10_000, dtype=torch.int8, device=dev)
    refs = [N.BatchRef(d_in[j % 8][0].data_ptr(), d_in[j % 8][1].data_ptr(), d_in[j % 8][2].data_ptr(),
                       d_in[j % 8][3].data_ptr(), 10_000, d_in[j % 8][4], out[j * 10_000:].data_ptr())
            for j in range(K)]
    ctx = N.Context(1)
    flags = N.TMV_FLAG_BATCH_EQUATION if a.method == "batch" else N.TMV_FLAG_PER_ENTRY
    st = torch.cuda.Stream(dev)
    for _ in range(2 + a.launches):
        ctx.verify_batches_device(0, N.TMV_KIND_ED25519, flags, refs, st.cuda_stream)
    torch.cuda.synchronize()
    assert int((out == 1).sum().item()) == 9950 * K
    print("launches", 2 + a.launches)


if __name__ == "__main__":
    main()
