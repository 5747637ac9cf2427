#!/usr/bin/env python3
"""C2 throughput with several independent 10k batches in flight on separate
streams (one workspace per stream) vs one at a time."""
import json, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np
import torch
from tendermint_amd import _native as N
from tendermint_amd.testing.factory import make_c2_batch

ctx = N.Context(1)
dev = torch.device("cuda:0")
b = make_c2_batch(10_000)
t = lambda x: torch.from_numpy(x).to(dev)
pk, sig, msg, off = t(b.pk), t(b.sig), t(b.msg), t(b.off.view(np.int32))
for k in [int(x) for x in os.environ.get("INFLIGHT", "1,2,3,4").split(",")]:
    streams = [torch.cuda.Stream(dev) for _ in range(k)]
    outs = [torch.zeros(b.n, dtype=torch.uint8, device=dev) for _ in range(k)]
    steps = 60
    def run(nsteps):
        for i in range(nsteps):
            s = streams[i % k]
            ctx.ed25519_verify_batch_device(0, pk.data_ptr(), sig.data_ptr(), msg.data_ptr(), off.data_ptr(), b.n,
                                            outs[i % k].data_ptr(), s.cuda_stream)
    run(2 * k); torch.cuda.synchronize()
    t0 = time.perf_counter(); run(steps); torch.cuda.synchronize(); dt = time.perf_counter() - t0
    ok = all(int((o == 1).sum()) == int(outs[0].sum()) for o in outs)
    print(json.dumps({"inflight": k, "ms_per_batch": round(dt / steps * 1e3, 4),
                      "verifies_per_s": round(steps * b.n / dt), "consistent": ok}), flush=True)
