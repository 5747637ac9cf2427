"""Quick GPU sanity + timing run (development tool, not part of the product).

Checks libtmgpu.so against the C oracle on random honest / corrupted /
ZIP-215 small-order inputs, then times the kernel on device-resident batches.
"""
import os, sys, time, json, random
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
import numpy as np
import torch
import oracle_c as C
import ed25519_ref as E
import openssl_ed25519 as O
from tendermint_amd import _native as N

random.seed(7)
ctx = N.Context(0)
print("devices", ctx.num_devices(), N.lib().tmv_version().decode())

ent = []
for i in range(3000):
    sd = os.urandom(32); m = os.urandom(random.randint(0, 200)); s = O.sign(sd, m); pk = O.public_key(sd)
    if i % 5 == 1:
        b = bytearray(s); b[random.randrange(64)] ^= 1 << random.randrange(8); s = bytes(b)
    ent.append((pk, m, s))
encs = E.small_order_encodings()
for a in encs:
    for r in encs:
        ent.append((a, b"msg", r + bytes(32)))
pk, sg, mg, off = C.pack(ent)
t = time.time(); ok_o, vec_o = C.ed25519_verify_packed(pk, sg, mg, off, threads=8); to = time.time() - t
t = time.time(); ok_g, vec_g = ctx.ed25519_verify_batch(pk, sg, mg, off); tg = time.time() - t
bad = np.nonzero(vec_o != vec_g)[0]
print("parity", len(bad) == 0, "mismatches", len(bad), "valid", int(vec_o.sum()), "of", len(vec_o),
      "oracle_s", round(to, 3), "gpu_s", round(tg, 3))
if len(bad):
    print("first mismatches", bad[:10].tolist())
    sys.exit(1)

# timing on device-resident inputs
dev = torch.device("cuda:0")
def timed(n, reps=5):
    k = n // len(ent) + 1
    big = (ent * k)[:n]
    pk, sg, mg, off = C.pack(big)
    tp = torch.from_numpy(pk).to(dev); ts = torch.from_numpy(sg).to(dev)
    tm = torch.from_numpy(mg).to(dev); to_ = torch.from_numpy(off.view(np.int32)).to(dev)
    tv = torch.zeros(n, dtype=torch.uint8, device=dev)
    stream = torch.cuda.Stream()
    st = stream.cuda_stream
    ctx.ed25519_verify_batch_device(0, tp.data_ptr(), ts.data_ptr(), tm.data_ptr(), to_.data_ptr(), n, tv.data_ptr(), st)
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        ctx.ed25519_verify_batch_device(0, tp.data_ptr(), ts.data_ptr(), tm.data_ptr(), to_.data_ptr(), n, tv.data_ptr(), st)
    e1.record(stream); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    _, ref = C.ed25519_verify_packed(pk, sg, mg, off, threads=16) if n <= 20000 else (None, None)
    par = None if ref is None else bool((tv.cpu().numpy() == ref).all())
    return ms, par

res = {}
for n in [150, 10000, 100000, 1000000]:
    ms, par = timed(n)
    res[n] = (ms, n / ms * 1e3, par)
    print(json.dumps({"n": n, "ms": round(ms, 3), "verifies_per_s": round(n / ms * 1e3), "parity": par}))
