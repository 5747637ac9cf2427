"""Host-buffer pipeline: batches of at least two chunks (TMV_HOST_CHUNK)
alternate between two staging lanes, so chunk k+1's staging and copy overlap
chunk k's kernels; uncached batch-equation batches are streamed instead (one
pipeline per chunk, inputs staged and copied in parts, each part's kernels
behind its copy: TMV_STREAM_FIRST / TMV_STREAM_PART).  Every path must still
give the oracle's vector, in order, across chunk and part edges, with key
builds and evictions between chunks."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

CODE = r"""
import random, sys, numpy as np
sys.path.insert(0, '.'); sys.path.insert(0, 'oracle'); sys.path.insert(0, 'tests')
import oracle_c as C
import vote_cases as V
from tendermint_amd import _native as N
from tendermint_amd.testing.factory import Batch, make_c2_batch, make_sr25519_batch
from test_gpu_key_merged import _keyed_batch
ctx = N.Context(1)
ED, SR = N.TMV_KIND_ED25519, N.TMV_KIND_SR25519

# uncached: per entry and batch equation, ragged chunk edges
b = make_c2_batch(10000, seed=81, edge_scale=3.0)
_, ref = C.ed25519_verify_packed(b.pk, b.sig, b.msg, b.off, threads=8)
for flags in (N.TMV_FLAG_PER_ENTRY, N.TMV_FLAG_BATCH_EQUATION):
    ok, st = ctx.verify_batch_ex(ED, flags, b.pk, b.sig, b.msg, b.off)
    assert np.array_equal(st.astype(np.uint8), ref), flags
ok, st = ctx.ed25519_verify_batch(b.pk, b.sig, b.msg, b.off)
assert np.array_equal(st.astype(np.uint8), ref)

# key cache: per entry and key-merged, keys spread over the chunks
k = _keyed_batch(12000, 150, 82, bad={3, 4100, 9000, 11999})
_, kref = C.ed25519_verify_packed(k.pk, k.sig, k.msg, k.off, threads=8)
for flags in (N.TMV_FLAG_KEY_CACHE | N.TMV_FLAG_PER_ENTRY, N.TMV_FLAG_KEY_CACHE | N.TMV_FLAG_BATCH_EQUATION):
    for _ in range(2):
        ok, st = ctx.verify_batch_ex(ED, flags, k.pk, k.sig, k.msg, k.off)
        assert np.array_equal(st.astype(np.uint8), kref), flags

# sr25519
s = make_sr25519_batch(5000, seed=83, bad_frac=0.02)
sref = C.sr25519_status_packed(s.pk, s.sig, s.msg, s.off, threads=8)
ok, st = ctx.verify_batch_ex(SR, N.TMV_FLAG_KEY_CACHE, s.pk, s.sig, s.msg, s.off)
assert np.array_equal(st, sref)
ok, st = ctx.sr25519_verify_batch(s.pk, s.sig, s.msg, s.off)
assert np.array_equal(st, sref)
ok, st = ctx.verify_batch_ex(SR, N.TMV_FLAG_BATCH_EQUATION, s.pk, s.sig, s.msg, s.off)
assert np.array_equal(st, sref)

# device-built vote messages, chunked
rng = random.Random(84)
tmpls, votes, msgs = V.random_votes(rng, 30, 9000)
from tendermint_amd.testing._openssl import Ed25519Signer
from tendermint_amd.testing.factory import key_seed
ents = []
for i, m in enumerate(msgs):
    sg = Ed25519Signer(key_seed(i % 61))
    sig = sg.sign(m)
    if i % 1000 == 7:
        sig = sig[:10] + bytes([sig[10] ^ 1]) + sig[11:]
    ents.append((sg.public_key, m, sig))
vb = Batch.from_entries(ents)
_, vref = C.ed25519_verify_packed(vb.pk, vb.sig, vb.msg, vb.off, threads=8)
segs = [V.segments(t) for t in tmpls]
for flags in (N.TMV_FLAG_KEY_CACHE, N.TMV_FLAG_KEY_CACHE | N.TMV_FLAG_BATCH_EQUATION):
    ok, st = ctx.verify_votes(ED, flags, segs, votes, vb.pk, vb.sig)
    assert np.array_equal(st.astype(np.uint8), vref)
print("ok")
"""


@pytest.mark.parametrize("chunk,capacity,extra", [
    ("2048", "4096", {}),
    ("3000", "100", {}),  # small chunks over the lanes; the keyed batch overflows the cache
    ("2048", "4096", {"TMV_STREAM_FIRST": "1000", "TMV_STREAM_PART": "3000"}),  # streamed in parts
], ids=["default", "small-chunks", "streamed"])
def test_chunked_host_batches(chunk, capacity, extra):
    """Capacity 100 < the keyed batch's 150 keys: that batch takes the
    uncached path; the votes' 61 keys fit and evict slots between calls."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, TMV_HOST_CHUNK=chunk, TMV_KEY_CACHE_CAPACITY=capacity, **extra)
    out = subprocess.run([sys.executable, "-c", CODE], env=env, cwd=root, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-3000:]
    assert "ok" in out.stdout


BIG = r"""
import json, sys, numpy as np
import torch  # before the engine's HIP init (pinned buffer below)
sys.path.insert(0, '.')
from tendermint_amd import _native as N
from tendermint_amd.testing.factory import Batch, make_c2_batch
gold = json.load(open('tests/golden/c2_expected.json'))
bits = np.unpackbits(np.frombuffer(bytes.fromhex(gold['valid_bits_hex']), np.uint8), bitorder='little')[:10000]
b = make_c2_batch(10000)
ctx = N.Context(1)
for reps in (20, 4):  # 200k: parts of 32k + 128k + a ragged tail; 40k: 32k + a ragged tail
    hb = Batch.concat([b] * reps)
    for _ in range(2):
        ok, st = ctx.verify_batch_ex(N.TMV_KIND_ED25519, N.TMV_FLAG_BATCH_EQUATION, hb.pk, hb.sig, hb.msg, hb.off)
        assert np.array_equal(st.astype(np.uint8), np.tile(bits, reps)), reps
# caller buffers at odd addresses (pinned pages start past each span's
# head, the bytes around them staged) and a buffer that is already pinned
# (its registration fails: staged)
def shifted(a, k):
    buf = np.zeros(a.nbytes + 64, np.uint8)
    v = buf[k:k + a.nbytes]
    v[:] = a.reshape(-1).view(np.uint8)
    return v.view(a.dtype).reshape(a.shape)
hb = Batch.concat([b] * 20)
want = np.tile(bits, 20)
ok, st = ctx.verify_batch_ex(N.TMV_KIND_ED25519, N.TMV_FLAG_BATCH_EQUATION, shifted(hb.pk, 1), shifted(hb.sig, 3),
                             shifted(hb.msg, 5), hb.off)
assert np.array_equal(st.astype(np.uint8), want)
assert torch.cuda.is_available()
pinned_sig = torch.from_numpy(hb.sig.copy()).pin_memory().numpy()
ctx.metrics_reset()
ok, st = ctx.verify_batch_ex(N.TMV_KIND_ED25519, N.TMV_FLAG_BATCH_EQUATION, hb.pk, pinned_sig, hb.msg, hb.off)
assert np.array_equal(st.astype(np.uint8), want)
# every byte crosses once, except the one offset two streamed parts share
# (each part carries its own [a, b] offsets; at most 64 parts)
payload = hb.pk.nbytes + hb.sig.nbytes + hb.msg.nbytes + hb.off.nbytes
h2d = ctx.metrics()["h2d_bytes"]
assert payload <= h2d <= payload + 4 * 64, (h2d, payload)
# two calls at once on the same caller buffers (each claims its own lanes):
# the second one's registrations of the same pages fail, so it stages them
from concurrent.futures import ThreadPoolExecutor
with ThreadPoolExecutor(2) as ex:
    res = list(ex.map(lambda _: ctx.verify_batch_ex(N.TMV_KIND_ED25519, N.TMV_FLAG_BATCH_EQUATION, hb.pk, hb.sig,
                                                    hb.msg, hb.off)[1], range(2)))
for st in res:
    assert np.array_equal(st.astype(np.uint8), want)
# read-only mappings of the caller's inputs (a file mapped PROT_READ)
import tempfile, os
with tempfile.TemporaryDirectory() as td:
    ro = []
    for name, a in (("pk", hb.pk), ("sig", hb.sig), ("msg", hb.msg)):
        path = os.path.join(td, name)
        a.tofile(path)
        ro.append(np.memmap(path, dtype=a.dtype, mode="r", shape=a.shape))
    ok, st = ctx.verify_batch_ex(N.TMV_KIND_ED25519, N.TMV_FLAG_BATCH_EQUATION, ro[0], ro[1], ro[2], hb.off)
    assert np.array_equal(st.astype(np.uint8), want)
    del ro
print("ok")
"""


def test_streamed_c2_host_batches():
    """The driver-sized host batch (BASELINE C2 tiled to 200k and 40k entries)
    streamed with the default parts: the vector equals the committed C2
    bitmap repeated, twice in a row on the same lane, with the caller's pages
    pinned -- misaligned buffers (the bytes around the pinned pages staged),
    an already-pinned buffer (its registration fails, so it is staged), two
    calls at once on the same buffers and read-only file mappings included;
    the statuses come back into the caller's pinned pages."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, "-c", BIG], cwd=root, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-3000:]
    assert "ok" in out.stdout
