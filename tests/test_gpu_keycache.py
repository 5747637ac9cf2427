"""Key-cached path (TMV_FLAG_KEY_CACHE: device-resident 64-row combs of the
validator keys, k_key_build + k_prep_cached + k_verify_comb) must give the
same vectors as the oracle, across cache hits, misses and LRU eviction."""
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle_c as C
from tendermint_amd import _native as N
from tendermint_amd.testing.factory import Batch, make_c2_batch, make_sr25519_batch

pytestmark = pytest.mark.gpu


def _repeat_keys(b: Batch, n_keys: int) -> Batch:
    """Same signatures, but only n_keys distinct public keys (wrong key for most
    entries -> mostly invalid, which exercises the vector)."""
    ents = [b.entry(i) for i in range(b.n)]
    ents = [(ents[i % n_keys][0], m, s) if i % 3 else (pk, m, s) for i, (pk, m, s) in enumerate(ents)]
    return Batch.from_entries(ents)


def test_ed25519_cached_matches_oracle(ctx):
    b = make_c2_batch(2000, seed=31, edge_scale=4.0)
    _, ref = C.ed25519_verify_packed(b.pk, b.sig, b.msg, b.off, threads=8)
    for _ in range(3):  # miss, then hits
        ok, st = ctx.verify_batch_ex(N.TMV_KIND_ED25519, N.TMV_FLAG_KEY_CACHE, b.pk, b.sig, b.msg, b.off)
        assert np.array_equal(st.astype(np.uint8), ref)
    s = ctx.key_cache_stats()
    assert s["hits"] > 0 and s["misses"] > 0


def test_ed25519_cached_repeated_keys(ctx):
    b = _repeat_keys(make_c2_batch(1500, seed=32), 40)
    _, ref = C.ed25519_verify_packed(b.pk, b.sig, b.msg, b.off, threads=8)
    ok, st = ctx.verify_batch_ex(N.TMV_KIND_ED25519, N.TMV_FLAG_KEY_CACHE, b.pk, b.sig, b.msg, b.off)
    assert np.array_equal(st.astype(np.uint8), ref)


def test_sr25519_cached_matches_oracle(ctx):
    b = make_sr25519_batch(1200, seed=33, bad_frac=0.05)
    ref = C.sr25519_status_packed(b.pk, b.sig, b.msg, b.off, threads=8)
    for _ in range(2):
        ok, st = ctx.verify_batch_ex(N.TMV_KIND_SR25519, N.TMV_FLAG_KEY_CACHE, b.pk, b.sig, b.msg, b.off)
        assert np.array_equal(st, ref)


def test_eviction_small_capacity():
    """Capacity 64 with 3 rounds over 200 keys (evictions) and one batch with
    more distinct keys than the capacity (uncached fallback)."""
    code = r"""
import sys, numpy as np
sys.path.insert(0, '.'); sys.path.insert(0, 'oracle')
import oracle_c as C
from tendermint_amd import _native as N
from tendermint_amd.testing.factory import make_c2_batch, Batch
ctx = N.Context(1)
b = make_c2_batch(200, seed=34, edge_scale=10.0)
_, ref = C.ed25519_verify_packed(b.pk, b.sig, b.msg, b.off, threads=4)
for lo in (0, 50, 100, 150, 0, 60):
    idx = list(range(lo, min(lo + 50, b.n)))
    sub = Batch.from_entries([b.entry(i) for i in idx])
    ok, st = ctx.verify_batch_ex(N.TMV_KIND_ED25519, N.TMV_FLAG_KEY_CACHE, sub.pk, sub.sig, sub.msg, sub.off)
    assert np.array_equal(st.astype(np.uint8), ref[idx]), lo
ok, st = ctx.verify_batch_ex(N.TMV_KIND_ED25519, N.TMV_FLAG_KEY_CACHE, b.pk, b.sig, b.msg, b.off)
assert np.array_equal(st.astype(np.uint8), ref)
# the over-capacity batch must not leave keys without tables behind
for lo in (0, 50, 100, 150, 120, 10):
    idx = list(range(lo, min(lo + 50, b.n)))
    sub = Batch.from_entries([b.entry(i) for i in idx])
    ok, st = ctx.verify_batch_ex(N.TMV_KIND_ED25519, N.TMV_FLAG_KEY_CACHE, sub.pk, sub.sig, sub.msg, sub.off)
    assert np.array_equal(st.astype(np.uint8), ref[idx]), ("after overflow", lo)
s = ctx.key_cache_stats()
assert s["used"] <= 64 and s["capacity"] == 64, s
print("ok", s)
"""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, TMV_KEY_CACHE_CAPACITY="64")
    out = subprocess.run([sys.executable, "-c", code], env=env, cwd=root, capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    assert "ok" in out.stdout


def test_two_kernel_form_matches_oracle():
    """Batches above TMV_CACHED_FUSED_MAX take k_prep_cached + k_verify_comb
    instead of the fused latency kernel; both must give the oracle's vector."""
    code = r"""
import sys, numpy as np
sys.path.insert(0, '.'); sys.path.insert(0, 'oracle')
import oracle_c as C
from tendermint_amd import _native as N
from tendermint_amd.testing.factory import make_c2_batch, make_sr25519_batch
ctx = N.Context(1)
b = make_c2_batch(1000, seed=35, edge_scale=6.0)
_, ref = C.ed25519_verify_packed(b.pk, b.sig, b.msg, b.off, threads=4)
for _ in range(2):
    ok, st = ctx.verify_batch_ex(N.TMV_KIND_ED25519, N.TMV_FLAG_KEY_CACHE, b.pk, b.sig, b.msg, b.off)
    assert np.array_equal(st.astype(np.uint8), ref)
s = make_sr25519_batch(600, seed=36, bad_frac=0.05)
ref = C.sr25519_status_packed(s.pk, s.sig, s.msg, s.off, threads=4)
ok, st = ctx.verify_batch_ex(N.TMV_KIND_SR25519, N.TMV_FLAG_KEY_CACHE, s.pk, s.sig, s.msg, s.off)
assert np.array_equal(st, ref)
print("ok")
"""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, TMV_CACHED_FUSED_MAX="0")
    out = subprocess.run([sys.executable, "-c", code], env=env, cwd=root, capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    assert "ok" in out.stdout


def test_parallel_key_resolution_scattered_keys():
    """Batches of >= 16,384 entries resolve their keys in 16 parts: missing
    keys are deduplicated per key-hash part in parallel and every entry gets
    its key's slot from that part's ordinal.  Keys here recur across all
    parts (3,000 distinct keys over 20,000 entries, most entries signed by
    another key), over three calls whose key sets overlap (hits, misses and
    LRU evictions at capacity 4,096), then over a capacity of 2,048, where
    the batch has more distinct keys than the cache and takes the uncached
    path; every vector equals the oracle's."""
    code = r"""
import sys, numpy as np
sys.path.insert(0, '.'); sys.path.insert(0, 'oracle')
import oracle_c as C
from tendermint_amd import _native as N
from tendermint_amd.testing.factory import make_c2_batch, Batch
ctx = N.Context(1)
base = make_c2_batch(20000, seed=37, edge_scale=2.0)
ents = [base.entry(i) for i in range(base.n)]
def keyed(n_keys, first):
    # entry i keeps its own key when i % 50 == 0, else takes key first + (7 i) % n_keys of the pool
    out = [(ents[first + (7 * i) % n_keys][0], m, s) if i % 50 else (pk, m, s) for i, (pk, m, s) in enumerate(ents)]
    return Batch.from_entries(out)
for n_keys, first in ((3000, 0), (3000, 1500), (2500, 3000)):
    b = keyed(n_keys, first)
    _, ref = C.ed25519_verify_packed(b.pk, b.sig, b.msg, b.off, threads=8)
    ok, st = ctx.verify_batch_ex(N.TMV_KIND_ED25519, N.TMV_FLAG_KEY_CACHE, b.pk, b.sig, b.msg, b.off)
    assert np.array_equal(st.astype(np.uint8), ref), (n_keys, first)
s = ctx.key_cache_stats()
if sys.argv[1] == "4096":  # ~3,400 distinct keys per call fit: hits, misses and evictions
    assert s["hits"] > 0 and s["misses"] > 0, s
print("ok", s)
"""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for cap in ("4096", "2048"):
        env = dict(os.environ, TMV_KEY_CACHE_CAPACITY=cap)
        out = subprocess.run([sys.executable, "-c", code, cap], env=env, cwd=root, capture_output=True, text=True,
                             timeout=300)
        assert out.returncode == 0, (cap, out.stderr[-2000:])
        assert "ok" in out.stdout

