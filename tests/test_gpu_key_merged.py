"""Key-merged batch equation (msm.h): key-cached
batches above the batch-equation threshold are ordered by key, the A terms
of a group collapse to one comb sum per key, and the vector must still be
the oracle's, entry for entry, in the caller's order."""
import os
import random
import subprocess
import sys

import numpy as np
import pytest

import oracle_c as C
from tendermint_amd import _native as N
from tendermint_amd.testing._openssl import Ed25519Signer
from tendermint_amd.testing.factory import Batch, key_seed, make_c2_batch

pytestmark = pytest.mark.gpu

KM = N.TMV_FLAG_KEY_CACHE | N.TMV_FLAG_BATCH_EQUATION


def _keyed_batch(n, n_keys, seed, bad=()):
    """n signatures by n_keys validators (interleaved like commits), entries in
    `bad` corrupted (bit flip in R, S or the message)."""
    rng = random.Random(seed)
    signers = [Ed25519Signer(key_seed(k, "km")) for k in range(n_keys)]
    ents = []
    for i in range(n):
        s = signers[i % n_keys]
        msg = b"vote %d %d" % (i, rng.randrange(1 << 30))
        sig = s.sign(msg)
        if i in bad:
            b = bytearray(sig)
            b[rng.randrange(64) if rng.randrange(2) else rng.randrange(32)] ^= 1 << rng.randrange(8)
            sig = bytes(b)
        ents.append((s.public_key, msg, sig))
    return Batch.from_entries(ents)


def _ref(b):
    _, ref = C.ed25519_verify_packed(b.pk, b.sig, b.msg, b.off, threads=8)
    return ref


def test_all_valid_no_group_fails(ctx):
    b = _keyed_batch(6000, 150, 61)
    ctx.set_batch_options(stats=True)
    try:
        s0 = ctx.batch_stats()
        ok, st = ctx.verify_batch_ex(N.TMV_KIND_ED25519, KM, b.pk, b.sig, b.msg, b.off)
        s1 = ctx.batch_stats()
    finally:
        ctx.set_batch_options()
    assert ok and (st == 1).all()
    assert s1["groups"] - s0["groups"] == (6000 + 255) // 256 and s1["failed"] == s0["failed"]


@pytest.mark.parametrize("group_log2", [5, 6, 8, 10])
def test_corrupted_entries_match_oracle(ctx, group_log2):
    rng = random.Random(62 + group_log2)
    n = 8000
    bad = set(rng.sample(range(n), 25))
    b = _keyed_batch(n, 97, 62 + group_log2, bad)
    ref = _ref(b)
    ctx.set_batch_options(group_log2=group_log2, stats=True)
    try:
        s0 = ctx.batch_stats()
        ok, st = ctx.verify_batch_ex(N.TMV_KIND_ED25519, KM, b.pk, b.sig, b.msg, b.off)
        s1 = ctx.batch_stats()
    finally:
        ctx.set_batch_options()
    assert np.array_equal(st.astype(np.uint8), ref)
    assert not ok
    # every failing group holds a corrupted entry, and there are corrupted entries
    assert s1["groups"] - s0["groups"] == (n + (1 << group_log2) - 1) >> group_log2
    assert 1 <= s1["failed"] - s0["failed"] <= len(bad)


def test_edge_cases_and_small_order(ctx):
    """C2's ZIP-215 edge cases (small-order A and R, non-canonical y, S + l,
    undecodable encodings) repeated so that their keys sit in the cache."""
    base = make_c2_batch(600, seed=63, edge_scale=20.0)
    b = base.tile(9000)
    ref = _ref(b)
    ok, st = ctx.verify_batch_ex(N.TMV_KIND_ED25519, KM, b.pk, b.sig, b.msg, b.off)
    assert np.array_equal(st.astype(np.uint8), ref)


def test_default_threshold_and_vote_path(ctx):
    """Without flags a keyed batch above 16,384 entries takes the key-merged
    form (commit traffic); same vector as per entry."""
    rng = random.Random(64)
    n = 20000
    bad = set(rng.sample(range(n), 10))
    b = _keyed_batch(n, 175, 64, bad)
    ref = _ref(b)
    ok, st = ctx.verify_batch_ex(N.TMV_KIND_ED25519, N.TMV_FLAG_KEY_CACHE, b.pk, b.sig, b.msg, b.off)
    assert np.array_equal(st.astype(np.uint8), ref)
    ok2, st2 = ctx.verify_batch_ex(N.TMV_KIND_ED25519, N.TMV_FLAG_KEY_CACHE | N.TMV_FLAG_PER_ENTRY, b.pk, b.sig,
                                   b.msg, b.off)
    assert np.array_equal(st, st2)


def test_distinct_keys_fall_back(ctx):
    """Every key once: too many runs per group, so the per-entry key-cached
    path runs; same vector."""
    b = make_c2_batch(3000, seed=65, edge_scale=3.0)
    ref = _ref(b)
    ok, st = ctx.verify_batch_ex(N.TMV_KIND_ED25519, KM, b.pk, b.sig, b.msg, b.off)
    assert np.array_equal(st.astype(np.uint8), ref)


def test_sr25519_key_merged(ctx):
    from tendermint_amd.testing.sr25519_factory import Sr25519Signer, mini_from_secret
    rng = random.Random(66)
    signers = [Sr25519Signer(mini_from_secret(b"km: %x" % k)) for k in range(40)]
    ents = []
    for i in range(4000):
        s = signers[i % 40]
        msg = b"sr vote %d" % i
        sig = s.sign(msg, b"%d" % i)
        r = rng.random()
        if r < 0.003:
            b_ = bytearray(sig); b_[3] ^= 8; sig = bytes(b_)
        elif r < 0.005:
            b_ = bytearray(sig); b_[63] &= 0x7F; sig = bytes(b_)  # no marker: Add error -2
        ents.append((s.public_key, msg, sig))
    # one undecodable key repeated (Add error -1)
    bad_pk = (int.from_bytes(signers[0].public_key, "little") | 1).to_bytes(32, "little")
    for i in range(0, 4000, 97):
        ents[i] = (bad_pk, ents[i][1], ents[i][2])
    b = Batch.from_entries(ents)
    ref = C.sr25519_status_packed(b.pk, b.sig, b.msg, b.off, threads=8)
    ok, st = ctx.verify_batch_ex(N.TMV_KIND_SR25519, KM, b.pk, b.sig, b.msg, b.off)
    assert np.array_equal(st, ref)


def test_repeated_calls_fresh_randomness(ctx):
    b = _keyed_batch(5000, 64, 67, bad={17, 4000})
    ref = _ref(b)
    for _ in range(3):
        ok, st = ctx.verify_batch_ex(N.TMV_KIND_ED25519, KM, b.pk, b.sig, b.msg, b.off)
        assert np.array_equal(st.astype(np.uint8), ref)


def test_small_cache_falls_back_uncached():
    """More distinct keys than the cache: the uncached batch equation runs."""
    code = r"""
import sys, numpy as np
sys.path.insert(0, '.'); sys.path.insert(0, 'oracle'); sys.path.insert(0, 'tests')
import oracle_c as C
from tendermint_amd import _native as N
from test_gpu_key_merged import _keyed_batch, KM
ctx = N.Context(1)
b = _keyed_batch(3000, 100, 68, bad={5, 2999})
_, ref = C.ed25519_verify_packed(b.pk, b.sig, b.msg, b.off, threads=4)
ok, st = ctx.verify_batch_ex(N.TMV_KIND_ED25519, KM, b.pk, b.sig, b.msg, b.off)
assert np.array_equal(st.astype(np.uint8), ref)
print("ok")
"""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, TMV_KEY_CACHE_CAPACITY="64")
    out = subprocess.run([sys.executable, "-c", code], env=env, cwd=root, capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    assert "ok" in out.stdout
