"""Every BASELINE.json config exercised by a -m gpu test at its own size
(C2 is tests/test_gpu_ed25519.py / test_gpu_batch_equation.py's committed 10k
batch; C3 / C4 are in tests/test_gpu_chains.py):

  C1  types.VerifyCommit on a 150-validator ed25519 commit through
      tmv_verify_commit (the key-cached fused latency path), valid and with
      one bad signature, error text equal to the oracle's
  C5  1M mixed ed25519 + sr25519 signatures in one batch (batch equation and
      per entry), status vector equal to the C oracle's
"""
import os

import numpy as np
import pytest

import chain_fixtures as CF
import light_ref as L
import oracle_c as C
from tendermint_amd import _native as N, host as H
from tendermint_amd.testing.factory import make_c1_commit, make_mixed_batch

pytestmark = pytest.mark.gpu
THREADS = min(16, os.cpu_count() or 1)


def _oracle_full(vals, bid, height, commit, chain="test_chain_id"):
    e = L.verify_commit(chain, CF.valset(vals), CF.block_id(bid), height, CF.commit(commit))
    return None if e is None else e.text


def test_c1_verify_commit_150(ctx):
    vals, bid, commit = make_c1_commit(150)
    for _ in range(3):  # cold (key table build) and warm key cache
        assert H.verify_commit(ctx, "test_chain_id", vals, bid, 3, commit) is None
        assert H.verify_commit_light(ctx, "test_chain_id", vals, bid, 3, commit) is None
    assert _oracle_full(vals, bid, 3, commit) is None
    # one bad signature deep in the commit: the batch path reports it with
    # %X of CommitSig.String() (types/validation.go:244-251)
    s = commit.signatures[117]
    b = bytearray(s.signature)
    b[20] ^= 0x04
    commit.signatures[117] = H.CommitSig(s.block_id_flag, s.validator_address, s.timestamp, bytes(b))
    want = _oracle_full(vals, bid, 3, commit)
    assert want.startswith("wrong signature (#117): ")
    assert H.verify_commit(ctx, "test_chain_id", vals, bid, 3, commit) == want
    # VerifyCommitLight stops at 2/3: #117 is beyond the 101-signature prefix
    assert H.verify_commit_light(ctx, "test_chain_id", vals, bid, 3, commit) is None
    # a wrong chain ID fails the first signature of the batch
    want = _oracle_full(vals, bid, 3, commit, chain="other")
    assert want.startswith("wrong signature (#0): ")
    assert H.verify_commit(ctx, "other", vals, bid, 3, commit) == want


def test_c1_prepared_call_latency_path(ctx):
    """The bench's C1 call (PreparedCommitCall) returns the reference's result."""
    vals, bid, commit = make_c1_commit(150)
    call = H.PreparedCommitCall(ctx, H.MODE_FULL, "test_chain_id", vals, bid, 3, commit)
    assert all(call() is None for _ in range(20))


def _mixed_oracle(kind, b):
    st = np.zeros(b.n, np.int8)
    for k in (0, 1):
        idx = np.nonzero(kind == k)[0]
        sub = b.take(idx)
        if k == 0:
            st[idx] = C.ed25519_verify_packed(sub.pk, sub.sig, sub.msg, sub.off, threads=THREADS)[1].astype(np.int8)
        else:
            st[idx] = C.sr25519_status_packed(sub.pk, sub.sig, sub.msg, sub.off, threads=THREADS)
    return st


def test_c5_1m_mixed_vs_oracle(ctx):
    """BASELINE C5: 1,000,000 mixed entries (20k distinct ed25519 + sr25519
    signatures with ~1% corrupted of each kind, tiled and shuffled so every
    batch-equation group mixes different entries) in one call; the oracle
    checks all 1M entries."""
    kind0, base = make_mixed_batch(20_000)
    rng = np.random.default_rng(5)
    idx = rng.permutation(np.arange(1_000_000) % base.n)
    b = base.take(idx)
    kind = kind0[idx]
    ref = _mixed_oracle(kind, b)
    assert set(np.unique(ref)) >= {-2, -1, 0, 1}
    for flags in (N.TMV_FLAG_BATCH_EQUATION, N.TMV_FLAG_PER_ENTRY, 0):
        ok, st = ctx.verify_mixed_batch_ex(flags, kind, b.pk, b.sig, b.msg, b.off)
        assert not ok
        assert np.array_equal(st, ref), (flags, int((st != ref).sum()))
