"""Host-buffer calls from several threads on one device (tmverify_runtime.cpp
run_batch: each call claims its own lanes and holds the device lock while it
stages and launches a chunk, not while it waits for the device).  Results
must equal the same calls made one at a time -- with a key cache small enough
that concurrent windows evict each other's keys (resolve_keys waits for
every chunk in flight before a new key takes a slot) and a streamed
uncached batch running beside them."""
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from tendermint_amd import _native as N, host as H
from tendermint_amd.testing.factory import make_block_chain, make_c2_batch

pytestmark = pytest.mark.gpu


def _corrupt(commit: H.Commit, i: int):
    s = commit.signatures[i]
    b = bytearray(s.signature)
    b[5] ^= 1
    commit.signatures[i] = H.CommitSig(s.block_id_flag, s.validator_address, s.timestamp, bytes(b))


def _windows(vals, blocks, per):
    jobs = []
    for i in range(1, len(blocks) - 1):
        f, s2 = blocks[i], blocks[i + 1]
        jobs.append(H.CommitJob(H.MODE_LIGHT, "test_chain_id", vals, f.block_id, f.height, s2.last_commit))
        jobs.append(H.CommitJob(H.MODE_FULL, "test_chain_id", vals, blocks[i - 1].block_id, f.height - 1,
                                f.last_commit))
    return [jobs[lo:lo + 2 * per] for lo in range(0, len(jobs), 2 * per)]


@pytest.mark.parametrize("capacity", [256, 4096])
def test_concurrent_commit_windows_and_streamed_batch(monkeypatch, capacity):
    # 4 chains of 175 distinct validators each: 700 keys against a cache of
    # 256 slots evict constantly; 4096 hold them all
    monkeypatch.setenv("TMV_KEY_CACHE_CAPACITY", str(capacity))
    ctx = N.Context(1)
    chains_ = [make_block_chain(61, 175, seed=100 + t) for t in range(4)]
    _corrupt(chains_[1][1][17].last_commit, 3)     # a full check fails
    _corrupt(chains_[3][1][40].last_commit, 120)   # past 2/3: only the full check reads it
    _corrupt(chains_[3][1][52].last_commit, 0)
    wins = [_windows(v, b, 12) for v, b in chains_]
    base = make_c2_batch(10_000, seed=5)
    big = base.tile(160_000)  # streamed (more than TMV_STREAM_FIRST entries, uncached)
    flags = N.TMV_FLAG_BATCH_EQUATION

    want = [[H.verify_commits(ctx, w) for w in ws] for ws in wins]
    want_big = ctx.verify_batch_ex(N.TMV_KIND_ED25519, flags, big.pk, big.sig, big.msg, big.off)[1].copy()
    assert any(e is not None for w in want[1] for e in w)
    assert any(e is not None for w in want[3] for e in w)
    assert all(e is None for t in (0, 2) for w in want[t] for e in w)
    valid = ("honest", "small_order", "noncanonical_y", "neg_zero")  # make_c2_batch's valid entries
    assert np.array_equal(want_big, np.array([1 if k in valid else 0 for k in big.kinds], np.int8))

    def chain_job(t):
        return [H.verify_commits(ctx, w) for w in wins[t]]

    def big_job(_):
        return ctx.verify_batch_ex(N.TMV_KIND_ED25519, flags, big.pk, big.sig, big.msg, big.off)[1]

    for _ in range(2):
        with ThreadPoolExecutor(6) as ex:
            fut = [ex.submit(chain_job, t) for t in range(4)] + [ex.submit(big_job, 0), ex.submit(chain_job, 1)]
            got = [f.result() for f in fut]
        for t in range(4):
            assert got[t] == want[t], t
        assert got[5] == want[1]
        assert np.array_equal(got[4], want_big)
    ctx.close()
