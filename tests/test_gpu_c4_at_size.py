"""BASELINE C4 at its configured size on the MI355X: blocksync replay of
10,000 blocks x 175 validators (internal/blocksync/reactor.go:582-586: the
light check of second.LastCommit, then ValidateBlock's full VerifyCommit of
first.LastCommit; look-ahead windows of 600, internal/blocksync/pool.go:32-35),
1.75 M commit signatures, every one checked against the C oracle
(tests/at_size.py states the three checks)."""
import random

import pytest

import at_size as A
import chain_fixtures as CF
import light_ref as L
from tendermint_amd import chains, host as H
from tendermint_amd.testing.factory import make_block_chain

pytestmark = pytest.mark.gpu
CHAIN = "test_chain_id"


@pytest.fixture(scope="module")
def c4(ctx):
    """The chain replayed clean, then with its seeded corruptions: the
    oracle's vector of every vote and the oracle's result of every light and
    full commit check blocksync makes (jobs 2(i-1), 2(i-1)+1 = block i's)."""
    vals, blocks, pv = make_block_chain(A.C4_BLOCKS, A.C4_VALS, packed=True)
    clean = chains.blocksync_replay(ctx, CHAIN, vals, blocks, H.BlockID())
    rng = random.Random(0xC4)
    # commit c of the packed votes is the commit for height c + 1, carried as
    # blocks[c + 1].last_commit (the last one by no block); commit 0 stays
    # clean (block 1's light check is not among the jobs)
    picks = sorted(rng.sample(range(1, A.C4_BLOCKS - 1), 50))
    for n_pick, c in enumerate(picks):
        i = rng.randrange(A.C4_VALS)
        A.corrupt_sig(blocks[c + 1].last_commit, i, pv, int(pv.commit_off[c]) + i, rng, s_plus_l=(n_pick % 10 == 0))
    A.progress("C4: chain generated and verified clean")
    vec = A.oracle_vector(pv)
    A.progress("C4: oracle vector")
    jobs, want = [], []
    ov = CF.valset(vals)
    oc = {}

    def commit(c):
        if id(c) not in oc:
            oc[id(c)] = CF.commit(c)
        return oc[id(c)]

    with L.signature_oracle(A.Verdicts(pv, vec)):
        for i in range(1, A.C4_BLOCKS - 1):
            f, s2 = blocks[i], blocks[i + 1]
            jobs.append(H.CommitJob(H.MODE_LIGHT, CHAIN, vals, f.block_id, f.height, s2.last_commit))
            e = L.verify_commit_light(CHAIN, ov, CF.block_id(f.block_id), f.height, commit(s2.last_commit))
            want.append(None if e is None else e.text)
            jobs.append(H.CommitJob(H.MODE_FULL, CHAIN, vals, blocks[i - 1].block_id, f.height - 1, f.last_commit))
            e = L.verify_commit(CHAIN, ov, CF.block_id(blocks[i - 1].block_id), f.height - 1, commit(f.last_commit))
            want.append(None if e is None else e.text)
            if i >= 2:
                oc.pop(id(blocks[i - 1].last_commit), None)
    A.progress("C4: oracle results of every job")
    return dict(vals=vals, blocks=blocks, pv=pv, picks=picks, vec=vec, jobs=jobs, want=want, clean=clean)


def test_c4_clean_chain_replays(c4):
    """The uncorrupted 10,000-block chain replays end to end (9,999 blocks
    applied: the last block has no successor carrying its commit)."""
    assert c4["clean"] == (A.C4_BLOCKS - 1, None)


def test_c4_signature_vector_vs_oracle(ctx, c4):
    """Every vote of every 600-commit window through the key-cached batch
    path equals the oracle's vector (50 invalid of 1,750,000)."""
    assert int((~c4["vec"].astype(bool)).sum()) == len(c4["picks"])
    A.engine_vector_check(ctx, c4["pv"], c4["vec"], 600)


def test_c4_every_commit_check_vs_oracle(ctx, c4):
    """tmv_verify_commits over windows of 600 blocks (1,200 jobs, shared
    commits verified once): every light and full check's result equals the
    oracle's."""
    jobs, want = c4["jobs"], c4["want"]
    got = []
    for lo in range(0, len(jobs), 1200):
        got += H.verify_commits(ctx, jobs[lo:lo + 1200])
    diff = [j for j, (g, w) in enumerate(zip(got, want)) if g != w]
    assert not diff, f"jobs {diff[:5]}: engine {[got[j] for j in diff[:2]]} vs oracle {[want[j] for j in diff[:2]]}"
    n_light_fail = sum(1 for j in range(0, len(want), 2) if want[j])
    n_full_fail = sum(1 for j in range(1, len(want), 2) if want[j])
    # every corrupted commit fails its full check; flips outside the light
    # 2/3 prefix pass the light one, as in the reference
    assert n_full_fail == len(c4["picks"]) and n_light_fail < n_full_fail


def test_c4_replay_first_error(ctx, c4):
    """blocksync_replay over all 10,000 blocks stops at the first block
    either check rejects, with that check's error (light first, as
    poolRoutine does)."""
    want, blocks = c4["want"], c4["blocks"]
    applied, err = chains.blocksync_replay(ctx, CHAIN, c4["vals"], blocks, H.BlockID())
    k = next(j for j, w in enumerate(want) if w)
    assert applied == k // 2 + 1 and err == (blocks[k // 2 + 1].height, want[k])
