"""Commit verification (types/validation.go) through the C++ host layer.

The cases restate types/validation_test.go:17-292 (same table, same
asserted error substrings).  Each runs on two backends:
  * fake — CPU, tests/native/commit_check.cpp: the same C++ control flow
    with a test-double signature scheme (no GPU);
  * gpu  — libtmgpu.so's tmv_verify_commit with real ed25519 / sr25519
    signatures verified on the MI355X (marked gpu).
"""
import pytest

from tendermint_amd import host as H
import commit_fixtures as F

ROUND, HEIGHT = 0, 100
CHAIN = "Lalande21185"
BLOCK_ID = F.make_block_id(b"blockhash", 1000, b"partshash")

CASES = [
    # description, vote chainID, vote blockID, valSize, commit height, blockVotes, nilVotes, absentVotes, expErr
    ("good (batch verification)", CHAIN, BLOCK_ID, 3, HEIGHT, 3, 0, 0, False),
    ("good (single verification)", CHAIN, BLOCK_ID, 1, HEIGHT, 1, 0, 0, False),
    ("wrong signature (#0)", "EpsilonEridani", BLOCK_ID, 2, HEIGHT, 2, 0, 0, True),
    ("wrong block ID", CHAIN, F.random_block_id(7), 2, HEIGHT, 2, 0, 0, True),
    ("wrong height", CHAIN, BLOCK_ID, 1, HEIGHT - 1, 1, 0, 0, True),
    ("wrong set size: 4 vs 3", CHAIN, BLOCK_ID, 4, HEIGHT, 3, 0, 0, True),
    ("wrong set size: 1 vs 2", CHAIN, BLOCK_ID, 1, HEIGHT, 2, 0, 0, True),
    ("insufficient voting power: got 30, needed more than 66", CHAIN, BLOCK_ID, 10, HEIGHT, 3, 2, 5, True),
    ("insufficient voting power: got 0, needed more than 6", CHAIN, BLOCK_ID, 1, HEIGHT, 0, 0, 1, True),
    ("insufficient voting power: got 60, needed more than 60", CHAIN, BLOCK_ID, 9, HEIGHT, 6, 3, 0, True),
]


@pytest.fixture(scope="module")
def fake():
    return F.FakeBackend()


def _backends(request):
    return request.param


@pytest.fixture(params=["fake", pytest.param("ed25519", marks=pytest.mark.gpu),
                        pytest.param("sr25519", marks=pytest.mark.gpu)])
def backend(request, fake):
    if request.param == "fake":
        return fake
    ctx = request.getfixturevalue("ctx")
    return F.GpuBackend(ctx, request.param)


def _scheme(backend):
    return backend.scheme


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_verify_commit_all(backend, case):
    """types/validation_test.go:17-141 TestValidatorSet_VerifyCommit_All."""
    desc, vote_chain, vote_bid, val_size, height, block_votes, nil_votes, absent_votes, exp_err = case
    vals, signers = F.rand_val_set(_scheme(backend), val_size, 10)
    total = block_votes + nil_votes + absent_votes
    sigs = []
    vi = 0
    for _ in range(absent_votes):
        sigs.append(H.CommitSig())
        vi += 1
    for i in range(block_votes + nil_votes):
        s = signers[vi % len(signers)]
        flag = H.BLOCK_ID_FLAG_COMMIT if i < block_votes else H.BLOCK_ID_FLAG_NIL
        sigs.append(F.sign_commit_sig(s, vote_chain, height, ROUND, vote_bid, flag, (1577836800 + vi, 5000 * vi)))
        vi += 1
    commit = H.Commit(height, ROUND, vote_bid, sigs)

    for fn in (backend.verify_commit, backend.verify_commit_light):
        err = fn(CHAIN, vals, BLOCK_ID, HEIGHT, commit)
        if exp_err:
            assert err is not None and desc in err, (fn.__name__, err)
        else:
            assert err is None, (fn.__name__, err)

    if total != val_size or not vote_bid.equals(BLOCK_ID) or height != HEIGHT:
        exp_err = False
    err = backend.verify_commit_light_trusting(CHAIN, vals, commit, (2, 3))
    if exp_err:
        assert err is not None and desc in err, err
    else:
        assert err is None, err


def _four_val_commit(backend, chain="test_chain_id", h=3):
    vals, signers = F.rand_val_set(_scheme(backend), 4, 10)
    bid = F.random_block_id(3)
    commit = F.make_commit(signers, chain, h, 0, bid)
    assert backend.verify_commit(chain, vals, bid, h, commit) is None
    return vals, signers, bid, commit


def test_check_all_signatures(backend):
    """TestValidatorSet_VerifyCommit_CheckAllSignatures (:143-172)."""
    vals, signers, bid, commit = _four_val_commit(backend)
    s = commit.signatures[3]
    commit.signatures[3] = F.sign_commit_sig(signers[3], "CentaurusA", 3, 0, bid, H.BLOCK_ID_FLAG_COMMIT, s.timestamp)
    err = backend.verify_commit("test_chain_id", vals, bid, 3, commit)
    assert err is not None and "wrong signature (#3)" in err
    # batch path error text: %X of CommitSig.String() (types/validation.go:249)
    assert err.startswith("wrong signature (#3): ")
    shown = bytes.fromhex(err.split(": ", 1)[1]).decode()
    assert shown.startswith("CommitSig{") and " @ 2020-01-01T00:00:00.000003Z}" in shown


def test_light_returns_at_two_thirds(backend):
    """TestValidatorSet_VerifyCommitLight_ReturnsAsSoonAsMajorityOfVotingPowerSigned (:174-201)."""
    vals, signers, bid, commit = _four_val_commit(backend)
    s = commit.signatures[3]
    commit.signatures[3] = F.sign_commit_sig(signers[3], "CentaurusA", 3, 0, bid, H.BLOCK_ID_FLAG_COMMIT, s.timestamp)
    assert backend.verify_commit_light("test_chain_id", vals, bid, 3, commit) is None


def test_light_trusting_returns_at_trust_level(backend):
    """TestValidatorSet_VerifyCommitLightTrusting_ReturnsAsSoonAsTrustLevelOfVotingPowerSigned (:203-229)."""
    vals, signers, bid, commit = _four_val_commit(backend)
    s = commit.signatures[2]
    commit.signatures[2] = F.sign_commit_sig(signers[2], "CentaurusA", 3, 0, bid, H.BLOCK_ID_FLAG_COMMIT, s.timestamp)
    assert backend.verify_commit_light_trusting("test_chain_id", vals, commit, (1, 3)) is None


def test_light_trusting_overlap(backend):
    """TestValidatorSet_VerifyCommitLightTrusting (:231-274)."""
    vals, signers = F.rand_val_set(_scheme(backend), 6, 1)
    bid = F.random_block_id(11)
    commit = F.make_commit(signers, "test_chain_id", 1, 1, bid)
    new_vals, _ = F.rand_val_set(_scheme(backend), 2, 1, tag="other")
    assert backend.verify_commit_light_trusting("test_chain_id", vals, commit, (1, 3)) is None
    assert backend.verify_commit_light_trusting("test_chain_id", new_vals, commit, (1, 3)) is not None
    merged = H.ValidatorSet(sorted(new_vals.validators + vals.validators, key=lambda v: v.address), 0)
    assert backend.verify_commit_light_trusting("test_chain_id", merged, commit, (1, 3)) is None


def test_light_trusting_overflow(backend):
    """TestValidatorSet_VerifyCommitLightTrustingErrorsOnOverflow (:276-292)."""
    max_total = (2**63 - 1) // 8  # MaxTotalVotingPower (types/validator_set.go:25)
    vals, signers = F.rand_val_set(_scheme(backend), 1, max_total)
    bid = F.random_block_id(5)
    commit = F.make_commit(signers, "test_chain_id", 1, 1, bid)
    err = backend.verify_commit_light_trusting("test_chain_id", vals, commit, (25, 55))
    assert err is not None and "int64 overflow" in err


def test_nil_args_and_zero_denominator(backend):
    vals, signers, bid, commit = _four_val_commit(backend)
    assert backend.verify_commit("c", None, bid, 3, commit) == "nil validator set"
    assert backend.verify_commit("c", vals, bid, 3, None) == "nil commit"
    assert backend.verify_commit_light_trusting("c", vals, commit, (1, 0)) == "trustLevel has zero Denominator"


def test_double_vote_by_address(backend):
    """verifyCommitBatch lookUpByIndex=false double-vote detection (types/validation.go:200-203)."""
    vals, signers, bid, commit = _four_val_commit(backend)
    commit.signatures[2] = commit.signatures[1]
    err = backend.verify_commit_light_trusting("test_chain_id", vals, commit, (9, 10))
    assert err is not None and err.startswith("double vote from Validator{") and "(1 and 2)" in err


def test_wrong_block_id_text(backend):
    vals, signers, bid, commit = _four_val_commit(backend)
    other = F.make_block_id(b"x", 7, b"y")
    err = backend.verify_commit("test_chain_id", vals, other, 3, commit)
    want = ("invalid commit -- wrong block ID: want " + other.hash.hex().upper() + ":7:" +
            other.psh_hash[:6].hex().upper() + ", got " + bid.hash.hex().upper() + ":" + str(bid.psh_total) + ":" +
            bid.psh_hash[:6].hex().upper())
    assert err == want


def test_verify_many_equals_single_fake(fake):
    """Cross-commit batching (CommitVerifier::VerifyMany / tmv_verify_commits)
    returns exactly the per-commit results, on 300 random commit checks."""
    jobs = F.random_jobs("fake", 300, seed=5)
    many = F.fake_verify_commits(fake, jobs)
    single = [F.single_result(fake, jb) for jb in jobs]
    assert many == single
    assert sum(r is None for r in many) > 20 and sum(r is not None for r in many) > 20


@pytest.mark.parametrize("slice_jobs", ["0", "500"])
def test_verify_many_equals_single_fake_large(fake, slice_jobs, monkeypatch):
    """Large enough (≈15k entries) for the multi-threaded packing and the
    shared-commit dedup slots of tmv_verify_commits; in one pass and in
    pipelined slices (3000 jobs = 6 slices of 500 taken by two threads,
    TMV_HOST_SLICE)."""
    monkeypatch.setenv("TMV_HOST_SLICE", slice_jobs)
    jobs = F.random_jobs("fake", 3000, seed=9)
    many = F.fake_verify_commits(fake, jobs)
    single = [F.single_result(fake, jb) for jb in jobs]
    assert many == single


@pytest.mark.gpu
@pytest.mark.parametrize("scheme,n", [("ed25519", 80), ("sr25519", 80), ("ed25519", 1100)])
def test_verify_many_equals_single_gpu(ctx, scheme, n, monkeypatch):
    """1,100 jobs in three pipelined slices (TMV_HOST_SLICE=400): two host
    threads, engine calls from both."""
    monkeypatch.setenv("TMV_HOST_SLICE", "400")
    jobs = F.random_jobs(scheme, n, seed=6)
    g = F.GpuBackend(ctx, scheme)
    many = H.verify_commits(ctx, jobs)
    single = [F.single_result(g, jb) for jb in jobs]
    assert many == single
