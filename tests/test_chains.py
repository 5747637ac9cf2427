"""The light-client and blocksync drivers (tendermint_amd/chains.py) on the
CPU: the product's C++ host layer with the C oracle's signature checks
(tests/native/commit_check.cpp) against the oracle's restatement of
light/client.go's loops (oracle/light_ref.py).  The GPU twin is
tests/test_gpu_chains.py."""
import pytest

import chain_fixtures as CF
import light_ref as L
from tendermint_amd import chains, host as H
from tendermint_amd.testing.factory import header_hash, make_block_chain, make_light_chain

PERIOD = 14 * 24 * 3600 * 10**9  # two weeks
DRIFT = 10 * 10**9


@pytest.fixture(scope="module")
def fake():
    import commit_fixtures as F
    fb = F.FakeBackend()
    fb.real_signatures(True)
    yield fb
    fb.real_signatures(False)


def _now(blocks):
    return (blocks[-1].signed_header.header.time[0] + 5, 0)


def _corrupt(commit: H.Commit, i: int):
    s = commit.signatures[i]
    b = bytearray(s.signature)
    b[5] ^= 1
    commit.signatures[i] = H.CommitSig(s.block_id_flag, s.validator_address, s.timestamp, bytes(b))


def test_factory_headers_hash_to_block_ids():
    trusted, blocks = make_light_chain(4, 5)
    for lb in [trusted] + blocks:
        sh = lb.signed_header
        assert header_hash(sh.header) == sh.commit.block_id.hash
        assert L.header_hash(CF.header(sh.header)) == sh.commit.block_id.hash


def _oracle_sequential(trusted, blocks, now):
    conv = CF.OracleBlocks()
    n, err = L.verify_sequential(conv(trusted), [conv(b) for b in blocks], PERIOD, now[0] * L.NS + now[1], DRIFT)
    return n, None if err is None else (err[0], err[1], err[2].kind, err[2].text)


def _seq(fake, trusted, blocks, now, window, depth=1):
    n, err = chains.verify_sequential(None, trusted, blocks, PERIOD, now, DRIFT, window=window,
                                      verify_many=fake.light_verify_many, depth=depth)
    return n, None if err is None else (err.from_height, err.to_height, err.kind, err.reason)


@pytest.mark.parametrize("window", [1, 7, 64])
def test_sequential_ok(fake, window):
    trusted, blocks = make_light_chain(20, 8)
    now = _now(blocks)
    assert _seq(fake, trusted, blocks, now, window) == (20, None) == _oracle_sequential(trusted, blocks, now)
    for depth in (2, 3):  # windows in flight on caller threads
        assert _seq(fake, trusted, blocks, now, window, depth) == (20, None)


def test_in_order_yields_in_window_order_and_stops():
    """chains.in_order: results in window order whatever order the threads
    finish in; a consumer that stops early leaves later windows unstarted
    or discarded."""
    import threading
    import time
    started = []
    lock = threading.Lock()

    def run(w):
        with lock:
            started.append(w)
        time.sleep(0.002 * ((7 * w) % 5))  # windows finish out of order
        return w * w

    for depth in (1, 2, 4):
        assert list(chains.in_order(iter(range(20)), run, depth)) == [w * w for w in range(20)]
    started.clear()
    for r in chains.in_order(iter(range(50)), run, 3):
        if r == 16:  # window 4 "fails"
            break
    assert max(started) <= 4 + 3  # at most `depth` windows started past it


def test_in_order_propagates_a_window_error_in_order():
    """An engine error in window k surfaces when window k's result is
    consumed (earlier windows' results first), whatever the depth."""
    def run(w):
        if w == 3:
            raise RuntimeError("engine failed on window 3")
        return w

    for depth in (1, 2, 3):
        got = []
        with pytest.raises(RuntimeError, match="window 3"):
            for r in chains.in_order(iter(range(8)), run, depth):
                got.append(r)
        assert got == [0, 1, 2]


@pytest.mark.parametrize("what", ["sig", "next_vals_hash", "vals_hash", "header_field", "chain_id", "expired",
                                  "future", "time_order"])
def test_sequential_first_error_matches_oracle(fake, what):
    trusted, blocks = make_light_chain(20, 8, seed=hash(what) & 0xFFFF)
    now = _now(blocks)
    b = blocks[11].signed_header
    if what == "sig":
        _corrupt(b.commit, 2)
        _corrupt(blocks[15].signed_header.commit, 0)
    elif what == "next_vals_hash":
        blocks[6].signed_header.header.next_validators_hash = b"\x01" * 32  # header no longer hashes to its BlockID
    elif what == "vals_hash":
        blocks[9].vals = blocks[8].vals
    elif what == "header_field":
        b.header.app_hash = b"tampered"  # a correctly signed commit no longer binds the header
    elif what == "chain_id":
        b.header.chain_id = "other"
    elif what == "expired":
        now = (trusted.signed_header.header.time[0] + 5, 0)
        return _check_expired(fake, trusted, blocks, now)
    elif what == "future":
        now = (blocks[12].signed_header.header.time[0] - 30, 0)
    elif what == "time_order":
        b.header.time = blocks[10].signed_header.header.time
    for window in (1, 8, 100):
        for depth in (1, 3):
            assert _seq(fake, trusted, blocks, now, window, depth) == _oracle_sequential(trusted, blocks, now)
    n, err = _seq(fake, trusted, blocks, now, 100)
    assert err is not None and n < 20


def _check_expired(fake, trusted, blocks, now):
    got = _seq(fake, trusted, blocks, (now[0] + 10**9, 0), 16)
    assert got == _oracle_sequential(trusted, blocks, (now[0] + 10**9, 0))
    assert got[1][2] in (H.LIGHT_ERR_OLD_HEADER_EXPIRED, H.LIGHT_ERR_INVALID_HEADER)


def _provider(blocks):
    by_h = {lb.height: lb for lb in blocks}
    return lambda h: by_h[h]


@pytest.mark.parametrize("rotate,n,speculate", [(1, 30, 8), (3, 40, 8), (4, 40, 0), (4, 60, 3)])
def test_skipping_matches_oracle(fake, rotate, n, speculate):
    """verifySkipping's bisection (trace and verdict) with pivots verified in
    speculative batches equals the one-candidate-at-a-time oracle loop."""
    trusted, blocks = make_light_chain(n, 8, rotate=rotate, seed=rotate * 100 + n)
    now = _now(blocks)
    conv = CF.OracleBlocks()
    by_h = {lb.height: lb for lb in blocks}
    want = L.verify_skipping(conv(trusted), conv(blocks[-1]), lambda h: conv(by_h[h]), PERIOD,
                             now[0] * L.NS + now[1], DRIFT)
    trace, err = chains.verify_skipping(None, trusted, blocks[-1], _provider(blocks), PERIOD, now, DRIFT,
                                        speculate=speculate, verify_many=fake.light_verify_many)
    assert (trace, None if err is None else (err.from_height, err.to_height, err.kind, err.reason)) == \
        (want[0], None if want[1] is None else (want[1][0], want[1][1], want[1][2].kind, want[1][2].text))
    if rotate >= 3:
        assert trace is not None and len(trace) > 2  # the bisection had to pivot


def test_skipping_error_matches_oracle(fake):
    trusted, blocks = make_light_chain(40, 8, rotate=3, seed=5)
    now = _now(blocks)
    _corrupt(blocks[-1].signed_header.commit, 0)
    _corrupt(blocks[-1].signed_header.commit, 1)
    _corrupt(blocks[-1].signed_header.commit, 2)
    _corrupt(blocks[-1].signed_header.commit, 3)
    _corrupt(blocks[-1].signed_header.commit, 4)
    _corrupt(blocks[-1].signed_header.commit, 5)
    conv = CF.OracleBlocks()
    by_h = {lb.height: lb for lb in blocks}
    want = L.verify_skipping(conv(trusted), conv(blocks[-1]), lambda h: conv(by_h[h]), PERIOD,
                             now[0] * L.NS + now[1], DRIFT)
    trace, err = chains.verify_skipping(None, trusted, blocks[-1], _provider(blocks), PERIOD, now, DRIFT,
                                        verify_many=fake.light_verify_many)
    assert trace is None and want[0] is None
    assert (err.from_height, err.to_height, err.kind, err.reason) == \
        (want[1][0], want[1][1], want[1][2].kind, want[1][2].text)


def _fake_commits(fake):
    import commit_fixtures as F
    return lambda jobs: F.fake_verify_commits(fake, jobs)


def _replay(fake, vals, blocks, last_bid, window, monkeypatch, depth=2):
    import commit_fixtures as F
    return chains.blocksync_replay(None, "test_chain_id", vals, blocks, last_bid, window=window, depth=depth,
                                   verify_commits=lambda jobs: F.fake_verify_commits(fake, jobs))


def _oracle_replay(vals, blocks, last_bid):
    """poolRoutine's per-pair checks one at a time (oracle)."""
    ov = CF.valset(vals)
    state_last = CF.block_id(last_bid)
    for i in range(len(blocks) - 1):
        first, second = blocks[i], blocks[i + 1]
        fid = CF.block_id(first.block_id)
        e = L.verify_commit_light("test_chain_id", ov, fid, first.height, CF.commit(second.last_commit))
        if e is None:
            if first.height == 1:
                e = None if not (first.last_commit and first.last_commit.signatures) else \
                    L.CommitError("initial block can't have LastCommit signatures")
            else:
                e = L.verify_commit("test_chain_id", ov, state_last, first.height - 1, CF.commit(first.last_commit))
        if e is not None:
            return i, (first.height, e.text)
        state_last = fid
    return len(blocks) - 1, None


def test_blocksync_replay_matches_oracle(fake, monkeypatch):
    vals, blocks = make_block_chain(24, 7)
    for window in (1, 5, 100):
        assert _replay(fake, vals, blocks, H.BlockID(), window, monkeypatch) == (23, None)
    assert _oracle_replay(vals, blocks, H.BlockID()) == (23, None)
    # the last signature is read only by the full check (ValidateBlock)
    _corrupt(blocks[13].last_commit, 6)
    want = _oracle_replay(vals, blocks, H.BlockID())
    assert want[1][0] == 14
    for window in (1, 5, 100):
        for depth in (1, 2, 3):
            assert _replay(fake, vals, blocks, H.BlockID(), window, monkeypatch, depth) == want


def test_blocksync_uses_stored_last_commit(fake, monkeypatch):
    """the light check reads second.LastCommit (the commit that is
    stored), not a separate copy, and the full check compares LastCommit with
    state.LastBlockID, so a wrong LastBlockID is caught."""
    import copy
    vals, blocks = make_block_chain(10, 5)
    # second.LastCommit differs from the commit the first block was built with
    blocks[5].last_commit = copy.deepcopy(blocks[5].last_commit)
    _corrupt(blocks[5].last_commit, 0)
    want = _oracle_replay(vals, blocks, H.BlockID())
    assert want[1] is not None and want[1][0] == 5
    assert _replay(fake, vals, blocks, H.BlockID(), 100, monkeypatch) == want
    # a replay starting after genesis with the wrong state.LastBlockID
    vals, blocks = make_block_chain(10, 5)
    wrong = H.BlockID(b"\x07" * 32, 1, b"\x08" * 32)
    got = _replay(fake, vals, blocks[3:], wrong, 100, monkeypatch)
    assert got[0] == 0 and got[1][0] == 4 and "wrong block ID" in got[1][1]
    assert _replay(fake, vals, blocks[3:], blocks[2].block_id, 100, monkeypatch) == (6, None)


def _failing_provider(blocks, fail):
    by_h = {lb.height: lb for lb in blocks}
    asked = []

    def get(h):
        asked.append(h)
        if h in fail:
            raise RuntimeError("provider: no light block at height %d" % h)
        return by_h[h]
    return get, asked


def test_skipping_speculative_provider_failure_is_harmless(fake):
    """A provider that fails on every height only the speculation asks for
    (the reference's bisection never requests them) leaves the trace
    unchanged."""
    trusted, blocks = make_light_chain(30, 20, rotate=1, seed=230)
    now = _now(blocks)
    conv = CF.OracleBlocks()
    by_h = {lb.height: lb for lb in blocks}
    oracle_asked = []

    def oprov(h):
        oracle_asked.append(h)
        return conv(by_h[h])
    want = L.verify_skipping(conv(trusted), conv(blocks[-1]), oprov, PERIOD, now[0] * L.NS + now[1], DRIFT)
    assert want[1] is None and len(want[0]) > 2
    prov, asked = _failing_provider(blocks, set())
    chains.verify_skipping(None, trusted, blocks[-1], prov, PERIOD, now, DRIFT, verify_many=fake.light_verify_many)
    extra = sorted(set(asked) - set(oracle_asked))
    assert extra, "the speculation asked for no pivot beyond the reference's"
    prov, _ = _failing_provider(blocks, set(extra))
    trace, err = chains.verify_skipping(None, trusted, blocks[-1], prov, PERIOD, now, DRIFT,
                                        verify_many=fake.light_verify_many)
    assert err is None and trace == want[0]


def test_skipping_required_provider_failure_matches_oracle(fake):
    """A provider error on a pivot the reference does request is returned as
    ErrVerificationFailed{verified, pivot, err} (light/client.go:706-709)."""
    trusted, blocks = make_light_chain(30, 20, rotate=1, seed=230)
    now = _now(blocks)
    conv = CF.OracleBlocks()
    by_h = {lb.height: lb for lb in blocks}
    oracle_asked = []

    def oprov(h):
        oracle_asked.append(h)
        return conv(by_h[h])
    L.verify_skipping(conv(trusted), conv(blocks[-1]), oprov, PERIOD, now[0] * L.NS + now[1], DRIFT)
    bad = oracle_asked[len(oracle_asked) // 2]

    def oprov_bad(h):
        if h == bad:
            raise RuntimeError("provider: no light block at height %d" % h)
        return conv(by_h[h])
    want = L.verify_skipping(conv(trusted), conv(blocks[-1]), oprov_bad, PERIOD, now[0] * L.NS + now[1], DRIFT)
    assert want[0] is None and want[1][1] == bad
    prov, _ = _failing_provider(blocks, {bad})
    trace, err = chains.verify_skipping(None, trusted, blocks[-1], prov, PERIOD, now, DRIFT,
                                        verify_many=fake.light_verify_many)
    assert trace is None
    assert (err.from_height, err.to_height, err.kind, err.reason) == \
        (want[1][0], want[1][1], want[1][2].kind, want[1][2].text)
