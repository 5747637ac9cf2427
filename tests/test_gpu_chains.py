"""Cross-commit batching drivers (tendermint_amd/chains.py) on the MI355X:
light-client sequential and skipping verification and blocksync replay
return what the reference's one-header-at-a-time loops return (the oracle,
oracle/light_ref.py, at sizes it finishes quickly; at BASELINE C3 / C4 sizes
the failing header / block is re-checked by the oracle alone)."""
import pytest

import chain_fixtures as CF
import light_ref as L
from tendermint_amd import chains, host as H
from tendermint_amd.testing.factory import make_block_chain, make_light_chain

pytestmark = pytest.mark.gpu

PERIOD = 14 * 24 * 3600 * 10**9
DRIFT = 10 * 10**9


def _corrupt(commit: H.Commit, i: int):
    s = commit.signatures[i]
    b = bytearray(s.signature)
    b[5] ^= 1
    commit.signatures[i] = H.CommitSig(s.block_id_flag, s.validator_address, s.timestamp, bytes(b))


def _now(blocks):
    return (blocks[-1].signed_header.header.time[0] + 5, 0)


def _oracle_sequential(trusted, blocks, now):
    conv = CF.OracleBlocks()
    n, err = L.verify_sequential(conv(trusted), [conv(b) for b in blocks], PERIOD, now[0] * L.NS + now[1], DRIFT)
    return n, None if err is None else (err[0], err[1], err[2].kind, err[2].text)


def _seq(ctx, trusted, blocks, now, window):
    n, err = chains.verify_sequential(ctx, trusted, blocks, PERIOD, now, DRIFT, window=window)
    return n, None if err is None else (err.from_height, err.to_height, err.kind, err.reason)


def test_light_sequential_vs_oracle(ctx):
    trusted, blocks = make_light_chain(30, 12)
    now = _now(blocks)
    assert _seq(ctx, trusted, blocks, now, 16) == (30, None) == _oracle_sequential(trusted, blocks, now)
    _corrupt(blocks[17].signed_header.commit, 3)
    _corrupt(blocks[25].signed_header.commit, 1)
    blocks[21].signed_header.header.app_hash = b"tampered"
    for window in (1, 8, 64):
        assert _seq(ctx, trusted, blocks, now, window) == _oracle_sequential(trusted, blocks, now)


def test_light_skipping_vs_oracle(ctx):
    trusted, blocks = make_light_chain(48, 10, rotate=3, seed=77)
    now = _now(blocks)
    conv = CF.OracleBlocks()
    by_h = {lb.height: lb for lb in blocks}
    want = L.verify_skipping(conv(trusted), conv(blocks[-1]), lambda h: conv(by_h[h]), PERIOD,
                             now[0] * L.NS + now[1], DRIFT)
    trace, err = chains.verify_skipping(ctx, trusted, blocks[-1], lambda h: by_h[h], PERIOD, now, DRIFT)
    assert err is None and want[1] is None and trace == want[0] and len(trace) > 2


def test_c3_light_sequential_1000_headers_x_100_vals(ctx):
    """BASELINE C3 shape (light/helpers_test.go:165-216: power 2, one key
    rotated per height, round 1) at 1,000 headers x 100 validators in windows
    of 500: the clean chain verifies; with a corrupted signature inside the
    2/3 prefix of header 700 and a tampered header at 850 the first error is
    the one the oracle's VerifyAdjacent gives for header 700 alone."""
    trusted, blocks = make_light_chain(1000, 100)
    now = _now(blocks)
    assert _seq(ctx, trusted, blocks, now, 500) == (1000, None)
    _corrupt(blocks[700].signed_header.commit, 10)
    blocks[850].signed_header.header.app_hash = b"x"
    n, err = _seq(ctx, trusted, blocks, now, 500)
    conv = CF.OracleBlocks()
    e = L.verify_adjacent(conv(blocks[699]).signed_header, conv(blocks[700]).signed_header, conv(blocks[700]).vals,
                          PERIOD, now[0] * L.NS + now[1], DRIFT)
    assert n == 700 and err == (blocks[699].height, blocks[700].height, e.kind, e.text)
    assert e.kind == L.INVALID_HEADER and "wrong signature (#10)" in e.text


def _oracle_commit_error(vals, bid, height, commit, full=True):
    f = L.verify_commit if full else L.verify_commit_light
    e = f("test_chain_id", CF.valset(vals), CF.block_id(bid), height, CF.commit(commit))
    return None if e is None else e.text


def test_c4_blocksync_1000_blocks_x_175_vals(ctx):
    """BASELINE C4 shape at 1,000 blocks x 175 validators, windows of 600
    (the pool's look-ahead): the chain applies; a signature outside the light
    2/3 prefix of block 500's LastCommit fails only the full check
    (ValidateBlock), with the oracle's error text for that commit."""
    vals, blocks = make_block_chain(1000, 175)
    assert chains.blocksync_replay(ctx, "test_chain_id", vals, blocks, H.BlockID()) == (999, None)
    _corrupt(blocks[500].last_commit, 170)
    applied, err = chains.blocksync_replay(ctx, "test_chain_id", vals, blocks, H.BlockID())
    want = _oracle_commit_error(vals, blocks[499].block_id, blocks[499].height, blocks[500].last_commit)
    assert want is not None and want.startswith("wrong signature (#170)")
    assert applied == 500 and err == (blocks[500].height, want)
    assert _oracle_commit_error(vals, blocks[499].block_id, blocks[499].height, blocks[500].last_commit,
                                full=False) is None


def test_blocksync_replay_small_vs_oracle(ctx):
    vals, blocks = make_block_chain(40, 9)
    assert chains.blocksync_replay(ctx, "test_chain_id", vals, blocks, H.BlockID(), window=16) == (39, None)
    _corrupt(blocks[20].last_commit, 0)
    applied, err = chains.blocksync_replay(ctx, "test_chain_id", vals, blocks, H.BlockID(), window=16)
    want = _oracle_commit_error(vals, blocks[19].block_id, blocks[19].height, blocks[20].last_commit, full=False)
    assert applied == 19 and err == (blocks[19].height, want)
