"""GPU parity of ValidatorSet.Hash (tmv_validator_set_hashes, SURVEY §8(f)
rank 4) against the oracle: golden sets, tree shapes around powers of two,
empty sets between others, a 10k-validator set (several passes of the tree
workgroup), mixed key kinds, edge powers, many sets in one launch, the
light-client check that uses it, and argument errors."""
import json
import os
import random

import numpy as np
import pytest

import merkle_ref as M
from tendermint_amd import _native as N
from tendermint_amd import chains
from tendermint_amd.testing.factory import make_light_chain

pytestmark = pytest.mark.gpu
GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "merkle_vectors.json")))
EDGE_POWERS = [0, 1, 127, 128, 16384, 2**31, 2**63 - 1, -1, -(2**63), 750, 10, 300]


@pytest.fixture(scope="module")
def ctx():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    c = N.Context(1)
    yield c
    c.close()


def _arrays(sets):
    n = sum(len(s) for s in sets)
    pk = np.zeros((n, 32), np.uint8)
    kind = np.zeros(n, np.uint8)
    power = np.zeros(n, np.int64)
    off = np.zeros(len(sets) + 1, np.uint32)
    i = 0
    for j, s in enumerate(sets):
        for p, k, w in s:
            pk[i] = np.frombuffer(p, np.uint8)
            kind[i], power[i] = k, w
            i += 1
        off[j + 1] = i
    return pk.reshape(-1), kind, power, off


def _random_set(rng, n):
    return [(bytes(rng.randrange(256) for _ in range(32)), rng.randrange(2),
             rng.choice(EDGE_POWERS) if rng.randrange(4) == 0 else rng.randrange(1, 1 << 40)) for _ in range(n)]


def _check(ctx, sets):
    got = ctx.validator_set_hashes(*_arrays(sets))
    for j, s in enumerate(sets):
        assert bytes(got[j]) == M.validator_set_hash(s), (j, len(s))


def test_golden_sets(ctx):
    sv = GOLD["simple_validator"]
    sets = [[(bytes.fromhex(sv[i]["pk"]), sv[i]["kind"], sv[i]["power"]) for i in s["members"]] for s in GOLD["valsets"]]
    got = ctx.validator_set_hashes(*_arrays(sets))
    assert [bytes(g).hex() for g in got] == [s["hash"] for s in GOLD["valsets"]]


def test_every_edge_power_and_kind(ctx):
    sets = [[(bytes([i]) * 32, k, p)] for i, p in enumerate(EDGE_POWERS) for k in (0, 1)]
    _check(ctx, sets)


def test_tree_shapes_and_empty_sets(ctx):
    rng = random.Random(1)
    sizes = [0, 1, 2, 3, 4, 5, 7, 8, 9, 15, 16, 17, 31, 32, 33, 63, 64, 65, 100, 127, 128, 129, 175, 255, 256, 257,
             511, 512, 513, 0, 1000]
    _check(ctx, [_random_set(rng, n) for n in sizes])


def test_only_empty_sets(ctx):
    got = ctx.validator_set_hashes(np.zeros(0, np.uint8), np.zeros(0, np.uint8), np.zeros(0, np.int64),
                                   np.zeros(4, np.uint32))
    assert all(bytes(g).hex() == GOLD["empty_valset"] for g in got) and len(got) == 3


def test_large_set(ctx):
    _check(ctx, [_random_set(random.Random(2), 10_000)])


def test_many_sets_one_launch(ctx):
    rng = random.Random(4)
    sets = [_random_set(rng, rng.choice([100, 150, 175])) for _ in range(400)]
    got = ctx.validator_set_hashes(*_arrays(sets))
    for j in range(0, 400, 37):
        assert bytes(got[j]) == M.validator_set_hash(sets[j])


def test_argument_errors(ctx):
    pk, kind, power, off = _arrays([_random_set(random.Random(5), 3)])
    bad = kind.copy()
    bad[1] = 2  # secp256k1: not supported
    with pytest.raises(N.NativeError):
        ctx.validator_set_hashes(pk, bad, power, off)
    with pytest.raises(N.NativeError):
        ctx.validator_set_hashes(pk, kind, power, np.array([1, 3], np.uint32))
    with pytest.raises(N.NativeError):
        ctx.validator_set_hashes(pk, kind, power, np.array([0, 3, 2], np.uint32))


def test_light_client_checks_supplied_set(ctx):
    trusted, blocks = make_light_chain(12, 20)
    period, now = 10**15, (blocks[-1].signed_header.header.time[0] + 1, 0)
    n, err = chains.verify_sequential(ctx, trusted, blocks, period, now)
    assert err is None and n == 12
    # a supplied set that does not hash to the header's ValidatorsHash
    vals = blocks[6].vals
    v0 = vals.validators[0]
    vals.validators[0] = type(v0)(v0.address, v0.pub_key, v0.voting_power + 1, v0.key_kind, v0.proposer_priority)
    n, err = chains.verify_sequential(ctx, trusted, blocks, period, now)
    assert n == 6 and err.reason.startswith("invalid header: expected new header validators (")
    assert err.reason.endswith("at height %d" % blocks[6].height)
