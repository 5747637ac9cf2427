"""ValidatorSet.Hash on the CPU side: the oracle
(oracle/merkle_ref.py) against the reference's own vectors and the
protobuf-generated encodings (tests/golden/merkle_vectors.json), the
factory's generated header hashes, and the recursive split against the
pairwise (iterative) tree the kernel uses (crypto/merkle/tree.go:68-99)."""
import hashlib
import json
import os
import random

import merkle_ref as M
from tendermint_amd import host as H
from tendermint_amd.testing import factory

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "merkle_vectors.json")))


def test_reference_tree_vectors():
    for t in GOLD["tree"]:
        assert M.hash_from_byte_slices([bytes.fromhex(x) for x in t["items"]]).hex() == t["hash"], t["name"]


def test_rfc6962_vectors():
    r = GOLD["rfc6962"]
    assert M.leaf_hash(b"L123456").hex() == r["leaf_L123456"]
    assert M.leaf_hash(b"").hex() == r["empty_leaf"]
    assert M.inner_hash(b"N123", b"N456").hex() == r["inner_N123_N456"]
    assert M.empty_hash().hex() == GOLD["empty_valset"] == M.validator_set_hash([]).hex()


def test_split_points():
    for n, k in GOLD["split"]:
        assert M.split_point(n) == k


def test_simple_validator_encoding_matches_protobuf():
    for s in GOLD["simple_validator"]:
        assert M.simple_validator_bytes(bytes.fromhex(s["pk"]), s["kind"], s["power"]).hex() == s["bytes"], s


def test_valset_vectors():
    sv = GOLD["simple_validator"]
    for s in GOLD["valsets"]:
        vals = [(bytes.fromhex(sv[i]["pk"]), sv[i]["kind"], sv[i]["power"]) for i in s["members"]]
        assert M.validator_set_hash(vals).hex() == s["hash"]


def _pairwise(items):
    nodes = [M.leaf_hash(x) for x in items]
    if not nodes:
        return M.empty_hash()
    while len(nodes) > 1:
        nxt = [M.inner_hash(nodes[i], nodes[i + 1]) for i in range(0, len(nodes) - 1, 2)]
        if len(nodes) % 2:
            nxt.append(nodes[-1])
        nodes = nxt
    return nodes[0]


def test_pairwise_tree_equals_recursive_split():
    rng = random.Random(3)
    for n in list(range(0, 70)) + [100, 127, 128, 129, 175, 255, 256, 257, 1000]:
        items = [bytes(rng.randrange(256) for _ in range(rng.randrange(40))) for _ in range(n)]
        assert _pairwise(items) == M.hash_from_byte_slices(items), n


def test_factory_headers_carry_the_set_hash():
    trusted, blocks = factory.make_light_chain(3, 7)
    for lb in blocks:
        vals = [(v.pub_key, v.key_kind, v.voting_power) for v in lb.vals.validators]
        assert lb.signed_header.header.validators_hash == M.validator_set_hash(vals)
    assert isinstance(H.ValidatorSet([]).validators, list)
    assert hashlib.sha256(b"").digest() == M.validator_set_hash([])
