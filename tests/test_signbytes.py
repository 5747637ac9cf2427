"""Sign-bytes mirror vs the reference's known-answer vectors
(types/vote_test.go:81-179)."""
from tendermint_amd.types.canonical import (BlockID, PartSetHeader, Timestamp, vote_sign_bytes, uvarint,
                                            canonical_vote, PRECOMMIT_TYPE)


def test_reference_kat_vectors(golden):
    for v in golden("signbytes_vectors.json")["vectors"]:
        got = vote_sign_bytes(v["chain_id"], v["type"], v["height"], v["round"], None, Timestamp(*v["timestamp"]))
        assert got.hex() == v["want"]


def test_commit_vote_shape():
    bid = BlockID(b"\x11" * 32, PartSetHeader(1000000, b"\x22" * 32))
    m = vote_sign_bytes("test_chain_id", PRECOMMIT_TYPE, 3, 0, bid, Timestamp(1577836800, 1_000_000))
    assert 109 <= len(m) <= 125
    body = canonical_vote("test_chain_id", PRECOMMIT_TYPE, 3, 0, bid, Timestamp(1577836800, 1_000_000))
    assert m == uvarint(len(body)) + body
    assert body.startswith(b"\x08\x02\x11\x03" + b"\x00" * 7)  # round 0 omitted
    assert b"\x22" in body and body.endswith(b"\x32\x0dtest_chain_id")


def test_nil_block_id_omitted():
    m1 = vote_sign_bytes("c", PRECOMMIT_TYPE, 5, 1, BlockID(), Timestamp(10, 0))
    m2 = vote_sign_bytes("c", PRECOMMIT_TYPE, 5, 1, None, Timestamp(10, 0))
    assert m1 == m2 and b"\x22" not in m1[1:20]


def test_uvarint():
    assert uvarint(0) == b"\x00" and uvarint(300) == b"\xac\x02"
    assert uvarint(-62135596800) == bytes.fromhex("8092b8c398feffffff01")
