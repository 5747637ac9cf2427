"""Vote templates and timestamps for the device sign-bytes path
(tmv_verify_votes): random and edge-case CanonicalVote fields, the Python
restatement of the template assembly (include/tmverify.h), and the expected
message from the sign-bytes mirror pinned by the reference's KAT vectors
(types/vote_test.go:81-179, tests/test_signbytes.py)."""
from __future__ import annotations

import random

import numpy as np

from tendermint_amd import _native as N
from tendermint_amd import host as H
from tendermint_amd.types.canonical import BlockID, PartSetHeader, Timestamp, uvarint, vote_sign_bytes

# (seconds, nanos): zero fields omitted, Go's zero time, negative values
# (10-byte varints), int64 / int32 extremes, varint length boundaries
EDGE_TS = [(0, 0), (0, 1), (1, 0), (-62135596800, 0), (-1, -1), (2**63 - 1, 999_999_999), (-2**63, -2**31),
           (1577836800, 10**9 - 1), (127, 127), (128, 128), (16383, 16384), (2**31 - 1, 2**31 - 1)]
CHAIN_IDS = ["", "c", "test_chain_id", "x" * 127, "y" * 128, "z" * 300]
HEIGHTS = [0, 1, -1, 2**63 - 1, -2**63, 3]
ROUNDS = [0, 1, -1, 2**31 - 1, -2**31]


def _rb(rng: random.Random, n: int) -> bytes:
    return bytes(rng.randrange(256) for _ in range(n))


def random_block_id(rng: random.Random):
    k = rng.randrange(7)
    if k == 0:
        return None
    if k == 1:
        return BlockID()                                     # nil: field 4 omitted
    if k == 2:
        return BlockID(_rb(rng, 32), PartSetHeader())        # hash only
    if k == 3:
        return BlockID(b"", PartSetHeader(rng.randrange(1, 1 << 32), b""))
    if k == 4:
        return BlockID(b"", PartSetHeader(0, _rb(rng, rng.randrange(1, 200))))
    return BlockID(_rb(rng, 32), PartSetHeader(rng.randrange(1, 1 << 32), _rb(rng, 32)))


def random_template(rng: random.Random) -> dict:
    return dict(chain_id=rng.choice(CHAIN_IDS + ["test_chain_id"] * 3),
                vtype=rng.choice([2, 2, 2, 1, 0, 32]),
                height=rng.choice(HEIGHTS + [rng.randrange(1, 1 << 40)] * 3),
                round_=rng.choice(ROUNDS + [0] * 3),
                block_id=random_block_id(rng))


def random_ts(rng: random.Random):
    if rng.randrange(4) == 0:
        return rng.choice(EDGE_TS)
    return 1577836800 + rng.randrange(1 << 30), rng.randrange(10**9)


def host_block_id(b):
    return None if b is None else H.BlockID(b.hash, b.part_set_header.total, b.part_set_header.hash)


def segments(t: dict, lib=None):
    """(head, block, chain) through the product's C++ template encoder."""
    return H.vote_template(t["chain_id"], t["vtype"], t["height"], t["round_"], host_block_id(t["block_id"]), lib=lib)


def assemble(seg, with_block: bool, ts) -> bytes:
    """uvarint(len(body)) || head || [block] || 0x2a uvarint(len(ts)) ts || chain."""
    head, block, chain = seg
    secs, nanos = ts
    t = (b"\x08" + uvarint(secs) if secs else b"") + (b"\x10" + uvarint(nanos) if nanos else b"")
    body = head + (block if with_block else b"") + b"\x2a" + uvarint(len(t)) + t + chain
    return uvarint(len(body)) + body


def expected(t: dict, with_block: bool, ts) -> bytes:
    """types.VoteSignBytes of the vote (BlockIDFor: nil unless the flag is Commit)."""
    return vote_sign_bytes(t["chain_id"], t["vtype"], t["height"], t["round_"],
                           t["block_id"] if with_block else None, Timestamp(*ts))


def random_votes(rng: random.Random, n_tmpl: int, n: int):
    """Templates, a VOTE_DTYPE array and the expected messages."""
    tmpls = [random_template(rng) for _ in range(n_tmpl)]
    votes = np.zeros(n, N.VOTE_DTYPE)
    msgs = []
    for i in range(n):
        t = rng.randrange(n_tmpl)
        wb = rng.randrange(4) != 0
        ts = random_ts(rng)
        votes[i] = (ts[0], ts[1], t | (N.TMV_VOTE_WITH_BLOCK if wb else 0))
        msgs.append(expected(tmpls[t], wb, ts))
    return tmpls, votes, msgs
