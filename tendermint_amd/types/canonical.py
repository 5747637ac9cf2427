"""Canonical vote sign-bytes (the message M every commit signature covers).

Restates, byte for byte:
  * types/vote.go:149-157            VoteSignBytes = MarshalDelimited(CanonicalizeVote)
  * types/canonical.go:18-66         CanonicalizeBlockID / CanonicalizeVote
  * types/block.go:836-862           Commit.GetVote / Commit.VoteSignBytes
  * proto/tendermint/types/canonical.pb.go:590-640, :443-501  field order + omission
  * internal/libs/protoio/writer.go:94-134  uvarint length prefix
Pinned by the six known-answer vectors of types/vote_test.go:81-179
(tests/golden/signbytes_vectors.json).

Layout: uvarint(L) || [08 type] || [11 h:8] || [19 r:8]
|| [22 len {0a 20 hash || 12 len {08 total || 12 20 psh}}] || 2a len {08 secs
|| 10 nanos} || [32 len chain_id]; zero fields omitted, timestamp always
present, block_id omitted when the BlockID is nil.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass
from typing import Optional

PREVOTE_TYPE = 1
PRECOMMIT_TYPE = 2
PROPOSAL_TYPE = 32

# Go's zero time.Time: 0001-01-01T00:00:00Z
ZERO_TIME_SECS = -62135596800


def uvarint(x: int) -> bytes:
    """Protobuf varint of a uint64 (negative int64 -> two's complement, 10 bytes)."""
    x &= (1 << 64) - 1
    out = bytearray()
    while x >= 0x80:
        out.append((x & 0x7F) | 0x80)
        x >>= 7
    out.append(x)
    return bytes(out)


@dataclass(frozen=True)
class PartSetHeader:
    total: int = 0
    hash: bytes = b""

    def is_zero(self) -> bool:
        return self.total == 0 and len(self.hash) == 0


@dataclass(frozen=True)
class BlockID:
    hash: bytes = b""
    part_set_header: PartSetHeader = PartSetHeader()

    def is_nil(self) -> bool:  # types/block.go:1398-1401
        return len(self.hash) == 0 and self.part_set_header.is_zero()

    def is_complete(self) -> bool:  # types/block.go:1404-1408
        return len(self.hash) == 32 and self.part_set_header.total > 0 and len(self.part_set_header.hash) == 32


@dataclass(frozen=True)
class Timestamp:
    """google.protobuf.Timestamp as gogoproto stdtime encodes it."""
    seconds: int = ZERO_TIME_SECS
    nanos: int = 0


def _canonical_part_set_header(psh: PartSetHeader) -> bytes:
    out = b""
    if psh.total != 0:
        out += b"\x08" + uvarint(psh.total)
    if psh.hash:
        out += b"\x12" + uvarint(len(psh.hash)) + psh.hash
    return out


def _canonical_block_id(bid: BlockID) -> bytes:
    out = b""
    if bid.hash:
        out += b"\x0a" + uvarint(len(bid.hash)) + bid.hash
    psh = _canonical_part_set_header(bid.part_set_header)
    out += b"\x12" + uvarint(len(psh)) + psh
    return out


def _timestamp(ts: Timestamp) -> bytes:
    out = b""
    if ts.seconds != 0:
        out += b"\x08" + uvarint(ts.seconds)
    if ts.nanos != 0:
        out += b"\x10" + uvarint(ts.nanos)
    return out


def canonical_vote_head(vtype: int, height: int, round_: int, block_id: Optional[BlockID]) -> bytes:
    """The CanonicalVote fields before the timestamp (type, height, round,
    block ID): the part every vote of one commit shares."""
    out = b""
    if vtype != 0:
        out += b"\x08" + uvarint(vtype)
    if height != 0:
        out += b"\x11" + struct.pack("<q", height)
    if round_ != 0:
        out += b"\x19" + struct.pack("<q", round_)
    if block_id is not None and not block_id.is_nil():
        cb = _canonical_block_id(block_id)
        out += b"\x22" + uvarint(len(cb)) + cb
    return out


def canonical_vote(chain_id: str, vtype: int, height: int, round_: int, block_id: Optional[BlockID],
                   timestamp: Timestamp) -> bytes:
    """Proto encoding of CanonicalVote (no length prefix)."""
    out = canonical_vote_head(vtype, height, round_, block_id)
    ts = _timestamp(timestamp)
    out += b"\x2a" + uvarint(len(ts)) + ts
    cid = chain_id.encode()
    if cid:
        out += b"\x32" + uvarint(len(cid)) + cid
    return out


def vote_sign_bytes(chain_id: str, vtype: int, height: int, round_: int, block_id: Optional[BlockID],
                    timestamp: Timestamp) -> bytes:
    """types.VoteSignBytes: MarshalDelimited(CanonicalizeVote(chainID, vote))."""
    body = canonical_vote(chain_id, vtype, height, round_, block_id, timestamp)
    return uvarint(len(body)) + body
