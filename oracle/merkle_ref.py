"""CPU restatement of ValidatorSet.Hash (TEST INFRASTRUCTURE: the checker for
tmv_validator_set_hashes, never part of the product path).

Follows, in the reference:
  types/validator_set.go:344-350   Hash() = merkle.HashFromByteSlices(val.Bytes() for val)
  types/validator.go:154-170       Bytes() = SimpleValidator{PubKey, VotingPower}.Marshal()
  proto/tendermint/types/validator.proto:22-25, proto/tendermint/crypto/keys.proto
                                   (PublicKey oneof: ed25519 = 1, secp256k1 = 2, sr25519 = 3)
  crypto/merkle/tree.go:11-27,100-112  recursive split at the largest power of two < n
  crypto/merkle/hash.go            emptyHash / leaf 0x00 / inner 0x01 (RFC 6962)
Pinned by the reference's own vectors (crypto/merkle/tree_test.go:21-33,
crypto/merkle/rfc6962_test.go:26-66, types/validator_set_test.go:51-53) and,
for the protobuf wire encoding, by google.protobuf encoding the same
messages (tests/golden/make_merkle_golden.py).
"""
import hashlib

KIND_ED25519, KIND_SR25519 = 0, 1
_KEY_FIELD = {KIND_ED25519: 1, KIND_SR25519: 3}


def empty_hash() -> bytes:
    return hashlib.sha256(b"").digest()


def leaf_hash(leaf: bytes) -> bytes:
    return hashlib.sha256(b"\x00" + leaf).digest()


def inner_hash(left: bytes, right: bytes) -> bytes:
    return hashlib.sha256(b"\x01" + left + right).digest()


def split_point(n: int) -> int:
    """Largest power of two strictly below n (tree.go:100-112)."""
    if n < 1:
        raise ValueError("split of a tree with size < 1")
    k = 1 << (n.bit_length() - 1)
    return k >> 1 if k == n else k


def hash_from_byte_slices(items) -> bytes:
    """merkle.HashFromByteSlices (tree.go:11-27), recursive as the reference."""
    n = len(items)
    if n == 0:
        return empty_hash()
    if n == 1:
        return leaf_hash(items[0])
    k = split_point(n)
    return inner_hash(hash_from_byte_slices(items[:k]), hash_from_byte_slices(items[k:]))


def _varint(u: int) -> bytes:
    out = bytearray()
    while True:
        b = u & 0x7F
        u >>= 7
        if u:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def simple_validator_bytes(pk: bytes, kind: int, power: int) -> bytes:
    """SimpleValidator{pub_key: PublicKey{<kind>: pk}, voting_power: power}.Marshal()."""
    field = _KEY_FIELD[kind]
    pub = bytes([(field << 3) | 2, len(pk)]) + pk          # PublicKey oneof bytes
    out = bytes([(1 << 3) | 2, len(pub)]) + pub              # SimpleValidator.pub_key (always set)
    if power:                                                # proto3: zero omitted
        out += bytes([(2 << 3) | 0]) + _varint(power & ((1 << 64) - 1))
    return out


def validator_set_hash(vals) -> bytes:
    """vals: [(pk32, kind, power)] in set order."""
    return hash_from_byte_slices([simple_validator_bytes(pk, k, p) for pk, k, p in vals])
