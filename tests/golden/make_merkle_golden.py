"""Generates tests/golden/merkle_vectors.json (run from the repo root).

* "tree", "rfc6962", "split", "empty_valset": the reference's own vectors,
  copied as data from crypto/merkle/tree_test.go:21-33,139-160,
  crypto/merkle/rfc6962_test.go:26-66 and types/validator_set_test.go:51-53.
* "simple_validator": SimpleValidator wire bytes produced by google.protobuf
  (the schema of proto/tendermint/types/validator.proto:22-25 and
  proto/tendermint/crypto/keys.proto built at run time), independent of the
  restatement in oracle/merkle_ref.py, with the validator-set hashes of
  small sets of them computed from those bytes by hashlib.
"""
import hashlib
import json
import os
import random

from google.protobuf import descriptor_pb2, descriptor_pool
try:
    from google.protobuf.message_factory import GetMessageClass
except ImportError:  # older protobuf
    from google.protobuf import message_factory
    GetMessageClass = lambda d: message_factory.MessageFactory().GetPrototype(d)  # noqa: E731

F = descriptor_pb2.FieldDescriptorProto


def _classes():
    fd = descriptor_pb2.FileDescriptorProto(name="tm_golden.proto", package="tmg", syntax="proto3")
    pk = fd.message_type.add(name="PublicKey")
    pk.oneof_decl.add(name="sum")
    for name, num in (("ed25519", 1), ("secp256k1", 2), ("sr25519", 3)):
        pk.field.add(name=name, number=num, type=F.TYPE_BYTES, label=F.LABEL_OPTIONAL, oneof_index=0)
    sv = fd.message_type.add(name="SimpleValidator")
    sv.field.add(name="pub_key", number=1, type=F.TYPE_MESSAGE, label=F.LABEL_OPTIONAL, type_name=".tmg.PublicKey")
    sv.field.add(name="voting_power", number=2, type=F.TYPE_INT64, label=F.LABEL_OPTIONAL)
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    return GetMessageClass(pool.FindMessageTypeByName("tmg.SimpleValidator"))


def _tree(items):
    n = len(items)
    if n == 0:
        return hashlib.sha256(b"").digest()
    if n == 1:
        return hashlib.sha256(b"\x00" + items[0]).digest()
    k = 1 << (n.bit_length() - 1)
    k = k >> 1 if k == n else k
    return hashlib.sha256(b"\x01" + _tree(items[:k]) + _tree(items[k:])).digest()


def main():
    SV = _classes()
    rng = random.Random(215)
    powers = [0, 1, 2, 10, 127, 128, 300, 16383, 16384, 750, 2**31 - 1, 2**31, 2**62, 2**63 - 1, -1, -10, -(2**63)]
    sv = []
    for i, p in enumerate(powers):
        kind = i % 2
        pk = bytes(rng.randrange(256) for _ in range(32))
        m = SV(voting_power=p)
        if kind == 0:
            m.pub_key.ed25519 = pk
        else:
            m.pub_key.sr25519 = pk
        sv.append({"pk": pk.hex(), "kind": kind, "power": p, "bytes": m.SerializeToString().hex()})
    sets = []
    for n in (1, 2, 3, 5, 7, 8, 9, 17):
        idx = [rng.randrange(len(sv)) for _ in range(n)]
        sets.append({"members": idx, "hash": _tree([bytes.fromhex(sv[i]["bytes"]) for i in idx]).hex()})
    out = {
        "tree": [
            {"name": "empty", "items": [], "hash": "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855"},
            {"name": "single", "items": ["010203"], "hash": "054edec1d0211f624fed0cbca9d4f9400b0e491c43742af2c5b0abebf0c990d8"},
            {"name": "single blank", "items": [""], "hash": "6e340b9cffb37a989ca544e6bb780a2c78901d3fb33738768511a30617afa01d"},
            {"name": "two", "items": ["010203", "040506"], "hash": "82e6cfce00453804379b53962939eaa7906b39904be0813fcadd31b100773c4b"},
            {"name": "many", "items": ["0102", "0304", "0506", "0708", "090a"],
             "hash": "f326493eceab4f2d9ffbc78c59432a0a005d6ea98392045c74df5d14a113be18"},
        ],
        "rfc6962": {
            "leaf_L123456": "395aa064aa4c29f7010acfe3f25db9485bbd4b91897b6ad7ad547639252b4d56",
            "empty_leaf": "6e340b9cffb37a989ca544e6bb780a2c78901d3fb33738768511a30617afa01d",
            "inner_N123_N456": "aa217fe888e47007fa15edab33c2b492a722cb106c64667fc2b044444de66bbb",
        },
        "split": [[1, 0], [2, 1], [3, 2], [4, 2], [5, 4], [10, 8], [20, 16], [100, 64], [255, 128], [256, 128],
                  [257, 256]],
        "empty_valset": "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855",
        "simple_validator": sv,
        "valsets": sets,
    }
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "merkle_vectors.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
