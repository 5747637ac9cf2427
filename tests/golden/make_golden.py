#!/usr/bin/env python3
"""Generate the committed golden fixtures in tests/golden/.

Sources (no reference code is copied; these are data):
  * signbytes_vectors.json  — the six known-answer vectors of
    types/vote_test.go:81-179 (inputs + expected bytes, transcribed as data).
  * ed25519_rfc8032.json    — RFC 8032 §7.1 TEST 1-3 seeds/messages; keys and
    signatures produced by OpenSSL 3 (RFC 8032 deterministic signing, which
    voi ed25519.Sign matches byte for byte).
  * ed25519_vectors.json    — honest OpenSSL signatures, random bit flips
    (OpenSSL's strict verifier agrees with ZIP-215 on these), S+l,
    undecodable points and the ZIP-215 small-order family; expected results
    from oracle/ed25519_ref.py (Python) cross-checked with oracle/c.
  * zip215_small_order.json — the 14 small-order encodings and the 196-pair
    (A, R, S=0) matrix, all valid under ZIP-215.
  * c2_expected.json        — digest of the deterministic C2 batch (10k) and
    its expected validity vector (bit-packed), from the C oracle.
  * sr25519_vectors.json    — merlin "test protocol" vector, Ristretto255
    generator multiples 0..3, and self-signed sr25519 cases with expected
    per-entry status (parity with voi unpinned beyond the merlin/Ristretto
    vectors).
Run from the repo root: python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))

import numpy as np  # noqa: E402
import ed25519_ref as E  # noqa: E402
import sr25519_ref as S  # noqa: E402
import openssl_ed25519 as O  # noqa: E402
import oracle_c as C  # noqa: E402
from tendermint_amd.testing.factory import make_c2_batch, undecodable_encodings  # noqa: E402


def dump(name, obj):
    with open(os.path.join(HERE, name), "w") as f:
        json.dump(obj, f, indent=1, sort_keys=True)
        f.write("\n")


def signbytes():
    zero_ts = "0b088092b8c398feffffff01"  # timestamp of Go's zero time.Time
    vecs = [
        {"chain_id": "", "type": 0, "height": 0, "round": 0,
         "want": "0d2a" + zero_ts},
        {"chain_id": "", "type": 2, "height": 1, "round": 1,
         "want": "21" "0802" "110100000000000000" "190100000000000000" "2a" + zero_ts},
        {"chain_id": "", "type": 1, "height": 1, "round": 1,
         "want": "21" "0801" "110100000000000000" "190100000000000000" "2a" + zero_ts},
        {"chain_id": "", "type": 0, "height": 1, "round": 1,
         "want": "1f" "110100000000000000" "190100000000000000" "2a" + zero_ts},
        {"chain_id": "test_chain_id", "type": 0, "height": 1, "round": 1,
         "want": "2e" "110100000000000000" "190100000000000000" "2a" + zero_ts + "320d" + b"test_chain_id".hex()},
        {"chain_id": "test_chain_id", "type": 0, "height": 1, "round": 1, "extension": "extension",
         "want": "2e" "110100000000000000" "190100000000000000" "2a" + zero_ts + "320d" + b"test_chain_id".hex()},
    ]
    for v in vecs:
        v["timestamp"] = [-62135596800, 0]
        v["block_id"] = None
    dump("signbytes_vectors.json", {"source": "types/vote_test.go:81-179 TestVoteSignBytesTestVectors",
                                    "vectors": vecs})


def rfc8032():
    cases = [("9d61b19deffd5a60ba844af492ec2cc44449c5697b326919703bac031cae7f60", ""),
             ("4ccd089b28ff96da9db6c346ec114e0f5b8a319f35aba624da8cf6ed4fb8a6fb", "72"),
             ("c5aa8df43f9f837bedb7442f31dcb7b166d38535076f094b85ce3a2e0b4458f7", "af82")]
    out = []
    for seed, msg in cases:
        sd, m = bytes.fromhex(seed), bytes.fromhex(msg)
        pk, sig = O.public_key(sd), O.sign(sd, m)
        assert pk == E.public_key(sd) and sig == E.sign(sd, m) and E.verify_zip215(pk, m, sig)
        out.append({"seed": seed, "pk": pk.hex(), "msg": msg, "sig": sig.hex(), "valid": True})
    dump("ed25519_rfc8032.json", {"source": "RFC 8032 7.1 TEST 1-3 via OpenSSL 3", "vectors": out})


def ed25519_vectors():
    rng = random.Random(0x215)
    out = []
    undec = undecodable_encodings(8, rng)
    encs = E.small_order_encodings()
    for i in range(96):
        sd = hashlib.sha256(b"golden %d" % i).digest()
        m = bytes(rng.randrange(256) for _ in range(rng.randrange(0, 260)))
        pk, sig = O.public_key(sd), O.sign(sd, m)
        kind = ["honest", "flip_r", "flip_s", "flip_m", "s_plus_l", "undec_a", "undec_r", "small_order"][i % 8]
        if kind == "flip_r":
            b = bytearray(sig); b[rng.randrange(32)] ^= 1 << rng.randrange(8); sig = bytes(b)
        elif kind == "flip_s":
            b = bytearray(sig); b[32 + rng.randrange(31)] ^= 1 << rng.randrange(8); sig = bytes(b)
        elif kind == "flip_m":
            b = bytearray(m or b"\0"); b[rng.randrange(len(b))] ^= 1 << rng.randrange(8); m = bytes(b)
        elif kind == "s_plus_l":
            sig = sig[:32] + (int.from_bytes(sig[32:], "little") + E.L).to_bytes(32, "little")
        elif kind == "undec_a":
            pk = undec[i % len(undec)]
        elif kind == "undec_r":
            sig = undec[(i + 3) % len(undec)] + sig[32:]
        elif kind == "small_order":
            pk, sig = rng.choice(encs), rng.choice(encs) + bytes(32)
        v = E.verify_zip215(pk, m, sig)
        rec = {"kind": kind, "pk": pk.hex(), "msg": m.hex(), "sig": sig.hex(), "valid": v}
        if kind in ("honest", "flip_r", "flip_s", "flip_m"):
            rec["openssl_strict"] = O.verify_strict(pk, m, sig)
            assert rec["openssl_strict"] == v
        out.append(rec)
    ents = [(bytes.fromhex(r["pk"]), bytes.fromhex(r["msg"]), bytes.fromhex(r["sig"])) for r in out]
    _, vec = C.ed25519_verify_packed(*C.pack(ents))
    assert [bool(x) for x in vec] == [r["valid"] for r in out]
    dump("ed25519_vectors.json", {"source": "OpenSSL-signed + oracle/ed25519_ref.py (ZIP-215)", "vectors": out})


def zip215():
    encs = E.small_order_encodings()
    matrix = []
    for a in encs:
        for r in encs:
            ok = E.verify_zip215(a, b"Zcash", r + bytes(32))
            assert ok
            matrix.append([a.hex(), r.hex()])
    dump("zip215_small_order.json", {"source": "SURVEY Appendix D; oracle/ed25519_ref.py",
                                     "encodings": [e.hex() for e in encs], "msg": b"Zcash".hex(),
                                     "pairs_all_valid_with_S0": matrix})


def c2():
    b = make_c2_batch()
    _, vec = C.ed25519_verify_packed(b.pk, b.sig, b.msg, b.off, threads=8)
    h = hashlib.sha256()
    for a in (b.pk, b.sig, b.msg, b.off):
        h.update(a.tobytes())
    # spot-check a slice with the independent Python oracle
    for i in range(0, b.n, 97):
        assert E.verify_zip215(*b.entry(i)) == bool(vec[i])
    dump("c2_expected.json", {"source": "tendermint_amd.testing.factory.make_c2_batch() + oracle/c",
                              "n": b.n, "inputs_sha256": h.hexdigest(), "valid_count": int(vec.sum()),
                              "valid_bits_hex": np.packbits(vec.astype(np.uint8), bitorder="little").tobytes().hex()})


def sr25519():
    t = S.Transcript(b"test protocol")
    t.append_message(b"some label", b"some data")
    merlin = t.challenge_bytes(b"challenge", 32).hex()
    assert merlin == "d5a21972d0d5fe320c0d263fac7fffb8145aa640af6e9bca177c03c7efcf0615"
    multiples = [S.ristretto_encode(E.pt_mul(i, E.BASE)).hex() for i in range(4)]
    rng = random.Random(0x5125519)
    out = []
    for i in range(48):
        mini = S.key_from_secret(b"key: %x" % i)
        pk = S.public_key(mini)
        m = bytes(rng.randrange(256) for _ in range(rng.randrange(0, 200)))
        sig = S.sign(mini, m, nonce_seed=b"%d" % i)
        kind = ["honest", "flip_r", "flip_s", "flip_m", "no_marker", "s_noncanon", "bad_pk", "bad_r"][i % 8]
        if kind == "flip_r":
            b = bytearray(sig); b[rng.randrange(32)] ^= 1 << rng.randrange(8); sig = bytes(b)
        elif kind == "flip_s":
            b = bytearray(sig); b[32 + rng.randrange(31)] ^= 1 << rng.randrange(8); sig = bytes(b)
        elif kind == "flip_m":
            b = bytearray(m or b"\0"); b[rng.randrange(len(b))] ^= 1 << rng.randrange(8); m = bytes(b)
        elif kind == "no_marker":
            b = bytearray(sig); b[63] &= 0x7F; sig = bytes(b)
        elif kind == "s_noncanon":
            s = (int.from_bytes(sig[32:], "little") & ((1 << 255) - 1)) + E.L
            b = bytearray(s.to_bytes(32, "little")); b[31] |= 0x80; sig = sig[:32] + bytes(b)
        elif kind == "bad_pk":
            pk = (int.from_bytes(pk, "little") | 1).to_bytes(32, "little")  # negative s -> invalid
        elif kind == "bad_r":
            sig = (int.from_bytes(sig[:32], "little") | 1).to_bytes(32, "little") + sig[32:]
        try:
            S.batch_add_check(pk, sig)
            status = 1 if S.verify(pk, m, sig) else 0
        except S.AddError as e:
            status = -1 if "public key" in str(e) else -2
        out.append({"kind": kind, "pk": pk.hex(), "msg": m.hex(), "sig": sig.hex(), "status": status})
    ents = [(bytes.fromhex(r["pk"]), bytes.fromhex(r["msg"]), bytes.fromhex(r["sig"])) for r in out]
    st = C.sr25519_status_packed(*C.pack(ents))
    assert [int(x) for x in st] == [r["status"] for r in out]
    dump("sr25519_vectors.json", {"source": "oracle/sr25519_ref.py (self-signed; parity with voi unpinned)",
                                  "merlin_test_protocol": merlin, "ristretto_multiples": multiples,
                                  "vectors": out})


if __name__ == "__main__":
    C.build()
    signbytes()
    rfc8032()
    ed25519_vectors()
    zip215()
    c2()
    sr25519()
    print("golden fixtures written to", HERE)
