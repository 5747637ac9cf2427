"""The CPU oracle pinned against every golden vector and independent source
(RFC 8032 via OpenSSL, hashlib, merlin/Ristretto published vectors, ZIP-215
small-order matrix, the reference's sign-bytes KATs)."""
import hashlib
import os

import numpy as np
import pytest

import ed25519_ref as E
import sr25519_ref as S
import oracle_c as C
import openssl_ed25519 as O


def _ents(vs):
    return [(bytes.fromhex(v["pk"]), bytes.fromhex(v["msg"]), bytes.fromhex(v["sig"])) for v in vs]


def test_rfc8032_vectors(golden):
    for v in golden("ed25519_rfc8032.json")["vectors"]:
        seed = bytes.fromhex(v["seed"])
        assert E.public_key(seed).hex() == v["pk"]
        assert E.sign(seed, bytes.fromhex(v["msg"])).hex() == v["sig"]
        assert E.verify_zip215(bytes.fromhex(v["pk"]), bytes.fromhex(v["msg"]), bytes.fromhex(v["sig"]))
        assert C.ed25519_verify(bytes.fromhex(v["pk"]), bytes.fromhex(v["msg"]), bytes.fromhex(v["sig"]))


def test_rfc8032_test1_literal():
    # RFC 8032 section 7.1 TEST 1 (public, well-known)
    seed = bytes.fromhex("9d61b19deffd5a60ba844af492ec2cc44449c5697b326919703bac031cae7f60")
    assert E.public_key(seed).hex() == "d75a980182b10ab7d54bfed3c964073a0ee172f3daa62325af021a68f707511a"
    assert E.sign(seed, b"").hex().startswith("e5564300c360ac729086e2cc806e828a84877f1eb8e5d974")


@pytest.mark.skipif(not O.available(), reason="no libcrypto")
def test_python_oracle_matches_openssl_on_honest_and_flips():
    rng = np.random.default_rng(1)
    for i in range(40):
        seed = rng.bytes(32)
        m = rng.bytes(int(rng.integers(0, 300)))
        pk, sig = O.public_key(seed), O.sign(seed, m)
        assert sig == E.sign(seed, m)
        assert E.verify_zip215(pk, m, sig) and O.verify_strict(pk, m, sig)
        b = bytearray(sig)
        b[int(rng.integers(64))] ^= 1 << int(rng.integers(8))
        assert E.verify_zip215(pk, m, bytes(b)) == O.verify_strict(pk, m, bytes(b)) == False  # noqa: E712


def test_golden_ed25519_vectors_python_and_c(golden):
    vs = golden("ed25519_vectors.json")["vectors"]
    ents = _ents(vs)
    py = [E.verify_zip215(*e) for e in ents]
    assert py == [v["valid"] for v in vs]
    ok, vec = C.ed25519_verify_packed(*C.pack(ents), threads=2)
    assert [bool(x) for x in vec] == py and ok == all(py)


def test_zip215_small_order_matrix(golden):
    g = golden("zip215_small_order.json")
    encs = [e.hex() for e in E.small_order_encodings()]
    assert sorted(encs) == sorted(g["encodings"]) and len(encs) == 14
    msg = bytes.fromhex(g["msg"])
    ents = [(bytes.fromhex(a), msg, bytes.fromhex(r) + bytes(32)) for a, r in g["pairs_all_valid_with_S0"]]
    assert len(ents) == 196
    ok, vec = C.ed25519_verify_packed(*C.pack(ents))
    assert ok and vec.all()


def test_sha512_and_scalar_reduce():
    rng = np.random.default_rng(2)
    for n in (0, 1, 111, 112, 127, 128, 129, 255, 256, 1000):
        m = rng.bytes(n)
        assert C.sha512(m) == hashlib.sha512(m).digest()


def test_keccak_pinned_to_sha3():
    rng = np.random.default_rng(3)
    for n in (0, 1, 135, 136, 137, 500):
        m = rng.bytes(n)
        assert S.sha3_256_via_keccak(m) == hashlib.sha3_256(m).digest()


def test_merlin_and_ristretto_published_vectors(golden):
    g = golden("sr25519_vectors.json")
    t = S.Transcript(b"test protocol")
    t.append_message(b"some label", b"some data")
    assert t.challenge_bytes(b"challenge", 32).hex() == g["merlin_test_protocol"]
    assert C.merlin_test_vector().hex() == g["merlin_test_protocol"]
    # RFC 9496 A.1: multiples of the ristretto255 generator
    assert g["ristretto_multiples"][1] == "e2f2ae0a6abc4e71a884a961c500515f58e30b6aa582dd8db6a65945e08d2d76"
    assert g["ristretto_multiples"][2] == "6a493210f7499cd17fecb510ae0cea23a110e8d5b901f8acadd3095c73a3b919"
    for i, enc in enumerate(g["ristretto_multiples"]):
        assert S.ristretto_encode(E.pt_mul(i, E.BASE)).hex() == enc
        if i:
            assert S.ristretto_equal(S.ristretto_decode(bytes.fromhex(enc)), E.pt_mul(i, E.BASE))


def test_golden_sr25519_python_and_c(golden):
    vs = golden("sr25519_vectors.json")["vectors"]
    ents = _ents(vs)
    st = C.sr25519_status_packed(*C.pack(ents), threads=2)
    assert [int(x) for x in st] == [v["status"] for v in vs]
    for v, e in zip(vs, ents):
        assert S.verify(*e) == (v["status"] == 1)


def test_c2_expected_vector(golden):
    from tendermint_amd.testing.factory import make_c2_batch
    g = golden("c2_expected.json")
    b = make_c2_batch()
    h = hashlib.sha256()
    for a in (b.pk, b.sig, b.msg, b.off):
        h.update(a.tobytes())
    assert h.hexdigest() == g["inputs_sha256"], "C2 generator drifted"
    ok, vec = C.ed25519_verify_packed(b.pk, b.sig, b.msg, b.off, threads=os.cpu_count() or 1)
    bits = np.packbits(vec.astype(np.uint8), bitorder="little").tobytes().hex()
    assert bits == g["valid_bits_hex"] and int(vec.sum()) == g["valid_count"] == 9950


def test_empty_batch_is_false():
    assert E.batch_verify([]) == (False, [])
    assert S.batch_verify([]) == (False, [])
    ok, vec = C.ed25519_verify_packed(np.zeros(0, np.uint8), np.zeros(0, np.uint8), np.zeros(0, np.uint8),
                                      np.zeros(1, np.uint32))
    assert ok is False and len(vec) == 0


def test_cpu_batch_verifier_matches_per_entry():
    """oracle/c/ed25519_batch_cpu.c (bench.py's cpu_baseline: voi's batch
    algorithm restated in C) gives the per-entry vector: honest batches pass
    their equation (no fallback), batches with edge cases fall back and still
    match, small-order ZIP-215 entries included."""
    import oracle_c as C
    from tendermint_amd.testing.factory import make_c2_batch, make_commit_batch
    h = make_commit_batch(300)
    ok, v, failed = C.ed25519_batch_verify_voi(h.pk, h.sig, h.msg, h.off, threads=2, batch=64)
    assert ok and v.all() and failed == 0
    c = make_c2_batch(1200, seed=77, edge_scale=3.0)
    _, ref = C.ed25519_verify_packed(c.pk, c.sig, c.msg, c.off, threads=4)
    for batch in (1, 50, 1200):
        ok, v, failed = C.ed25519_batch_verify_voi(c.pk, c.sig, c.msg, c.off, threads=3, batch=batch)
        assert np.array_equal(v, ref) and not ok and failed >= 1


def test_commit_cpu_baseline_matches_oracle():
    """bench.py's C1 CPU baseline (oracle_verify_commit_cpu): the sign-bytes
    it builds are the votes' (the honest C1 commit verifies) and a corrupted
    vote is found at its index, as the per-entry oracle finds it."""
    import numpy as np

    import oracle_c
    from tendermint_amd.testing.bulk import commit_vote_head
    from tendermint_amd.testing.factory import make_c1_commit
    from tendermint_amd.types.canonical import BlockID, PartSetHeader
    vals, bid, commit = make_c1_commit(40)
    head = commit_vote_head(3, 0, BlockID(bid.hash, PartSetHeader(bid.psh_total, bid.psh_hash)))
    pk = np.frombuffer(b"".join(v.pub_key for v in vals.validators), np.uint8)
    sig = np.frombuffer(b"".join(s.signature for s in commit.signatures), np.uint8).copy()
    secs = [s.timestamp[0] for s in commit.signatures]
    nanos = [s.timestamp[1] for s in commit.signatures]
    assert oracle_c.CommitCPU(head, "test_chain_id", secs, nanos, pk, sig)()
    sig[64 * 17 + 40] ^= 4
    c = oracle_c.CommitCPU(head, "test_chain_id", secs, nanos, pk, sig)
    assert not c() and list(np.flatnonzero(c.out[:40] == 0)) == [17]
    assert not oracle_c.CommitCPU(head, "other_chain", secs, nanos, pk, sig)()
