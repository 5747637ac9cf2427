"""The exact device arithmetic (tendermint_amd/csrc/*.h) compiled for the
host with limb-bound assertions, checked against the oracle.  No GPU."""
import ctypes
import hashlib
import os
import subprocess

import numpy as np
import pytest

import ed25519_ref as E
import oracle_c as C

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(REPO, "oracle", "_build", "libhostcheck.so")


@pytest.fixture(scope="module")
def H():
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "tests", "native")], check=True)
    return ctypes.CDLL(SO)


def p(a, t=ctypes.c_uint8):
    return a.ctypes.data_as(ctypes.POINTER(t))


def _u8(b):
    return np.frombuffer(b, np.uint8).copy()


def test_fe_mul(H):
    rng = np.random.default_rng(5)
    for _ in range(300):
        a = int.from_bytes(rng.bytes(32), "little") >> 1
        b = int.from_bytes(rng.bytes(32), "little") >> 1
        out = np.zeros(32, np.uint8)
        H.hostcheck_fe_mul(p(_u8(a.to_bytes(32, "little"))), p(_u8(b.to_bytes(32, "little"))), p(out))
        assert int.from_bytes(out.tobytes(), "little") == a * b % E.P


def test_fe_pow_chains(H):
    """fe_pow22523 = x^((p-5)/8) and fe_invert = x^(p-2), whose fe_sqn runs
    the floor-carry squarings, against Python integers (limb bounds asserted
    in this build), on random values, 0, 1, p-1 and values >= p."""
    rng = np.random.default_rng(11)
    vals = [0, 1, 2, E.P - 1, E.P, E.P + 1, (1 << 255) - 1] + [int.from_bytes(rng.bytes(32), "little") & ((1 << 255) - 1)
                                                             for _ in range(300)]
    for v in vals:
        po = ctypes.create_string_buffer(32)
        io = ctypes.create_string_buffer(32)
        H.hostcheck_fe_pow(v.to_bytes(32, "little"), po, io)
        x = v % E.P
        assert int.from_bytes(po.raw, "little") == pow(x, (E.P - 5) // 8, E.P)
        assert int.from_bytes(io.raw, "little") == pow(x, E.P - 2, E.P)


def test_fe_mul_two_round_carry(H):
    """The quad formulas' two-round parallel carry (fe_mul_par,
    TMV_QUAD_PCARRY) encodes the same product as the twelve-step carry, over
    chains of 40 products whose inputs are pushed to level 3, from random
    limbs and from the level-3 extremes (limb bounds asserted in this build)."""
    import ctypes
    H.hostcheck_fe_mul_par.restype = ctypes.c_int
    rng = np.random.default_rng(9)
    i32 = ctypes.POINTER(ctypes.c_int32)
    cases = []
    for _ in range(300):
        lim = np.array([3 << (25 if i % 2 == 0 else 24) for i in range(10)], np.int64)
        cases.append((rng.integers(-lim, lim + 1).astype(np.int32), rng.integers(-lim, lim + 1).astype(np.int32)))
    ext = np.array([3 << (25 if i % 2 == 0 else 24) for i in range(10)], np.int32)
    cases += [(ext, ext), (-ext, ext), (-ext, -ext), (ext, np.zeros(10, np.int32))]
    for f, g in cases:
        assert H.hostcheck_fe_mul_par(f.ctypes.data_as(i32), g.ctypes.data_as(i32), 40) == 1


def test_sc_reduce512(H):
    rng = np.random.default_rng(6)
    cases = [rng.bytes(64) for _ in range(1000)] + [b"\xff" * 64, bytes(64), E.L.to_bytes(64, "little"),
                                                    (E.L - 1).to_bytes(64, "little"),
                                                    (E.L * 2**259 - 1).to_bytes(64, "little")]
    for x in cases:
        out = np.zeros(32, np.uint8)
        H.hostcheck_sc_reduce512(p(_u8(x)), p(out))
        assert int.from_bytes(out.tobytes(), "little") == int.from_bytes(x, "little") % E.L


def test_sha512_pq_msg(H):
    rng = np.random.default_rng(7)
    for n in list(range(0, 64)) + [110, 111, 112, 125, 200, 239, 240, 300]:
        P_, Q, m = rng.bytes(32), rng.bytes(32), rng.bytes(n)
        out = np.zeros(64, np.uint8)
        H.hostcheck_sha512_pq_msg(p(_u8(P_)), p(_u8(Q)), p(_u8(m + b"\0")), n, p(out))
        assert out.tobytes() == hashlib.sha512(P_ + Q + m).digest()


def test_verify_core_vs_oracle(H, golden):
    vs = golden("ed25519_vectors.json")["vectors"]
    ents = [(bytes.fromhex(v["pk"]), bytes.fromhex(v["msg"]), bytes.fromhex(v["sig"])) for v in vs]
    g = golden("zip215_small_order.json")
    ents += [(bytes.fromhex(a), b"x", bytes.fromhex(r) + bytes(32)) for a, r in g["pairs_all_valid_with_S0"]]
    pk, sig, msg, off = C.pack(ents)
    _, ref = C.ed25519_verify_packed(pk, sig, msg, off)
    out = np.zeros(len(ents), np.uint8)
    H.hostcheck_ed25519_verify_batch(p(pk), p(sig), p(msg), p(off, ctypes.c_uint32), len(ents), p(out))
    assert np.array_equal(out, ref)


def _chacha20_py(key: bytes, counter: int, nonce: bytes) -> bytes:
    """RFC 8439 §2.3 block function, restated in Python (checker)."""
    M = 0xFFFFFFFF
    rotl = lambda x, n: ((x << n) | (x >> (32 - n))) & M  # noqa: E731
    st = [0x61707865, 0x3320646E, 0x79622D32, 0x6B206574] + [int(x) for x in np.frombuffer(key, "<u4")] + \
         [counter] + [int(x) for x in np.frombuffer(nonce, "<u4")]
    s = list(st)

    def qr(a, b, c, d):
        s[a] = (s[a] + s[b]) & M; s[d] = rotl(s[d] ^ s[a], 16)
        s[c] = (s[c] + s[d]) & M; s[b] = rotl(s[b] ^ s[c], 12)
        s[a] = (s[a] + s[b]) & M; s[d] = rotl(s[d] ^ s[a], 8)
        s[c] = (s[c] + s[d]) & M; s[b] = rotl(s[b] ^ s[c], 7)
    for _ in range(10):
        qr(0, 4, 8, 12); qr(1, 5, 9, 13); qr(2, 6, 10, 14); qr(3, 7, 11, 15)
        qr(0, 5, 10, 15); qr(1, 6, 11, 12); qr(2, 7, 8, 13); qr(3, 4, 9, 14)
    return b"".join(int((a + b) & M).to_bytes(4, "little") for a, b in zip(s, st))


def _chacha20_openssl(key: bytes, counter: int, nonce: bytes) -> bytes:
    """One keystream block from OpenSSL's EVP_chacha20 (IV = counter || nonce)."""
    lib = ctypes.CDLL("libcrypto.so.3")
    lib.EVP_CIPHER_CTX_new.restype = ctypes.c_void_p
    lib.EVP_chacha20.restype = ctypes.c_void_p
    lib.EVP_EncryptInit_ex.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_char_p,
                                       ctypes.c_char_p]
    lib.EVP_EncryptUpdate.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int),
                                      ctypes.c_char_p, ctypes.c_int]
    lib.EVP_CIPHER_CTX_free.argtypes = [ctypes.c_void_p]
    c = lib.EVP_CIPHER_CTX_new()
    assert lib.EVP_EncryptInit_ex(c, lib.EVP_chacha20(), None, key, counter.to_bytes(4, "little") + nonce) == 1
    out = ctypes.create_string_buffer(64)
    n = ctypes.c_int(0)
    assert lib.EVP_EncryptUpdate(c, out, ctypes.byref(n), bytes(64), 64) == 1
    lib.EVP_CIPHER_CTX_free(c)
    return out.raw


def test_chacha20_known_answer(H):
    """The device ChaCha20 (msm.h chacha20_block, the batch equation's z_i,
    SURVEY row I) against RFC 8439 §2.3.2's test vector, a Python restatement
    and OpenSSL's EVP_chacha20 on random keys / counters / nonces: a weight
    generator bug (zero or low-entropy z_i) would let a bad signature pass its
    group check."""
    H.hostcheck_chacha20_block.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_char_p]

    def dev(key, counter, nonce):
        out = ctypes.create_string_buffer(64)
        H.hostcheck_chacha20_block(key, counter, nonce, out)
        return out.raw

    key = bytes(range(32))
    nonce = bytes.fromhex("000000090000004a00000000")
    want = bytes.fromhex("10f1e7e4d13b5915500fdd1fa32071c4c7d1f4c733c068030422aa9ac3d46c4e"
                         "d2826446079faa0914c2d705d98b02a2b5129cd1de164eb9cbd083e8a2503c4e")
    assert _chacha20_py(key, 1, nonce) == want
    assert _chacha20_openssl(key, 1, nonce) == want
    assert dev(key, 1, nonce) == want
    rng = np.random.default_rng(8439)
    for _ in range(200):
        k = rng.bytes(32)
        n = rng.bytes(12)
        ctr = int(rng.integers(0, 2**32))
        assert dev(k, ctr, n) == _chacha20_openssl(k, ctr, n)
    # weights for consecutive entries (counter = entry index) are distinct and nonzero
    z = {dev(key, e, nonce)[:16] for e in range(4096)}
    assert len(z) == 4096 and bytes(16) not in z


def test_sr25519_transcript_fast_path(H):
    """The register-state transcript (merlin_dev.h sr25519_challenge_fast,
    messages of 98..127 bytes) gives the generic STROBE path's challenge for
    every eligible length; other lengths are refused (they take the generic
    path on the device)."""
    H.hostcheck_sr25519_challenge.restype = ctypes.c_int
    rng = np.random.default_rng(98127)
    eligible = 0
    for mlen in range(0, 141):
        for _ in range(3):
            pk = rng.integers(0, 256, 32, dtype=np.uint8)
            r = rng.integers(0, 256, 32, dtype=np.uint8)
            m = rng.integers(0, 256, mlen + 1, dtype=np.uint8)
            gen = np.zeros(32, np.uint8)
            fast = np.zeros(32, np.uint8)
            assert H.hostcheck_sr25519_challenge(p(pk), p(r), p(m), mlen, 0, p(gen)) == 1
            ok = H.hostcheck_sr25519_challenge(p(pk), p(r), p(m), mlen, 1, p(fast))
            assert ok == (98 <= mlen <= 127), mlen
            if ok:
                eligible += 1
                assert np.array_equal(gen, fast), mlen
    assert eligible == 30 * 3


def test_p1p1_to_cached_matches_two_step(H):
    """ge_p1p1_to_cached (k_msm_wpart's cached U, one lane per window) equals
    p1p1_to_p3 followed by p3_to_cached, coordinate by coordinate."""
    import random
    rng = random.Random(1717)
    enc = []
    while len(enc) < 400:
        y = rng.randrange(E.P) if hasattr(E, "P") else rng.randrange(2**255 - 19)
        b = bytearray(y.to_bytes(32, "little"))
        b[31] |= rng.randrange(2) << 7
        enc.append(bytes(b))
    buf = np.frombuffer(b"".join(enc), np.uint8).copy()
    H.hostcheck_p1p1_to_cached.restype = ctypes.c_int
    assert H.hostcheck_p1p1_to_cached(p(buf), len(enc)) == 0


def test_degenerate_point_fails_every_verdict(H):
    """A point never computed ((0 : 0 : 0 : 0), a zeroed slot nobody wrote)
    passes X == 0, Y == Z and both Ristretto equalities; every verdict also
    requires Z != 0, so a missing write fails a group instead of passing it
    (the quad forms in quad.h carry the same test, covered on the GPU)."""
    assert H.hostcheck_degenerate_verdicts() == 1
