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
