"""Half-size verification scalars (tendermint_amd/csrc/halfscalar.h) on the
host: the lattice reduction against Python's extended Euclid, and the short
verification equation [8]([b]B + [u](-R) + [v](-A)) == O (sr25519: the
Ristretto identity) against the oracle's [8]([s]B - R - [k]A) == O on the
reference-shaped edge vectors.  No GPU."""
import ctypes
import os
import random
import subprocess

import numpy as np
import pytest

import oracle_c as C

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(REPO, "oracle", "_build", "libhostcheck.so")
L = 2**252 + 27742317777372353535851937790883648493


@pytest.fixture(scope="module")
def H():
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "tests", "native")], check=True)
    return ctypes.CDLL(SO)


def euclid_half(k, with_qmax=False):
    """Extended Euclid on (l, k): the first remainder r_i < 2^126 and its
    cofactor t_i (r_i == t_i k mod l); with_qmax: also the largest quotient."""
    r0, r1, t0, t1, qmax = L, k, 0, 1, 0
    while r1 >= 1 << 126:
        q = r0 // r1
        qmax = max(qmax, q)
        r0, r1, t0, t1 = r1, r0 - q * r1, t1, t0 - q * t1
    return (t1, r1, qmax) if with_qmax else (t1, r1)


def reduce(H, k):
    u = ctypes.create_string_buffer(16)
    v = ctypes.create_string_buffer(16)
    neg = ctypes.c_int(0)
    ok = H.hostcheck_half_reduce(k.to_bytes(32, "little"), u, v, ctypes.byref(neg))
    um = int.from_bytes(u.raw, "little")
    return ok, (-um if neg.value else um), int.from_bytes(v.raw, "little")


EDGE_K = [0, 1, 2, 3, L - 1, L - 2, L - 3, (L - 1) // 2, (L + 1) // 2, L // 3, 2 * L // 3, (1 << 126) - 1, 1 << 126,
          (1 << 126) + 1, 1 << 127, (1 << 127) + 12345, 1 << 200, (1 << 252) - 1, 1 << 252, L - (1 << 126),
          L - (1 << 127), 3 * (1 << 126) + 5, L // 5, L // 7 + 1, L // (1 << 20), L // (1 << 40) + 3]


def test_reduce_matches_euclid(H):
    """Every fast-path result is exactly Euclid's first remainder below 2^126
    and its cofactor (so |u| < 2^126.6 and v < 2^126 by Euclid's bound);
    random k never takes the slow path."""
    rng = random.Random(7)
    ks = [rng.randrange(L) for _ in range(20000)]
    for k in ks:
        ok, u, v = reduce(H, k)
        assert ok, hex(k)
        assert (u, v) == euclid_half(k), hex(k)
        assert abs(u) < 1 << 127 and v < 1 << 126
        assert (u * k - v) % L == 0


def test_reduce_edge_values(H):
    """Quotients of 1 and 2 in the first steps (k near l, l / 2, l / 3), k
    already short, quotients of 2^20 .. 2^40: the fast path gives Euclid's
    pair whenever every quotient before the crossing is below 2^31; only a
    larger quotient (k = 2^200, 2^127, l / 2^40 ...) takes the slow path,
    which verifies with the full k."""
    for k in EDGE_K:
        ok, u, v = reduce(H, k)
        eu, ev, qmax = euclid_half(k, True)
        if qmax < 1 << 31:
            assert ok and (u, v) == (eu, ev), hex(k)
        elif ok:
            assert (u, v) == (eu, ev), hex(k)


def _verify_half(H, pk, sig, msg, off, sr):
    n = len(off) - 1
    out = np.zeros(n, np.int8)
    slow = ctypes.c_int(0)
    pp = lambda a, t=ctypes.c_uint8: a.ctypes.data_as(ctypes.POINTER(t))  # noqa: E731
    H.hostcheck_verify_half(pp(pk), pp(sig), pp(msg), pp(off, ctypes.c_uint32), n, sr, pp(out, ctypes.c_int8),
                            ctypes.byref(slow))
    return out, slow.value


def test_short_equation_ed25519_vs_oracle(H, golden):
    """ZIP-215 edge vectors (S + l, undecodable, small order, non-canonical y,
    -0), the 196-pair small-order matrix and a C2-shaped batch: the short
    equation gives the oracle's vector bit for bit."""
    from tendermint_amd.testing.factory import make_c2_batch
    vs = golden("ed25519_vectors.json")["vectors"]
    ents = [(bytes.fromhex(v["pk"]), bytes.fromhex(v["msg"]), bytes.fromhex(v["sig"])) for v in vs]
    g = golden("zip215_small_order.json")
    ents += [(bytes.fromhex(a), b"x", bytes.fromhex(r) + bytes(32)) for a, r in g["pairs_all_valid_with_S0"]]
    pk, sig, msg, off = C.pack(ents)
    _, ref = C.ed25519_verify_packed(pk, sig, msg, off)
    out, _ = _verify_half(H, pk, sig, msg, off, 0)
    assert np.array_equal(out.astype(np.uint8), ref)
    b = make_c2_batch(600, seed=99)
    _, ref = C.ed25519_verify_packed(b.pk, b.sig, b.msg, b.off)
    out, slow = _verify_half(H, b.pk, b.sig, b.msg, b.off, 0)
    assert np.array_equal(out.astype(np.uint8), ref) and slow == 0
    assert 0 < int(ref.sum()) < b.n


def test_short_equation_sr25519_vs_oracle(H, golden):
    """sr25519 statuses (1 / 0 / -1 / -2) through the Ristretto-identity form
    of the short equation, against the C oracle (the published-vector-pinned
    verifier)."""
    from tendermint_amd.testing.factory import make_mixed_batch
    kind, mb = make_mixed_batch(1200, seed=0x5E)
    sr = mb.take(np.flatnonzero(kind == 1))
    ref = C.sr25519_status_packed(sr.pk, sr.sig, sr.msg, sr.off, threads=4)
    out, slow = _verify_half(H, sr.pk, sr.sig, sr.msg, sr.off, 1)
    assert np.array_equal(out, np.asarray(ref, np.int8)) and slow == 0
    assert (np.asarray(ref) == 1).any() and (np.asarray(ref) == 0).any()
