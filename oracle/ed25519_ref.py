"""TEST INFRASTRUCTURE ONLY — CPU oracle, never on the product path.

Pure-Python (big-integer) restatement of the ed25519 verification semantics
Tendermint uses on its commit/vote path:

  * ``crypto/ed25519/ed25519.go:27-29``  — verify options = ZIP-215
  * ``crypto/ed25519/ed25519.go:173-180`` — PubKey.VerifySignature (len(sig)!=64 -> false)
  * ``crypto/ed25519/ed25519.go:209-233`` — BatchVerifier.Add / Verify
  * ZIP-215 as adopted in ``spec/core/encoding.md:52`` and
    ``docs/architecture/adr-079-ed25519-verification.md:14-24``.

The arithmetic itself lives in the third-party module
``github.com/oasisprotocol/curve25519-voi v0.0.0-20210609091139-0a56a4bca00b``
(``go.mod:22``; absent from this container).  This file restates its
published algorithm (RFC 8032 + ZIP-215 decoding/cofactored equation):

  accept(A, M, R||S) iff
     S < l                                  (strictly canonical S)
     A, R decode under *lax* rules           (y taken mod p, x=0 with sign=1 ok)
     k = SHA-512(R_bytes || A_bytes || M) mod l   (original encodings)
     [8]([S]B - R - [k]A) == O               (cofactored)

Batch semantics (voi ``BatchVerifier.Verify``): empty batch -> (False, []);
otherwise the vector equals per-entry single verification (ZIP-215 makes the
random-linear-combination check agree with single verification), and
``ok == all(vector)``.

Pinning: SHA-512 from hashlib; honest signatures cross-checked against
OpenSSL 3 (RFC 8032 deterministic signing, byte-identical to voi
``ed25519.Sign``), see tests/test_oracle.py.
"""
from __future__ import annotations

import hashlib

P = 2**255 - 19
L = 2**252 + 27742317777372353535851937790883648493
D = (-121665 * pow(121666, P - 2, P)) % P
SQRT_M1 = pow(2, (P - 1) // 4, P)


def _inv(x: int) -> int:
    return pow(x, P - 2, P)


# --- points in extended twisted Edwards coordinates (X, Y, Z, T), x*y = T/Z ---

IDENT = (0, 1, 1, 0)


def pt_add(p1, p2):
    X1, Y1, Z1, T1 = p1
    X2, Y2, Z2, T2 = p2
    A = (Y1 - X1) * (Y2 - X2) % P
    B = (Y1 + X1) * (Y2 + X2) % P
    C = 2 * D * T1 * T2 % P
    Dd = 2 * Z1 * Z2 % P
    E, F, G, H = B - A, Dd - C, Dd + C, B + A
    return (E * F % P, G * H % P, F * G % P, E * H % P)


def pt_neg(p):
    X, Y, Z, T = p
    return ((-X) % P, Y, Z, (-T) % P)


def pt_mul(k: int, p):
    q = IDENT
    while k > 0:
        if k & 1:
            q = pt_add(q, p)
        p = pt_add(p, p)
        k >>= 1
    return q


def pt_is_identity(p) -> bool:
    X, Y, Z, _ = p
    return X % P == 0 and (Y - Z) % P == 0


def pt_equal(p1, p2) -> bool:
    X1, Y1, Z1, _ = p1
    X2, Y2, Z2, _ = p2
    return (X1 * Z2 - X2 * Z1) % P == 0 and (Y1 * Z2 - Y2 * Z1) % P == 0


def pt_encode(p) -> bytes:
    X, Y, Z, _ = p
    zi = _inv(Z)
    x, y = X * zi % P, Y * zi % P
    return int.to_bytes(y | ((x & 1) << 255), 32, "little")


def recover_x(y: int, sign: int):
    """x from y on -x^2 + y^2 = 1 + d x^2 y^2; None if (y^2-1)/(d y^2+1) is not square."""
    u = (y * y - 1) % P
    v = (D * y * y + 1) % P
    x = u * pow(v, 3, P) * pow(u * pow(v, 7, P), (P - 5) // 8, P) % P
    vx2 = v * x * x % P
    if vx2 == u % P:
        pass
    elif vx2 == (-u) % P:
        x = x * SQRT_M1 % P
    else:
        return None
    if (x & 1) != sign:
        x = (-x) % P  # x == 0 stays 0: ZIP-215 accepts the "-0" encoding
    return x


def decode_point_zip215(b: bytes):
    """Lax decoding (ZIP-215): y >= p accepted (reduced), '-0' accepted."""
    if len(b) != 32:
        return None
    v = int.from_bytes(b, "little")
    sign = v >> 255
    y = (v & ((1 << 255) - 1)) % P
    x = recover_x(y, sign)
    if x is None:
        return None
    return (x, y, 1, x * y % P)


def decode_point_strict(b: bytes):
    """RFC 8032 strict decoding (used only for fixture generation)."""
    v = int.from_bytes(b, "little")
    y = v & ((1 << 255) - 1)
    if y >= P:
        return None
    x = recover_x(y, v >> 255)
    if x is None or (x == 0 and (v >> 255) == 1):
        return None
    return (x, y, 1, x * y % P)


BY = 4 * _inv(5) % P
BX = recover_x(BY, 0)
BASE = (BX, BY, 1, BX * BY % P)


def sha512_modl(*parts: bytes) -> int:
    h = hashlib.sha512()
    for x in parts:
        h.update(x)
    return int.from_bytes(h.digest(), "little") % L


# --- signing (RFC 8032, deterministic); voi ed25519.Sign is byte-identical ---

def expand_seed(seed: bytes):
    h = hashlib.sha512(seed).digest()
    a = int.from_bytes(h[:32], "little")
    a &= (1 << 254) - 8
    a |= 1 << 254
    return a, h[32:]


def public_key(seed: bytes) -> bytes:
    a, _ = expand_seed(seed)
    return pt_encode(pt_mul(a, BASE))


def sign(seed: bytes, msg: bytes) -> bytes:
    a, prefix = expand_seed(seed)
    A = pt_encode(pt_mul(a, BASE))
    r = sha512_modl(prefix, msg)
    R = pt_encode(pt_mul(r, BASE))
    k = sha512_modl(R, A, msg)
    S = (r + k * a) % L
    return R + int.to_bytes(S, 32, "little")


# --- verification (ZIP-215, cofactored) ---

def verify_zip215(pk: bytes, msg: bytes, sig: bytes) -> bool:
    """crypto/ed25519/ed25519.go:173-180 -> voi VerifyWithOptions(ZIP_215)."""
    if len(sig) != 64 or len(pk) != 32:
        return False
    S = int.from_bytes(sig[32:], "little")
    if S >= L:
        return False
    A = decode_point_zip215(pk)
    if A is None:
        return False
    R = decode_point_zip215(sig[:32])
    if R is None:
        return False
    k = sha512_modl(sig[:32], pk, msg)
    # [S]B - R - [k]A
    Q = pt_add(pt_mul(S, BASE), pt_neg(pt_add(R, pt_mul(k, A))))
    Q = pt_add(Q, Q)
    Q = pt_add(Q, Q)
    Q = pt_add(Q, Q)
    return pt_is_identity(Q)


def batch_verify(entries):
    """voi BatchVerifier.Verify semantics: (all_ok, per-entry vector).

    Empty batch -> (False, []).  ``entries`` = iterable of (pk, msg, sig).
    """
    vec = [verify_zip215(pk, m, s) for (pk, m, s) in entries]
    if not vec:
        return False, []
    return all(vec), vec


# --- small-order / torsion helpers for ZIP-215 fixture generation ---

def torsion_points():
    """The 8 points of order dividing 8, in affine (x, y)."""
    # order-2: (0,-1); order-4: (+-sqrt(-1)... ) found by solving; simplest: scan
    pts = []
    # y candidates: 1, -1, 0, and the two order-8 y values (roots of d y^4 ... )
    # Derive generically: T8 = [l]Q for Q of full order; use hash-to-point scan.
    y = 2
    while True:
        x = recover_x(y, 0)
        if x is not None:
            Qp = (x, y, 1, x * y % P)
            T = pt_mul(L, Qp)
            # need a generator of the 8-torsion
            T2 = pt_add(T, T)
            T4 = pt_add(T2, T2)
            if not pt_is_identity(T4):
                break
        y += 1
    acc = IDENT
    for _ in range(8):
        pts.append(acc)
        acc = pt_add(acc, T)
    out = []
    for p in pts:
        X, Y, Z, _ = p
        zi = _inv(Z)
        out.append((X * zi % P, Y * zi % P))
    return out


def small_order_encodings():
    """All 32-byte encodings that decode (ZIP-215 lax) to a small-order point.

    Canonical encodings of the 8 torsion points plus the non-canonical ones
    (y+p < 2^255, and sign-bit variants of x = 0).  SURVEY Appendix D.
    """
    encs = set()
    for (x, y) in torsion_points():
        for yy in (y, y + P):
            if yy >= 2**255:
                continue
            for s in (0, 1):
                e = int.to_bytes(yy | (s << 255), 32, "little")
                pt = decode_point_zip215(e)
                if pt is None:
                    continue
                if pt_is_identity(pt_mul(8, pt)):
                    encs.add(e)
    return sorted(encs)
