"""TEST INFRASTRUCTURE ONLY — CPU oracle, never on the product path.

Pure-Python restatement of the sr25519 (Schnorrkel over Ristretto255, merlin
transcripts) verification Tendermint runs behind crypto.BatchVerifier:

  * ``crypto/sr25519/privkey.go:18``     signing context = NewSigningContext([]byte{})
  * ``crypto/sr25519/privkey.go:157-170`` GenPrivKeyFromSecret (sha256 seed -> mini secret)
  * ``crypto/sr25519/pubkey.go:49-62``   PubKey.VerifySignature
  * ``crypto/sr25519/batch.go:23-47``    BatchVerifier.Add / Verify

The algorithms live in the absent third-party module
``github.com/oasisprotocol/curve25519-voi v0.0.0-20210609091139-0a56a4bca00b``
(``primitives/sr25519``, ``primitives/merlin``; ``go.mod:22``), which follows
schnorrkel / merlin / STROBE-128 / Ristretto255 as published:

  transcript  = merlin("SigningContext"); append("", ctx=""); append("sign-bytes", M)
  verify      : append("proto-name", "Schnorr-sig"); append("sign:pk", A_bytes);
                append("sign:R", R_bytes); k = challenge("sign:c", 64 B) mod l
                accept iff R == [s]B - [k]A   (Ristretto equality)
  signature   = R(32) || s(32) with bit 7 of byte 63 set (schnorrkel marker);
                s must be canonical (< l) after clearing the marker.

Pinning: Keccak-f[1600] against hashlib.sha3_256; merlin against its published
"test protocol" vector; Ristretto255 against the published multiples of the
generator (RFC 9496 App. A.1).  sr25519 signature validity itself is pinned
only by this restatement (voi/schnorrkel are absent): "parity unpinned" for
sr25519 signature fixtures.

Add-time behaviour (crypto/sr25519/batch.go:30-37): an undecodable public key
or a signature failing the marker / canonical-s check makes ``Add`` return an
error.  An R that is not a valid Ristretto encoding is *not* an Add error
(schnorrkel keeps R compressed); the entry simply fails verification.
"""
from __future__ import annotations

import hashlib

from ed25519_ref import (P, L, D, SQRT_M1, BASE, IDENT, pt_add, pt_neg, pt_mul)

# ---------------------------------------------------------------- Keccak-f[1600]

_RC = [
    0x0000000000000001, 0x0000000000008082, 0x800000000000808A, 0x8000000080008000,
    0x000000000000808B, 0x0000000080000001, 0x8000000080008081, 0x8000000000008009,
    0x000000000000008A, 0x0000000000000088, 0x0000000080008009, 0x000000008000000A,
    0x000000008000808B, 0x800000000000008B, 0x8000000000008089, 0x8000000000008003,
    0x8000000000008002, 0x8000000000000080, 0x000000000000800A, 0x800000008000000A,
    0x8000000080008081, 0x8000000000008080, 0x0000000080000001, 0x8000000080008008]
_ROT = [[0, 36, 3, 41, 18], [1, 44, 10, 45, 2], [62, 6, 43, 15, 61],
        [28, 55, 25, 21, 56], [27, 20, 39, 8, 14]]
_M64 = (1 << 64) - 1


def _rol(x, n):
    return ((x << n) | (x >> (64 - n))) & _M64 if n else x


def keccak_f1600(state: bytearray) -> None:
    """In-place Keccak-f[1600] on a 200-byte state (lanes little-endian, A[x][y] = lane x+5y)."""
    A = [[int.from_bytes(state[8 * (x + 5 * y):8 * (x + 5 * y) + 8], "little") for y in range(5)]
         for x in range(5)]
    for rnd in range(24):
        C = [A[x][0] ^ A[x][1] ^ A[x][2] ^ A[x][3] ^ A[x][4] for x in range(5)]
        Dd = [C[(x - 1) % 5] ^ _rol(C[(x + 1) % 5], 1) for x in range(5)]
        A = [[A[x][y] ^ Dd[x] for y in range(5)] for x in range(5)]
        Bm = [[0] * 5 for _ in range(5)]
        for x in range(5):
            for y in range(5):
                Bm[y][(2 * x + 3 * y) % 5] = _rol(A[x][y], _ROT[x][y])
        A = [[Bm[x][y] ^ ((~Bm[(x + 1) % 5][y]) & Bm[(x + 2) % 5][y]) for y in range(5)]
             for x in range(5)]
        A[0][0] ^= _RC[rnd]
    for x in range(5):
        for y in range(5):
            state[8 * (x + 5 * y):8 * (x + 5 * y) + 8] = A[x][y].to_bytes(8, "little")


def sha3_256_via_keccak(msg: bytes) -> bytes:
    """SHA3-256 built on keccak_f1600 — used only to pin the permutation."""
    rate = 136
    st = bytearray(200)
    m = bytearray(msg) + b"\x06"
    while len(m) % rate:
        m += b"\x00"
    m[-1] |= 0x80
    for off in range(0, len(m), rate):
        for i in range(rate):
            st[i] ^= m[off + i]
        keccak_f1600(st)
    return bytes(st[:32])


# ---------------------------------------------------------------- STROBE-128 / merlin

STROBE_R = 166
FLAG_I, FLAG_A, FLAG_C, FLAG_T, FLAG_M, FLAG_K = 1, 2, 4, 8, 16, 32


class Strobe128:
    def __init__(self, protocol_label: bytes):
        st = bytearray(200)
        st[0:6] = bytes([1, STROBE_R + 2, 1, 0, 1, 96])
        st[6:18] = b"STROBEv1.0.2"
        keccak_f1600(st)
        self.st, self.pos, self.pos_begin, self.cur_flags = st, 0, 0, 0
        self.meta_ad(protocol_label, False)

    def clone(self):
        c = Strobe128.__new__(Strobe128)
        c.st, c.pos, c.pos_begin, c.cur_flags = bytearray(self.st), self.pos, self.pos_begin, self.cur_flags
        return c

    def _run_f(self):
        self.st[self.pos] ^= self.pos_begin
        self.st[self.pos + 1] ^= 0x04
        self.st[STROBE_R + 1] ^= 0x80
        keccak_f1600(self.st)
        self.pos = 0
        self.pos_begin = 0

    def _absorb(self, data: bytes):
        for b in data:
            self.st[self.pos] ^= b
            self.pos += 1
            if self.pos == STROBE_R:
                self._run_f()

    def _squeeze(self, n: int) -> bytes:
        out = bytearray()
        for _ in range(n):
            out.append(self.st[self.pos])
            self.st[self.pos] = 0
            self.pos += 1
            if self.pos == STROBE_R:
                self._run_f()
        return bytes(out)

    def _begin_op(self, flags: int, more: bool):
        if more:
            assert self.cur_flags == flags
            return
        assert flags & FLAG_T == 0
        old_begin = self.pos_begin
        self.pos_begin = self.pos + 1
        self.cur_flags = flags
        self._absorb(bytes([old_begin, flags]))
        if flags & (FLAG_C | FLAG_K) and self.pos != 0:
            self._run_f()

    def meta_ad(self, data: bytes, more: bool):
        self._begin_op(FLAG_M | FLAG_A, more)
        self._absorb(data)

    def ad(self, data: bytes, more: bool):
        self._begin_op(FLAG_A, more)
        self._absorb(data)

    def prf(self, n: int, more: bool = False) -> bytes:
        self._begin_op(FLAG_I | FLAG_A | FLAG_C, more)
        return self._squeeze(n)


class Transcript:
    def __init__(self, label: bytes, _strobe=None):
        if _strobe is not None:
            self.strobe = _strobe
            return
        self.strobe = Strobe128(b"Merlin v1.0")
        self.append_message(b"dom-sep", label)

    def clone(self):
        return Transcript(b"", _strobe=self.strobe.clone())

    def append_message(self, label: bytes, message: bytes):
        self.strobe.meta_ad(label, False)
        self.strobe.meta_ad(len(message).to_bytes(4, "little"), True)
        self.strobe.ad(message, False)

    def challenge_bytes(self, label: bytes, n: int) -> bytes:
        self.strobe.meta_ad(label, False)
        self.strobe.meta_ad(n.to_bytes(4, "little"), True)
        return self.strobe.prf(n)


def signing_transcript(msg: bytes, context: bytes = b"") -> Transcript:
    """NewSigningContext(context).NewTranscriptBytes(msg) (crypto/sr25519/batch.go:39)."""
    t = Transcript(b"SigningContext")
    t.append_message(b"", context)
    t.append_message(b"sign-bytes", msg)
    return t


# ---------------------------------------------------------------- Ristretto255

def _is_neg(x: int) -> bool:
    return (x % P) & 1 == 1


def _abs(x: int) -> int:
    x %= P
    return (P - x) % P if x & 1 else x


INVSQRT_A_MINUS_D = None  # set below


def sqrt_ratio_i(u: int, v: int):
    """(was_square, r) with r = sqrt(u/v) or sqrt(i*u/v), r non-negative."""
    u %= P
    v %= P
    v3 = v * v % P * v % P
    v7 = v3 * v3 % P * v % P
    r = u * v3 % P * pow(u * v7 % P, (P - 5) // 8, P) % P
    check = v * r % P * r % P
    correct = check == u
    flipped = check == (-u) % P
    flipped_i = check == (-u * SQRT_M1) % P
    r_prime = r * SQRT_M1 % P
    if flipped or flipped_i:
        r = r_prime
    r = _abs(r)
    return (correct or flipped), r


INVSQRT_A_MINUS_D = sqrt_ratio_i(1, (-1 - D) % P)[1]


def ristretto_decode(b: bytes):
    """Canonical Ristretto255 decoding; None on failure."""
    if len(b) != 32:
        return None
    s = int.from_bytes(b, "little")
    if s >= P or s.to_bytes(32, "little") != b or _is_neg(s):
        return None
    ss = s * s % P
    u1 = (1 - ss) % P
    u2 = (1 + ss) % P
    u2_sqr = u2 * u2 % P
    v = (-(D * u1 % P * u1) - u2_sqr) % P
    ok, I = sqrt_ratio_i(1, v * u2_sqr % P)
    Dx = I * u2 % P
    Dy = I * Dx % P * v % P
    x = _abs(2 * s * Dx)
    y = u1 * Dy % P
    t = x * y % P
    if not ok or _is_neg(t) or y == 0:
        return None
    return (x, y, 1, t)


def ristretto_encode(pt) -> bytes:
    X, Y, Z, T = (c % P for c in pt)
    u1 = (Z + Y) * (Z - Y) % P
    u2 = X * Y % P
    _, invsqrt = sqrt_ratio_i(1, u1 * u2 % P * u2 % P)
    den1 = invsqrt * u1 % P
    den2 = invsqrt * u2 % P
    z_inv = den1 * den2 % P * T % P
    ix = X * SQRT_M1 % P
    iy = Y * SQRT_M1 % P
    enchanted = den1 * INVSQRT_A_MINUS_D % P
    if _is_neg(T * z_inv):
        X, Y = iy, ix
        den_inv = enchanted
    else:
        den_inv = den2
    if _is_neg(X * z_inv):
        Y = (-Y) % P
    s = _abs(den_inv * (Z - Y))
    return s.to_bytes(32, "little")


def ristretto_equal(p1, p2) -> bool:
    X1, Y1, _, _ = p1
    X2, Y2, _, _ = p2
    return (X1 * Y2 - Y1 * X2) % P == 0 or (Y1 * Y2 - X1 * X2) % P == 0


# ---------------------------------------------------------------- schnorrkel

def expand_mini_secret(mini: bytes):
    """MiniSecretKey.ExpandEd25519: (key scalar, nonce)."""
    h = hashlib.sha512(mini).digest()
    key = bytearray(h[:32])
    key[0] &= 248
    key[31] &= 63
    key[31] |= 64
    k = int.from_bytes(key, "little") >> 3  # divide_scalar_bytes_by_cofactor
    return k, h[32:]


def public_key(mini: bytes) -> bytes:
    k, _ = expand_mini_secret(mini)
    return ristretto_encode(pt_mul(k, BASE))


def key_from_secret(secret: bytes) -> bytes:
    """GenPrivKeyFromSecret (crypto/sr25519/privkey.go): mini secret = sha256(secret)."""
    return hashlib.sha256(secret).digest()


def sign(mini: bytes, msg: bytes, nonce_seed: bytes = b"") -> bytes:
    """Schnorrkel sign.  The reference signs with fresh randomness
    (crypto/sr25519/privkey.go:53); here the witness r is derived
    deterministically so fixtures are reproducible (verification is
    independent of how r was chosen)."""
    key, nonce = expand_mini_secret(mini)
    A = ristretto_encode(pt_mul(key, BASE))
    t = signing_transcript(msg)
    t.append_message(b"proto-name", b"Schnorr-sig")
    t.append_message(b"sign:pk", A)
    r = int.from_bytes(hashlib.sha512(b"witness" + nonce + nonce_seed + msg).digest(), "little") % L
    R = ristretto_encode(pt_mul(r, BASE))
    t.append_message(b"sign:R", R)
    k = int.from_bytes(t.challenge_bytes(b"sign:c", 64), "little") % L
    s = (k * key + r) % L
    sb = bytearray(s.to_bytes(32, "little"))
    sb[31] |= 128
    return R + bytes(sb)


class AddError(Exception):
    pass


def decode_signature(sig: bytes):
    """Signature.UnmarshalBinary: marker bit + canonical s.  Returns (R_bytes, s) or raises."""
    if len(sig) != 64:
        raise AddError("sr25519: bad signature size")
    if sig[63] & 128 == 0:
        raise AddError("sr25519: signature is not marked as a schnorrkel signature")
    sb = bytearray(sig[32:])
    sb[31] &= 127
    s = int.from_bytes(sb, "little")
    if s >= L:
        raise AddError("sr25519: signature scalar is not canonical")
    return sig[:32], s


def challenge(pk: bytes, R_bytes: bytes, msg: bytes) -> int:
    t = signing_transcript(msg)
    t.append_message(b"proto-name", b"Schnorr-sig")
    t.append_message(b"sign:pk", pk)
    t.append_message(b"sign:R", R_bytes)
    return int.from_bytes(t.challenge_bytes(b"sign:c", 64), "little") % L


def verify(pk: bytes, msg: bytes, sig: bytes) -> bool:
    """PubKey.VerifySignature (crypto/sr25519/pubkey.go:49-62)."""
    A = ristretto_decode(pk)
    if A is None:
        return False
    try:
        R_bytes, s = decode_signature(sig)
    except AddError:
        return False
    R = ristretto_decode(R_bytes)
    if R is None:
        return False
    k = challenge(pk, R_bytes, msg)
    Rp = pt_add(pt_mul(s, BASE), pt_neg(pt_mul(k, A)))
    return ristretto_equal(Rp, R)


def batch_add_check(pk: bytes, sig: bytes):
    """Raises AddError exactly where BatchVerifier.Add returns an error."""
    if ristretto_decode(pk) is None:
        raise AddError("sr25519: invalid public key")
    decode_signature(sig)


def batch_verify(entries):
    vec = [verify(pk, m, s) for (pk, m, s) in entries]
    if not vec:
        return False, []
    return all(vec), vec
