"""Differential fuzzing of the device paths against the oracle: random and
mutated inputs (garbage keys and signatures, single-bit flips at every
position class, S near l, messages across the SHA-512 block boundaries of
R || A || M), through every kernel family, must give the oracle's vector
entry for entry."""
import random

import numpy as np
import pytest

import oracle_c as C
from tendermint_amd import _native as N
from tendermint_amd.testing._openssl import Ed25519Signer
from tendermint_amd.testing.factory import (SMALL_ORDER_CANONICAL, SMALL_ORDER_NEG_ZERO, SMALL_ORDER_NONCANONICAL_Y,
                                            Batch, key_seed)

pytestmark = pytest.mark.gpu

L = 2**252 + 27742317777372353535851937790883648493
# 64-byte R || A prefix: SHA-512 pads at 112 mod 128 and blocks are 128 bytes,
# so these message lengths put the padding on either side of a block edge
EDGE_LENS = [0, 1, 47, 48, 49, 63, 64, 111, 112, 113, 175, 176, 177, 239, 240, 241, 1000]
ED, SR = N.TMV_KIND_ED25519, N.TMV_KIND_SR25519
FLAGS = [N.TMV_FLAG_PER_ENTRY, N.TMV_FLAG_BATCH_EQUATION, N.TMV_FLAG_KEY_CACHE,
         N.TMV_FLAG_KEY_CACHE | N.TMV_FLAG_BATCH_EQUATION]


def _rb(rng, n):
    return bytes(rng.randrange(256) for _ in range(n))


def _ed_corpus(n, seed):
    rng = random.Random(seed)
    signers = [Ed25519Signer(key_seed(k, "fuzz")) for k in range(64)]
    small = SMALL_ORDER_CANONICAL + SMALL_ORDER_NEG_ZERO + SMALL_ORDER_NONCANONICAL_Y
    ents = []
    for i in range(n):
        s = signers[rng.randrange(len(signers))]
        mlen = rng.choice(EDGE_LENS) if rng.randrange(3) == 0 else rng.randrange(300)
        msg = _rb(rng, mlen)
        pk, sig = s.public_key, s.sign(msg)
        kind = rng.randrange(12)
        if kind == 0:          # garbage key
            pk = _rb(rng, 32)
        elif kind == 1:        # garbage signature
            sig = _rb(rng, 64)
        elif kind == 2:        # one bit anywhere in R, S, A or the message
            where = rng.randrange(4)
            if where == 0 or where == 1:
                b = bytearray(sig)
                b[(0 if where == 0 else 32) + rng.randrange(32)] ^= 1 << rng.randrange(8)
                sig = bytes(b)
            elif where == 2:
                b = bytearray(pk)
                b[rng.randrange(32)] ^= 1 << rng.randrange(8)
                pk = bytes(b)
            elif msg:
                b = bytearray(msg)
                b[rng.randrange(len(msg))] ^= 1 << rng.randrange(8)
                msg = bytes(b)
        elif kind == 3:        # S + l, S + 2^253, S = l - 1, S = 0
            sv = int.from_bytes(sig[32:], "little")
            sv = rng.choice([sv + L, sv + (1 << 253), L - 1, 0, L, (1 << 256) - 1])
            sig = sig[:32] + (sv % (1 << 256)).to_bytes(32, "little")
        elif kind == 4:        # small-order / non-canonical R and A
            sig = rng.choice(small) + sig[32:]
            if rng.randrange(2):
                pk = rng.choice(small)
        ents.append((pk, msg, sig))
    return Batch.from_entries(ents)


@pytest.mark.parametrize("flags", FLAGS)
def test_ed25519_fuzz(ctx, flags):
    b = _ed_corpus(6000, 91 + flags)
    _, ref = C.ed25519_verify_packed(b.pk, b.sig, b.msg, b.off, threads=8)
    assert 0 < int(ref.sum()) < b.n
    ok, st = ctx.verify_batch_ex(ED, flags, b.pk, b.sig, b.msg, b.off)
    assert np.array_equal(st.astype(np.uint8), ref)


def test_ed25519_fuzz_large_default(ctx):
    """Above the batch-equation threshold without flags; tiled so groups mix
    many corrupted entries with valid ones."""
    b = _ed_corpus(5000, 97).tile(40000)
    _, ref = C.ed25519_verify_packed(b.pk, b.sig, b.msg, b.off, threads=8)
    ok, st = ctx.ed25519_verify_batch(b.pk, b.sig, b.msg, b.off)
    assert np.array_equal(st.astype(np.uint8), ref)


@pytest.mark.parametrize("flags", [N.TMV_FLAG_PER_ENTRY, N.TMV_FLAG_BATCH_EQUATION, N.TMV_FLAG_KEY_CACHE])
def test_sr25519_fuzz(ctx, flags):
    from tendermint_amd.testing.sr25519_factory import Sr25519Signer, mini_from_secret
    rng = random.Random(98 + flags)
    signers = [Sr25519Signer(mini_from_secret(b"fuzz: %x" % k)) for k in range(32)]
    ents = []
    for i in range(3000):
        s = signers[rng.randrange(len(signers))]
        msg = _rb(rng, rng.choice(EDGE_LENS) if rng.randrange(3) == 0 else rng.randrange(300))
        pk, sig = s.public_key, s.sign(msg, b"%d" % i)
        kind = rng.randrange(10)
        if kind == 0:
            pk = _rb(rng, 32)
        elif kind == 1:
            sig = _rb(rng, 64)
        elif kind == 2:
            b = bytearray(sig)
            b[rng.randrange(64)] ^= 1 << rng.randrange(8)
            sig = bytes(b)
        elif kind == 3 and msg:
            b = bytearray(msg)
            b[rng.randrange(len(msg))] ^= 1 << rng.randrange(8)
            msg = bytes(b)
        ents.append((pk, msg, sig))
    b = Batch.from_entries(ents)
    ref = C.sr25519_status_packed(b.pk, b.sig, b.msg, b.off, threads=8)
    assert set(np.unique(ref)) >= {-2, -1, 0, 1}
    ok, st = ctx.verify_batch_ex(SR, flags, b.pk, b.sig, b.msg, b.off)
    assert np.array_equal(st, ref)
