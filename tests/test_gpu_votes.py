"""Device-side vote sign-bytes (k_vote_signbytes, tmv_verify_votes): the
messages the device writes are byte-identical to the reference's
sign-bytes, and verification over them gives the oracle's vector."""
import random

import numpy as np
import pytest

import oracle_c as C
import vote_cases as V
from tendermint_amd import _native as N
from tendermint_amd.testing._openssl import Ed25519Signer
from tendermint_amd.testing.factory import Batch, key_seed

pytestmark = pytest.mark.gpu


def test_device_messages_match_reference(ctx):
    rng = random.Random(51)
    tmpls, votes, msgs = V.random_votes(rng, 40, 3000)
    segs = [V.segments(t) for t in tmpls]
    got, off = ctx.vote_sign_bytes_device(segs, votes)
    want_off = np.zeros(len(msgs) + 1, np.uint32)
    want_off[1:] = np.cumsum([len(m) for m in msgs])
    assert np.array_equal(off, want_off)
    assert got == b"".join(msgs)


def test_device_messages_edge_timestamps(ctx):
    rng = random.Random(52)
    tmpls = [V.random_template(rng) for _ in range(12)]
    segs = [V.segments(t) for t in tmpls]
    rows, msgs = [], []
    for t in range(len(tmpls)):
        for ts in V.EDGE_TS:
            for wb in (True, False):
                rows.append((ts[0], ts[1], t | (N.TMV_VOTE_WITH_BLOCK if wb else 0)))
                msgs.append(V.expected(tmpls[t], wb, ts))
    votes = np.array(rows, N.VOTE_DTYPE)
    got, _ = ctx.vote_sign_bytes_device(segs, votes)
    assert got == b"".join(msgs)


def test_bad_template_index_rejected(ctx):
    votes = np.array([(1, 2, 3)], N.VOTE_DTYPE)
    with pytest.raises(N.NativeError):
        ctx.vote_sign_bytes_device([(b"", b"", b"")], votes)


def _signed_votes(rng, n_tmpl, n, bad_frac=0.05):
    tmpls, votes, msgs = V.random_votes(rng, n_tmpl, n)
    ents = []
    for i, m in enumerate(msgs):
        s = Ed25519Signer(key_seed(i % 97))  # validator keys repeat across commits
        sig = s.sign(m)
        if rng.random() < bad_frac:
            b = bytearray(sig)
            b[rng.randrange(64)] ^= 1 << rng.randrange(8)
            sig = bytes(b)
        ents.append((s.public_key, m, sig))
    return tmpls, votes, Batch.from_entries(ents)


@pytest.mark.parametrize("flags", [N.TMV_FLAG_KEY_CACHE, 0, N.TMV_FLAG_BATCH_EQUATION, N.TMV_FLAG_PER_ENTRY])
def test_verify_votes_matches_oracle(ctx, flags):
    rng = random.Random(53 + flags)
    tmpls, votes, b = _signed_votes(rng, 25, 1500)
    _, ref = C.ed25519_verify_packed(b.pk, b.sig, b.msg, b.off, threads=8)
    segs = [V.segments(t) for t in tmpls]
    ok, st = ctx.verify_votes(N.TMV_KIND_ED25519, flags, segs, votes, b.pk, b.sig)
    assert np.array_equal(st.astype(np.uint8), ref)
    assert ok == bool(ref.all())
    # the same entries through host-built messages
    ok2, st2 = ctx.verify_batch_ex(N.TMV_KIND_ED25519, flags, b.pk, b.sig, b.msg, b.off)
    assert np.array_equal(st, st2)


def test_verify_votes_sr25519(ctx):
    from tendermint_amd.testing.sr25519_factory import Sr25519Signer, mini_from_secret
    rng = random.Random(54)
    tmpls, votes, msgs = V.random_votes(rng, 10, 400)
    ents = []
    for i, m in enumerate(msgs):
        s = Sr25519Signer(mini_from_secret(b"key: %x" % (i % 31)))
        sig = s.sign(m, b"%d" % i)
        if i % 17 == 0:
            b = bytearray(sig)
            b[5] ^= 4
            sig = bytes(b)
        ents.append((s.public_key, m, sig))
    b = Batch.from_entries(ents)
    ref = C.sr25519_status_packed(b.pk, b.sig, b.msg, b.off, threads=8)
    segs = [V.segments(t) for t in tmpls]
    for flags in (N.TMV_FLAG_KEY_CACHE, 0):
        ok, st = ctx.verify_votes(N.TMV_KIND_SR25519, flags, segs, votes, b.pk, b.sig)
        assert np.array_equal(st, ref)


def test_verify_votes_large_batch_equation(ctx):
    """Through the batch equation (the flag: 20k is below the default
    threshold of 32768): device messages feed the MSM pipeline; honest
    entries all valid, flipped ones caught."""
    rng = random.Random(55)
    n = 20000
    tmpls, votes, b = _signed_votes(rng, 60, n, bad_frac=0.002)
    _, ref = C.ed25519_verify_packed(b.pk, b.sig, b.msg, b.off, threads=8)
    segs = [V.segments(t) for t in tmpls]
    ok, st = ctx.verify_votes(N.TMV_KIND_ED25519, N.TMV_FLAG_BATCH_EQUATION, segs, votes, b.pk, b.sig)
    assert np.array_equal(st.astype(np.uint8), ref)
