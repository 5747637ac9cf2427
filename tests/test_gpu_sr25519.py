"""GPU parity for sr25519 (k_prep<SR> + k_verify_quad<SR>) and mixed
ed25519+sr25519 batches (k_partition) vs the CPU oracle / golden vectors."""
import numpy as np
import pytest

import oracle_c as C
from tendermint_amd.testing.factory import make_sr25519_batch, make_mixed_batch

pytestmark = pytest.mark.gpu


def test_golden_sr25519(ctx, golden):
    vs = golden("sr25519_vectors.json")["vectors"]
    ents = [(bytes.fromhex(v["pk"]), bytes.fromhex(v["msg"]), bytes.fromhex(v["sig"])) for v in vs]
    ok, st = ctx.sr25519_verify_batch(*C.pack(ents))
    assert [int(x) for x in st] == [v["status"] for v in vs]
    assert ok is False


def test_sr25519_batch_vs_oracle(ctx):
    b = make_sr25519_batch(3000, bad_frac=0.05)
    ok, st = ctx.sr25519_verify_batch(b.pk, b.sig, b.msg, b.off)
    ref = C.sr25519_status_packed(b.pk, b.sig, b.msg, b.off, threads=8)
    assert np.array_equal(st, ref)
    assert ok == bool((ref == 1).all())


def test_sr25519_all_valid(ctx):
    b = make_sr25519_batch(500, bad_frac=0.0)
    ok, st = ctx.sr25519_verify_batch(b.pk, b.sig, b.msg, b.off)
    assert ok and (st == 1).all()


def test_mixed_batch_vs_oracle(ctx):
    kind, b = make_mixed_batch(4000)
    ok, st = ctx.verify_mixed_batch(kind, b.pk, b.sig, b.msg, b.off)
    ed = kind == 0
    idx_ed, idx_sr = np.nonzero(ed)[0], np.nonzero(~ed)[0]
    for idx, fn in ((idx_ed, "ed"), (idx_sr, "sr")):
        ents = [b.entry(int(i)) for i in idx]
        pk, sig, msg, off = C.pack(ents)
        if fn == "ed":
            _, ref = C.ed25519_verify_packed(pk, sig, msg, off, threads=8)
            ref = ref.astype(np.int8)
        else:
            ref = C.sr25519_status_packed(pk, sig, msg, off, threads=8)
        assert np.array_equal(st[idx], ref), fn
    assert ok is False


def test_mixed_unknown_kind_is_invalid(ctx):
    kind, b = make_mixed_batch(64, seed=3)
    kind = kind.copy()
    kind[5] = 7
    _, st = ctx.verify_mixed_batch(kind, b.pk, b.sig, b.msg, b.off)
    assert st[5] == 0


@pytest.mark.parametrize("n", [150, 4000])
@pytest.mark.parametrize("flag", ["per_entry", "batch", "key_cache"])
def test_sr25519_transcript_lengths(ctx, n, flag):
    """Every message length around the register-state transcript's range
    (98..127 bytes, merlin_dev.h sr25519_challenge_fast) and outside it
    (generic STROBE path), mixed in the same waves, at any alignment, with a
    fraction of message bit flips -- vs the oracle, on the per-entry,
    batch-equation and key-cached kernels (small n: the latency kernels)."""
    import random
    from tendermint_amd import _native as N
    from tendermint_amd.testing.factory import Batch
    from tendermint_amd.testing.sr25519_factory import Sr25519Signer, mini_from_secret
    rng = random.Random(9127 + n)
    signers = [Sr25519Signer(mini_from_secret(b"len: %x" % k)) for k in range(16)]
    ents = []
    for i in range(n):
        mlen = 90 + i % 46 if i % 5 else rng.randrange(200)
        msg = bytes(rng.randrange(256) for _ in range(mlen))
        s = signers[i % len(signers)]
        sig = s.sign(msg, b"%d" % i)
        if i % 13 == 0 and msg:
            b = bytearray(msg)
            b[rng.randrange(len(b))] ^= 1 << rng.randrange(8)
            msg = bytes(b)
        ents.append((s.public_key, msg, sig))
    b = Batch.from_entries(ents)
    ref = C.sr25519_status_packed(b.pk, b.sig, b.msg, b.off, threads=8)
    assert (ref == 1).sum() > n // 2 and (ref == 0).sum() > 0
    flags = {"per_entry": N.TMV_FLAG_PER_ENTRY, "batch": N.TMV_FLAG_BATCH_EQUATION,
             "key_cache": N.TMV_FLAG_KEY_CACHE}[flag]
    _, st = ctx.verify_batch_ex(N.TMV_KIND_SR25519, flags, b.pk, b.sig, b.msg, b.off)
    assert np.array_equal(st, ref)
