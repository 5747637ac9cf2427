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
