"""GPU parity of the half-size-scalar per-entry check (halfscalar.h,
k_verify_quad / k_verify_quad_list): [8]([b]B + [u](-R) + [v](-A)) == O with
|u|, v < 2^127 (sr25519: the Ristretto identity) must give the reference's
validity bit for every input.  Every path that runs the per-entry kernels --
the per-entry pipeline with LDS tables (<= 12,288 entries) and with global
tables, the batch equation's compacted fallback of failing groups, the
located fallback's entry list (launches >= TMV_LOCATE_MIN entries) -- is compared with
the C oracle in three modes, set through the library's test hook
(tmv_internal_option "half_scalars"): 1 (the product), 0 (the full 253-bit
k, the rounds 1-4 check, which an entry whose reduction does not finish
takes) and 2 (every third entry on the full-k path beside half-size quads of
the same wave)."""
import numpy as np
import pytest

import oracle_c as C
from tendermint_amd import _native as N
from tendermint_amd.testing.factory import Batch, make_c2_batch, make_mixed_batch

pytestmark = pytest.mark.gpu

MODES = ("1", "0", "2")


def _edge_batch(golden):
    vs = golden("ed25519_vectors.json")["vectors"]
    ents = [(bytes.fromhex(v["pk"]), bytes.fromhex(v["msg"]), bytes.fromhex(v["sig"])) for v in vs]
    g = golden("zip215_small_order.json")
    msg = bytes.fromhex(g["msg"])
    ents += [(bytes.fromhex(a), msg, bytes.fromhex(r) + bytes(32)) for a, r in g["pairs_all_valid_with_S0"]]
    return C.pack(ents)


@pytest.fixture
def half_mode():
    """The half-size scalar mode through the library's test hook
    (tmv_internal_option "half_scalars": 1 = the product, 0 = every entry on
    the full-k chain, 2 = every third entry); reset to 1 afterwards."""
    import ctypes
    L = N.lib()
    L.tmv_internal_option.argtypes = [ctypes.c_char_p, ctypes.c_int64]

    def set_mode(mode):
        assert L.tmv_internal_option(b"half_scalars", int(mode)) == 0

    yield set_mode
    set_mode(1)


@pytest.fixture(scope="module")
def c2_mix():
    """The edge vectors ahead of 3 C2 batches' worth of entries (3,300)."""
    return Batch.concat([make_c2_batch(1100, seed=0xA0 + j) for j in range(3)])


@pytest.mark.parametrize("mode", MODES)
def test_ed25519_per_entry_and_fallback(ctx, golden, c2_mix, mode, half_mode, monkeypatch):
    half_mode(mode)
    pk, sig, msg, off = _edge_batch(golden)
    _, want = C.ed25519_verify_packed(pk, sig, msg, off)
    for flags in (N.TMV_FLAG_PER_ENTRY, N.TMV_FLAG_BATCH_EQUATION):
        _, got = ctx.verify_batch_ex(N.TMV_KIND_ED25519, flags, pk, sig, msg, off)
        assert np.array_equal(np.asarray(got, np.uint8), want), f"edge vectors, flags {flags}, mode {mode}"
    b = c2_mix
    _, want = C.ed25519_verify_packed(b.pk, b.sig, b.msg, b.off, threads=8)
    assert 0 < int(want.sum()) < b.n
    for flags in (N.TMV_FLAG_PER_ENTRY, N.TMV_FLAG_BATCH_EQUATION):
        _, got = ctx.verify_batch_ex(N.TMV_KIND_ED25519, flags, b.pk, b.sig, b.msg, b.off)
        bad = np.flatnonzero(np.asarray(got, np.uint8) != want)
        assert not len(bad), f"flags {flags}, mode {mode}: entries {bad[:8]}"


@pytest.mark.parametrize("mode", ("1", "2"))
def test_ed25519_per_entry_global_tables(ctx, mode, half_mode, monkeypatch):
    """20k entries per entry: more than 768 quad blocks, so the -A / -R tables
    live in global memory (GT) outside the fallback too."""
    half_mode(mode)
    b = Batch.concat([make_c2_batch(10_000, seed=0xB0 + j) for j in range(2)])
    _, want = C.ed25519_verify_packed(b.pk, b.sig, b.msg, b.off, threads=16)
    _, got = ctx.verify_batch_ex(N.TMV_KIND_ED25519, N.TMV_FLAG_PER_ENTRY, b.pk, b.sig, b.msg, b.off)
    assert np.array_equal(np.asarray(got, np.uint8), want)


@pytest.mark.parametrize("mode", MODES)
def test_sr25519_statuses(ctx, mode, half_mode, monkeypatch):
    """sr25519 (and mixed) statuses 1 / 0 / -1 / -2 per entry and through the
    batch equation's fallback, against the C oracle."""
    half_mode(mode)
    kind, mb = make_mixed_batch(4000, seed=0x77)
    ed, sr = np.flatnonzero(kind == 0), np.flatnonzero(kind == 1)
    want = np.zeros(mb.n, np.int8)
    be, bs = mb.take(ed), mb.take(sr)
    want[ed] = C.ed25519_verify_packed(be.pk, be.sig, be.msg, be.off, threads=8)[1]
    want[sr] = C.sr25519_status_packed(bs.pk, bs.sig, bs.msg, bs.off, threads=8)
    assert (want[sr] == 1).any() and (want[sr] == 0).any()
    for flags in (N.TMV_FLAG_PER_ENTRY, N.TMV_FLAG_BATCH_EQUATION):
        _, got = ctx.verify_mixed_batch_ex(flags, kind, mb.pk, mb.sig, mb.msg, mb.off)
        bad = np.flatnonzero(np.asarray(got, np.int8) != want)
        assert not len(bad), f"flags {flags}, mode {mode}: entries {bad[:8]}"
        _, got = ctx.verify_batch_ex(N.TMV_KIND_SR25519, flags, bs.pk, bs.sig, bs.msg, bs.off)
        assert np.array_equal(np.asarray(got, np.int8), want[sr])


@pytest.mark.parametrize("mode", ("1", "2"))
def test_located_fallback_list(ctx, mode, half_mode, monkeypatch):
    """A 160k-entry C2-shaped launch runs the located fallback: its entry
    list goes through k_verify_quad_list (global tables, grid-stride)."""
    half_mode(mode)
    monkeypatch.setenv("TMV_LOCATE_MIN", "150000")  # 160k entries: the located pass
    base = [make_c2_batch(10_000, seed=0xC0 + j) for j in range(4)]
    want1 = [C.ed25519_verify_packed(b.pk, b.sig, b.msg, b.off, threads=16)[1] for b in base]
    b = Batch.concat([base[j % 4] for j in range(16)])
    want = np.concatenate([want1[j % 4] for j in range(16)])
    _, got = ctx.verify_batch_ex(N.TMV_KIND_ED25519, N.TMV_FLAG_BATCH_EQUATION, b.pk, b.sig, b.msg, b.off)
    bad = np.flatnonzero(np.asarray(got, np.uint8) != want)
    assert not len(bad), f"mode {mode}: entries {bad[:8]}"
