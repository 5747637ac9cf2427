"""Streamed mixed ed25519 + sr25519 host batches (tmverify_runtime.cpp
mixed_check_streamed): the caller's pages DMA'd part by part, each part split
by key kind on the device into the two kinds' work-slot lists at bases the
host counted, each kind's pipeline running the groups the parts complete,
one tail per kind.  The statuses must equal the C oracle's for every
layout of kinds over the parts (the unstreamed host path is an A/B variant
now, -DTMV_AB builds only; the device-resident mixed path is tested in
test_gpu_configs.py): runs of one kind longer than a part (a kind absent from whole parts,
groups spanning parts), alternating kinds, unknown kinds (status 0) and a
kind absent altogether (crypto/batch/batch.go:11-21 mixed batches)."""
import numpy as np
import pytest

import oracle_c as C
from tendermint_amd import _native as N
from tendermint_amd.testing.factory import make_mixed_batch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def base():
    kind, mb = make_mixed_batch(20_000, seed=0x5EED)
    ed, sr = np.flatnonzero(kind == 0), np.flatnonzero(kind == 1)
    want = np.zeros(mb.n, np.int8)
    be, bs = mb.take(ed), mb.take(sr)
    want[ed] = C.ed25519_verify_packed(be.pk, be.sig, be.msg, be.off, threads=16)[1]
    want[sr] = C.sr25519_status_packed(bs.pk, bs.sig, bs.msg, bs.off, threads=16)
    return kind, mb, want


def _layout(kind, name, n):
    """Entry order over the base (indices) for a named layout."""
    ed, sr = np.flatnonzero(kind == 0), np.flatnonzero(kind == 1)
    if name == "interleaved":
        return np.arange(n) % len(kind)
    if name == "runs":  # 150k ed25519, then 150k sr25519, then interleaved (runs longer than a part)
        a = ed[np.arange(150_000) % len(ed)]
        b = sr[np.arange(150_000) % len(sr)]
        c = np.arange(n - 300_000) % len(kind)
        return np.concatenate([a, b, c])
    if name == "ed_only":
        return ed[np.arange(n) % len(ed)]
    if name == "sr_only":
        return sr[np.arange(n) % len(sr)]
    raise ValueError(name)


@pytest.mark.parametrize("layout", ["interleaved", "runs", "ed_only", "sr_only"])
def test_mixed_streamed_vs_oracle(ctx, base, layout, monkeypatch):
    kind, mb, want1 = base
    n = 420_000
    idx = _layout(kind, layout, n)
    hb = mb.take(idx)
    kinds = np.ascontiguousarray(kind[idx]).astype(np.uint8)
    want = want1[idx].copy()
    if layout == "interleaved":  # unknown key kinds: status 0, never verified
        kinds[::997] = 7
        want[::997] = 0
    for lmin in ("150000", "400000"):  # each kind's half with and without the located fallback
        monkeypatch.setenv("TMV_LOCATE_MIN", lmin)
        _, st = ctx.verify_mixed_batch_ex(N.TMV_FLAG_BATCH_EQUATION, kinds, hb.pk, hb.sig, hb.msg, hb.off)
        got = np.asarray(st, np.int8)
        bad = np.flatnonzero(got != want)
        assert not len(bad), (f"{layout}, TMV_LOCATE_MIN={lmin}: entries {bad[:8]}: "
                              f"{got[bad[:8]]} vs {want[bad[:8]]}")


def test_mixed_streamed_stats(ctx, base, monkeypatch):
    """The batch statistics see both kinds' groups on the streamed path (the
    partition's device counts): ed25519 in groups of 64 streamed
    (tmverify_runtime.cpp make_opts: p_ed_streamed, even at >= TMV_LOCATE_MIN
    entries, 150k here), sr25519 in groups of 64."""
    monkeypatch.setenv("TMV_LOCATE_MIN", "150000")
    kind, mb, _ = base
    idx = np.arange(300_000) % mb.n
    hb = mb.take(idx)
    kinds = np.ascontiguousarray(kind[idx])
    ctx.set_batch_options(stats=True)
    g0 = ctx.batch_stats()["groups"]
    ctx.verify_mixed_batch_ex(N.TMV_FLAG_BATCH_EQUATION, kinds, hb.pk, hb.sig, hb.msg, hb.off)
    groups = ctx.batch_stats()["groups"] - g0
    ctx.set_batch_options()
    n_ed, n_sr = int(np.sum(kinds == 0)), int(np.sum(kinds == 1))
    g = lambda k, m: (k + m - 1) // m  # noqa: E731
    assert groups == g(n_ed, 64) + g(n_sr, 64), groups
