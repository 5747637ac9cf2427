"""GPU parity of the batch equation: the
random-linear-combination group check (k_msm_sort / k_msm_accum /
k_msm_group) with the per-entry fallback over failing groups must give the
same validity vector as the oracle, and honest groups must actually pass the
equation (tmv_batch_stats), so a broken MSM cannot hide behind the fallback.
"""
import os

import numpy as np
import pytest

import oracle_c as C
from tendermint_amd import _native as N
from tendermint_amd.testing.factory import (make_c2_batch, make_commit_batch, make_mixed_batch,
                                            make_sr25519_batch)

pytestmark = pytest.mark.gpu

SEED = bytes(range(32))
ED, SR = N.TMV_KIND_ED25519, N.TMV_KIND_SR25519
BEQ = N.TMV_FLAG_BATCH_EQUATION


@pytest.fixture(scope="module")
def bctx():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    c = N.Context(1)
    c.set_batch_options(seed=SEED, stats=True)
    yield c
    c.close()


@pytest.fixture(scope="module")
def honest():
    return make_commit_batch(1500)


def _run(ctx, kind, b, sub=False, **opts):
    ctx.set_batch_options(seed=opts.pop("seed", SEED), stats=True, **opts)
    s0 = ctx.batch_stats()
    ok, st = ctx.verify_batch_ex(kind, BEQ, b.pk, b.sig, b.msg, b.off)
    s1 = ctx.batch_stats()
    r = (ok, st, s1["groups"] - s0["groups"], s1["failed"] - s0["failed"])
    if sub:
        r += (s1["subgroups"] - s0["subgroups"], s1["sub_failed"] - s0["sub_failed"])
    return r


def test_c2_full_size_bit_exact(bctx, golden):
    g = golden("c2_expected.json")
    b = make_c2_batch()
    ok, st, groups, failed = _run(bctx, ED, b)
    bits = np.packbits(st.astype(np.uint8), bitorder="little").tobytes().hex()
    assert bits == g["valid_bits_hex"] and not ok
    assert groups == (10_000 + 63) // 64
    # exactly the groups holding a bit-flipped entry that still decodes fail
    want = C.failing_groups(C.ed25519_prechecks(b.pk, b.sig), st == 1, 64)
    assert 0 < want <= 20 and failed == want, (failed, want)


def test_c2_subgroups_bisect(bctx):
    """k_msm_subcheck (groups >= 256): every sub-group (8 entries) of a failing group is
    re-checked; exactly those holding a pre-valid invalid entry fail, so the
    per-entry fallback only runs over the 16-entry blocks that hold them."""
    b = make_c2_batch()
    ok, st, groups, failed, subs, sub_failed = _run(bctx, ED, b, sub=True, group_log2=8)
    pre = C.ed25519_prechecks(b.pk, b.sig)
    assert failed == C.failing_groups(pre, st == 1, 256) and failed > 0
    assert subs == failed * 32
    assert sub_failed == C.failing_groups(pre, st == 1, 8) and 0 < sub_failed < subs
    # m = 64 (the default for C2-sized launches) skips the bisection
    ok, st2, groups, failed, subs, sub_failed = _run(bctx, ED, b, sub=True)
    assert np.array_equal(st, st2) and failed > 0 and subs == 0


@pytest.mark.parametrize("n,bad", [
    (200, [0]), (200, [7, 8]), (200, [63, 64, 127]), (600, [255, 256, 511]), (1000, list(range(256, 512))),
    (1000, list(range(0, 1000, 9))), (999, [998]), (1001, [1000, 992]), (65, [64]),
])
def test_subgroup_placements(bctx, n, bad):
    """Invalid signatures at sub-group / block / group edges, whole failing
    groups, dense failures and ragged tails: the vector equals the oracle's
    and exactly the sub-groups holding a pre-valid invalid entry fail."""
    b = make_commit_batch(n, seed=11)
    sig = b.sig.copy()
    for i in bad:
        sig[64 * i + 5] ^= 0x10  # R byte: R mostly still decodes, the equation fails
    ok_o, vec_o = C.ed25519_verify_packed(b.pk, sig, b.msg, b.off, threads=4)
    ok, st, groups, failed, subs, sub_failed = _run(bctx, ED, _B(b.pk, sig, b.msg, b.off), sub=True, group_log2=8)
    assert ok == ok_o and np.array_equal(st.astype(np.uint8), vec_o)
    pre = C.ed25519_prechecks(b.pk, sig)
    assert failed == C.failing_groups(pre, vec_o == 1, 256) and subs == failed * 32
    assert sub_failed == C.failing_groups(pre, vec_o == 1, 8)


def test_sr25519_subgroups(bctx):
    b = make_sr25519_batch(600, seed=9, bad_frac=0.02)
    ok, st, groups, failed, subs, sub_failed = _run(bctx, SR, b, sub=True, group_log2=8)
    ref = C.sr25519_status_packed(b.pk, b.sig, b.msg, b.off, threads=8)
    assert np.array_equal(st, ref)
    pre = C.sr25519_prechecks(b.pk, b.sig)
    assert failed > 0 and subs == failed * 32 and sub_failed == C.failing_groups(pre, ref == 1, 8)


def test_honest_groups_pass(bctx, honest):
    ok, st, groups, failed = _run(bctx, ED, honest)
    assert ok and (st == 1).all()
    assert groups == (1500 + 63) // 64 and failed == 0


_C2S = {}


def _c2_small():
    if "b" not in _C2S:
        _C2S["b"] = make_c2_batch(2000, seed=5, edge_scale=5.0)
    return _C2S["b"]


def _c2_small_pre():
    if "pre" not in _C2S:
        b = _c2_small()
        _C2S["pre"] = C.ed25519_prechecks(b.pk, b.sig)
    return _C2S["pre"]


@pytest.mark.parametrize("m_log2,c", [(5, 4), (6, 5), (7, 6), (8, 7), (9, 8), (10, 9), (6, 9), (10, 4)])
def test_group_window_sweep(bctx, honest, m_log2, c):
    ok, st, groups, failed = _run(bctx, ED, honest, group_log2=m_log2, window_bits=c)
    assert ok and (st == 1).all() and failed == 0
    assert groups == (1500 + (1 << m_log2) - 1) >> m_log2
    b = _c2_small()
    ok, st, _, failed = _run(bctx, ED, b, group_log2=m_log2, window_bits=c)
    _, ref = C.ed25519_verify_packed(b.pk, b.sig, b.msg, b.off, threads=8)
    assert np.array_equal(st.astype(np.uint8), ref) and not ok
    assert failed == C.failing_groups(_c2_small_pre(), ref == 1, 1 << m_log2)


def test_zip215_small_order_matrix_passes_equation(bctx, golden):
    """All 196 small-order (A, R) pairs with S = 0 are valid under the
    cofactored equation: every group must pass, none may fall back."""
    g = golden("zip215_small_order.json")
    msg = bytes.fromhex(g["msg"])
    ents = [(bytes.fromhex(a), msg, bytes.fromhex(r) + bytes(32)) for a, r in g["pairs_all_valid_with_S0"]]
    ok, st, groups, failed = _run(bctx, ED, _B(*C.pack(ents)), group_log2=5)
    assert ok and (st == 1).all() and len(st) == 196
    assert groups == 7 and failed == 0


class _B:
    def __init__(self, pk, sig, msg, off):
        self.pk, self.sig, self.msg, self.off = pk, sig, msg, off


def test_golden_edge_vectors(bctx, golden):
    vs = golden("ed25519_vectors.json")["vectors"]
    b = _B(*C.pack([(bytes.fromhex(v["pk"]), bytes.fromhex(v["msg"]), bytes.fromhex(v["sig"])) for v in vs]))
    ok, st, _, _ = _run(bctx, ED, b, group_log2=5)
    assert [bool(x) for x in st] == [v["valid"] for v in vs] and not ok


@pytest.mark.parametrize("n", [1, 2, 31, 33, 64, 65, 1000])
def test_ragged_sizes(bctx, honest, n):
    b = _B(*C.pack([honest.entry(i) for i in range(n)]))
    ok, st, groups, failed = _run(bctx, ED, b)
    assert ok and (st == 1).all() and groups == (n + 63) // 64 and failed == 0


def test_fresh_randomness(bctx):
    """Production mode: a new getrandom() key per call; the vector is the same."""
    b = make_c2_batch(3000, seed=77, edge_scale=3.0)
    _, ref = C.ed25519_verify_packed(b.pk, b.sig, b.msg, b.off, threads=8)
    bctx.set_batch_options(seed=None, stats=True)
    for _ in range(3):
        ok, st = bctx.verify_batch_ex(ED, BEQ, b.pk, b.sig, b.msg, b.off)
        assert np.array_equal(st.astype(np.uint8), ref)


def test_sr25519_vs_oracle(bctx):
    b = make_sr25519_batch(2000, bad_frac=0.03)
    ok, st, groups, failed = _run(bctx, SR, b)
    ref = C.sr25519_status_packed(b.pk, b.sig, b.msg, b.off, threads=8)
    assert np.array_equal(st, ref) and ok == bool((ref == 1).all())
    want = C.failing_groups(C.sr25519_prechecks(b.pk, b.sig), ref == 1, 64)
    assert 0 < want < groups and failed == want, (failed, want)


def test_sr25519_honest_groups_pass(bctx):
    b = make_sr25519_batch(700, bad_frac=0.0, seed=11)
    ok, st, groups, failed = _run(bctx, SR, b)
    assert ok and (st == 1).all() and groups == 11 and failed == 0


def test_mixed_vs_per_entry(bctx):
    kind, b = make_mixed_batch(3000, seed=21)
    bctx.set_batch_options(seed=SEED, stats=True)
    s0 = bctx.batch_stats()
    ok, st = bctx.verify_mixed_batch_ex(BEQ, kind, b.pk, b.sig, b.msg, b.off)
    s1 = bctx.batch_stats()
    ok2, ref = bctx.verify_mixed_batch_ex(N.TMV_FLAG_PER_ENTRY, kind, b.pk, b.sig, b.msg, b.off)
    assert np.array_equal(st, ref) and ok == ok2
    groups, failed = s1["groups"] - s0["groups"], s1["failed"] - s0["failed"]
    assert groups == (1500 + 63) // 64 * 2 and failed < groups


def test_device_resident_entry_point(bctx):
    import torch
    b = make_c2_batch(4096, seed=3)
    _, ref = C.ed25519_verify_packed(b.pk, b.sig, b.msg, b.off, threads=8)
    dev = torch.device("cuda:0")
    t = {k: torch.from_numpy(np.ascontiguousarray(getattr(b, k))).to(dev) for k in ("pk", "sig", "msg", "off")}
    out = torch.zeros(b.n, dtype=torch.int8, device=dev)
    torch.cuda.synchronize()
    bctx.verify_batch_device_ex(0, ED, BEQ, 0, t["pk"].data_ptr(), t["sig"].data_ptr(), t["msg"].data_ptr(),
                                t["off"].data_ptr(), b.n, out.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().astype(np.uint8), ref)


@pytest.mark.parametrize("flags", [BEQ, N.TMV_FLAG_PER_ENTRY])
def test_multi_batch_launch(bctx, flags):
    """tmv_verify_batches_device: several independent batches (different
    sizes, one empty, one unaligned, one whose message offsets do not start
    at 0) in one launch equal separate checks."""
    import torch
    dev = torch.device("cuda:0")
    specs = [(make_c2_batch(700, seed=41, edge_scale=8.0), 0, 0), (make_c2_batch(0, seed=42), 0, 0),
             (make_c2_batch(1300, seed=43, edge_scale=4.0), 3, 0), (make_sr25519_batch(0), 0, 0),
             (make_c2_batch(65, seed=44, edge_scale=20.0), 1, 0), (make_c2_batch(300, seed=45, edge_scale=10.0), 2, 7)]
    keep, refs, want = [], [], []
    for b, shift, base in specs:
        if b.n == 0:
            refs.append(N.BatchRef(0, 0, 0, 0, 0, 0, 0))
            continue
        raw = {}
        for k in ("pk", "sig", "msg"):
            a = getattr(b, k)
            buf = torch.zeros(len(a) + 16, dtype=torch.uint8, device=dev)
            buf[shift:shift + len(a)] = torch.from_numpy(a).to(dev)
            raw[k] = buf
        off = torch.from_numpy((b.off + base).view(np.int32)).to(dev)
        out = torch.full((b.n,), -7, dtype=torch.int8, device=dev)
        keep += [raw, off, out]
        refs.append(N.BatchRef(raw["pk"].data_ptr() + shift, raw["sig"].data_ptr() + shift,
                               raw["msg"].data_ptr() + shift - base, off.data_ptr(), b.n, int(b.off[-1] - b.off[0]),
                               out.data_ptr()))
        _, ref = C.ed25519_verify_packed(b.pk, b.sig, b.msg, b.off, threads=8)
        want.append((out, ref))
    bctx.set_batch_options(seed=SEED, stats=True)
    torch.cuda.synchronize()
    bctx.verify_batches_device(0, ED, flags, refs, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    for out, ref in want:
        assert np.array_equal(out.cpu().numpy().astype(np.uint8), ref)


@pytest.mark.parametrize("kind,m_log2", [(ED, 0), (ED, 6), (SR, 0)], ids=["ed-default", "ed-64", "sr-default"])
def test_located_fallback_placements(bctx, kind, m_log2, monkeypatch):
    """Launches of >= TMV_LOCATE_MIN entries (400k by default; 150k here, read
    at every launch) re-check a failing group
    with index weights (j + 1) z_j and verify only the entry that locates;
    groups with two or more bad entries fall back to every entry.  One bad
    entry at each group edge (j = 0, 31, 63), pairs, a whole bad group and a
    ragged tail: the vector equals the oracle's."""
    monkeypatch.setenv("TMV_LOCATE_MIN", "150000")
    n = 150_000 + 37
    base = make_commit_batch(1500, seed=21) if kind == ED else make_sr25519_batch(1500, seed=22, bad_frac=0.0)
    b = base.tile(n)
    sig = b.sig.copy()
    bad = [0, 64 + 31, 128 + 63, 640 + 5, 640 + 6, 1280 + 1, 1280 + 40, 1280 + 62] + list(range(1920, 1984))
    bad += [n - 1, n - 30, 77_777, 149_999]
    for i in bad:
        sig[64 * i + 5] ^= 0x10  # R byte: R mostly still decodes, the equation fails
    bb = _B(b.pk, sig, b.msg, b.off)
    # default group size at this launch size: 128 for ed25519, 64 for sr25519
    m = 1 << m_log2 if m_log2 else (128 if kind == ED else 64)
    ok, st, groups, failed = _run(bctx, kind, bb, group_log2=m_log2)
    if kind == ED:
        ok_o, ref = C.ed25519_verify_packed(b.pk, sig, b.msg, b.off, threads=16)
        assert ok == ok_o and np.array_equal(st.astype(np.uint8), ref)
        pre = C.ed25519_prechecks(b.pk, sig)
    else:
        ref = C.sr25519_status_packed(b.pk, sig, b.msg, b.off, threads=16)
        assert np.array_equal(st, ref)
        pre = C.sr25519_prechecks(b.pk, sig)
    assert groups == (n + m - 1) // m
    assert failed == C.failing_groups(pre, ref == 1, m) and failed >= 3


def test_kernel_timing_records_each_launch(bctx):
    """tmv_kernel_timing (bench.py's dominant-kernel roofline): every
    batch-equation launch while it is on adds one k_msm_accum / k_msm_wpart /
    k_prep_fused record of positive duration; none while it is off; a read
    forgets what it returned; an unknown name is an argument error."""
    b = make_c2_batch(20_000, seed=91)
    for k in ("k_msm_accum", "k_msm_wpart", "k_prep_fused"):
        bctx.kernel_timing_read(k)
    bctx.kernel_timing(True)
    try:
        for _ in range(3):
            bctx.verify_batch_ex(ED, BEQ, b.pk, b.sig, b.msg, b.off)
    finally:
        bctx.kernel_timing(False)
    for k in ("k_msm_accum", "k_msm_wpart", "k_prep_fused"):
        ms, cnt = bctx.kernel_timing_read(k)
        assert cnt == 3 and ms > 0, (k, ms, cnt)
        assert bctx.kernel_timing_read(k) == (0.0, 0)
    bctx.verify_batch_ex(ED, BEQ, b.pk, b.sig, b.msg, b.off)
    assert bctx.kernel_timing_read("k_msm_accum") == (0.0, 0)
    with pytest.raises(N.NativeError):
        bctx.kernel_timing_read("k_nonexistent")


def test_multi_batch_launch_over_64(bctx):
    """More batches than one kernel argument holds (kMaxBatches = 64): 150
    batches of ragged sizes -- empty ones at the 64 / 128 edges -- gathered
    by three gather launches into one pipeline; each vector equals the
    oracle's, and 257 batches are refused."""
    import torch
    dev = torch.device("cuda:0")
    pool = make_c2_batch(3000, seed=47, edge_scale=6.0)
    _, ref_all = C.ed25519_verify_packed(pool.pk, pool.sig, pool.msg, pool.off, threads=8)
    t = {k: torch.from_numpy(getattr(pool, k)).to(dev) for k in ("pk", "sig", "msg")}
    doff = torch.from_numpy(pool.off.view(np.int32)).to(dev)
    refs, want, lo = [], [], 0
    for b in range(150):
        n = 0 if b in (63, 64, 127, 128) else 1 + (b * 7) % 37
        if n == 0:
            refs.append(N.BatchRef(0, 0, 0, 0, 0, 0, 0))
            continue
        n = min(n, pool.n - lo)
        out = torch.full((n,), -7, dtype=torch.int8, device=dev)
        refs.append(N.BatchRef(t["pk"].data_ptr() + 32 * lo, t["sig"].data_ptr() + 64 * lo, t["msg"].data_ptr(),
                               doff.data_ptr() + 4 * lo, n, int(pool.off[lo + n] - pool.off[lo]), out.data_ptr()))
        want.append((out, ref_all[lo:lo + n]))
        lo += n
    assert lo > 2000
    for flags in (BEQ, N.TMV_FLAG_PER_ENTRY):
        torch.cuda.synchronize()
        bctx.verify_batches_device(0, ED, flags, refs, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        for out, ref in want:
            assert np.array_equal(out.cpu().numpy().astype(np.uint8), ref), flags
    with pytest.raises(N.NativeError):
        bctx.verify_batches_device(0, ED, BEQ, [N.BatchRef(0, 0, 0, 0, 0, 0, 0)] * 257)


def _located_case(n=150_000 + 91, m=256):
    """n honest commit signatures (tiled) with bad entries placed so that
    some groups of m hold one bad entry and some two (S's low bit flipped: S
    stays canonical and R, A still decode, so every bad entry passes the
    pre-checks and fails only the equation)."""
    b = make_commit_batch(1500, seed=23).tile(n)
    sig = b.sig.copy()
    singles = [0, m + m - 1, 5 * m + 17, 9 * m + 200, 40 * m + 3, n - 2]
    pairs = [(12 * m + 1, 12 * m + 9), (30 * m + 100, 30 * m + 101)]
    for i in singles + [x for p in pairs for x in p]:
        sig[64 * i + 32] ^= 0x01
    return b, sig, singles, pairs


@pytest.mark.parametrize("m_log2,c", [(8, 8), (8, 6), (10, 9), (7, 6)])
def test_located_pass_width_and_metrics(bctx, m_log2, c, monkeypatch):
    """the located pass's weights z (j + 1) < 2^(128 + m_log2) need
    ceil((129 + m_log2) / c) windows.  With groups of 256 / 1024 (sub-group
    checks off) the located pass must still name every single bad entry:
    tmv_metrics counts one located group and one per-entry verification per
    single-bad group, and whole groups only for the two-bad ones; the vector
    equals the oracle's."""
    monkeypatch.setenv("TMV_LOCATE_MIN", "150000")  # the launch (150k + 91) runs the located pass
    m = 1 << m_log2
    b, sig, singles, pairs = _located_case(m=m)
    n = b.n
    bctx.set_batch_options(group_log2=m_log2, window_bits=c, seed=SEED, stats=True, subcheck=False)
    bctx.metrics_reset()
    try:
        ok, st = bctx.verify_batch_ex(ED, BEQ, b.pk, sig, b.msg, b.off)
        met = bctx.metrics()
    finally:
        bctx.set_batch_options(seed=SEED, stats=True)
    ok_o, ref = C.ed25519_verify_packed(b.pk, sig, b.msg, b.off, threads=16)
    assert ok == ok_o and np.array_equal(st.astype(np.uint8), ref)
    bad_groups = {i // m for i in singles} | {p[0] // m for p in pairs}
    assert met["groups_failed"] == len(bad_groups)
    assert met["located_groups"] == len(singles)
    whole = sum(min(m, n - (p[0] // m) * m) for p in pairs)
    assert met["fallback_signatures"] == len(singles) + whole
    assert met["calls"] == 1 and met["signatures"] == n and met["batch_eq_signatures"] == n
    assert met["h2d_bytes"] >= b.pk.nbytes + sig.nbytes + b.msg.nbytes and met["d2h_bytes"] == n
    assert met["host_signatures"] == n and met["verifies_per_s_host"] > 0


def test_metrics_counts_calls_and_resets(bctx):
    """tmv_metrics: calls, entries, the largest call and the batch-equation
    share over host-buffer and device-resident calls; reset zeroes them."""
    import torch
    bctx.metrics_reset()
    b = make_c2_batch(3000, seed=77)
    bctx.verify_batch_ex(ED, N.TMV_FLAG_PER_ENTRY, b.pk, b.sig, b.msg, b.off)
    bctx.verify_batch_ex(ED, BEQ, b.pk, b.sig, b.msg, b.off)
    dev = torch.device("cuda:0")
    t = {k: torch.from_numpy(getattr(b, k)).to(dev) for k in ("pk", "sig", "msg")}
    off = torch.from_numpy(b.off.view(np.int32)).to(dev)
    out = torch.zeros(b.n, dtype=torch.int8, device=dev)
    bctx.verify_batch_device_ex(0, ED, BEQ, 0, t["pk"].data_ptr(), t["sig"].data_ptr(), t["msg"].data_ptr(),
                                off.data_ptr(), 1000, out.data_ptr())
    torch.cuda.synchronize()
    met = bctx.metrics()
    assert (met["calls"], met["signatures"], met["max_batch"]) == (3, 7000, 3000)
    assert met["batch_eq_signatures"] == 4000 and met["host_signatures"] == 6000
    assert met["groups"] >= (3000 + 63) // 64 and met["groups_failed"] >= 1
    assert met["fallback_signatures"] >= met["groups_failed"]
    bctx.metrics_reset()
    met = bctx.metrics()
    assert all(v == 0 for k, v in met.items() if k not in ("key_cache_hits", "key_cache_misses"))


@pytest.mark.parametrize("kind", [ED, SR], ids=["ed25519", "sr25519"])
def test_duplicate_entries(bctx, kind):
    """The same signature many times in one group (a replayed vote): each copy
    gets its own random weight, but the points coincide, so one bucket adds a
    point to itself (and to its negation, digits of opposite sign) -- the
    complete addition law must hold there.  Groups of copies of a valid
    signature pass the equation; a group holding a copy of an invalid one
    fails, and every copy of it is invalid, as the oracle says."""
    base = make_commit_batch(200, seed=31) if kind == ED else make_sr25519_batch(200, seed=32, bad_frac=0.0)
    sig = base.sig.copy()
    bad = 5
    sig[64 * bad + 32] ^= 0x01  # S stays canonical: the entry fails the equation only
    idx = ([0] * 64                                  # one valid signature 64 times
           + [1 + (i // 2) for i in range(64)]       # 32 valid ones twice each
           + [bad] * 64                              # one invalid signature 64 times
           + [3] * 63 + [bad]                        # 63 copies of a valid one, one invalid
           + list(range(40, 104))                    # 64 distinct
           + [7, bad] * 16 + [8] * 7)                # alternating, then a ragged tail
    ents = [(bytes(base.pk[32 * i:32 * i + 32]), bytes(base.msg[base.off[i]:base.off[i + 1]]),
             bytes(sig[64 * i:64 * i + 64])) for i in idx]
    b = _B(*C.pack(ents))
    ok, st, groups, failed = _run(bctx, kind, b, group_log2=6)
    if kind == ED:
        ok_o, ref = C.ed25519_verify_packed(b.pk, b.sig, b.msg, b.off, threads=8)
        assert ok == ok_o and np.array_equal(st.astype(np.uint8), ref)
    else:
        ref = C.sr25519_status_packed(b.pk, b.sig, b.msg, b.off, threads=8)
        assert np.array_equal(st, ref)
    assert int((ref != 1).sum()) == idx.count(bad)
    assert groups == (len(idx) + 63) // 64 == 6
    # the groups holding a copy of the invalid signature (the pairs' group too:
    # entry 5 is among them)
    assert failed == len({j // 64 for j, i in enumerate(idx) if i == bad}) == 4


def _bisect_case(kind, m, n=150_000 + 91):
    """Bad entries (S's low bit flipped: every pre-check passes) placed so
    that failing groups of m hold one bad entry, two in the same half (either
    half), two in different halves, three (two + one), and two in the ragged
    last group."""
    base = make_commit_batch(1500, seed=23) if kind == ED else make_sr25519_batch(1500, seed=24, bad_frac=0.0)
    b = base.tile(n)
    sig = b.sig.copy()
    h = m // 2
    bad = [0, m + m - 1, 5 * m + 17,                      # one bad entry
           12 * m + 1, 12 * m + 9,                        # two, first half
           14 * m + h + 3, 14 * m + m - 1,                # two, second half
           30 * m + 3, 30 * m + h + 4,                    # one in each half
           40 * m + 1, 40 * m + 2, 40 * m + m - 2,        # two + one
           n - 1, n - 2]                                  # the ragged last group
    for i in bad:
        sig[64 * i + 32] ^= 0x01
    return b, sig, bad


def _located_expect(bad, n, m):
    """(located, one-by-one) the located fallback gives: a failing group with
    one bad entry names it (one verification); a group with two or more is
    verified whole (its live entries).  (Round 5's bisection of such groups
    and the sub-group checks were measured slower and removed.)"""
    groups = {}
    for i in bad:
        groups.setdefault(i // m, []).append(i)
    located = fallback = 0
    for g, es in groups.items():
        if len(es) == 1:
            located += 1
            fallback += 1
        else:
            fallback += min(m, n - g * m)
    return located, fallback


@pytest.mark.parametrize("kind,m_log2", [(ED, 7), (ED, 8), (SR, 6)], ids=["ed-128", "ed-256", "sr-64"])
def test_located_two_bad_groups(bctx, kind, m_log2, monkeypatch):
    """The located fallback (TMV_LOCATE_MIN, 150k here, read at every launch)
    on groups holding one, two or more bad entries: tmv_metrics counts
    exactly the entries the rule implies (_located_expect), and the vector
    equals the oracle's."""
    monkeypatch.setenv("TMV_LOCATE_MIN", "150000")
    m = 1 << m_log2
    b, sig, bad = _bisect_case(kind, m)
    n = b.n
    bctx.set_batch_options(group_log2=m_log2, seed=SEED, stats=True, subcheck=False)
    bctx.metrics_reset()
    try:
        ok, st = bctx.verify_batch_ex(kind, BEQ, b.pk, sig, b.msg, b.off)
        met = bctx.metrics()
    finally:
        bctx.set_batch_options(seed=SEED, stats=True)
    if kind == ED:
        ok_o, ref = C.ed25519_verify_packed(b.pk, sig, b.msg, b.off, threads=16)
        assert ok == ok_o and np.array_equal(st.astype(np.uint8), ref)
        assert int((ref == 0).sum()) == len(bad)
    else:
        ref = C.sr25519_status_packed(b.pk, sig, b.msg, b.off, threads=16)
        assert np.array_equal(st, ref)
        assert int((ref != 1).sum()) == len(bad)
    located, fallback = _located_expect(bad, n, m)
    assert met["groups_failed"] == len({i // m for i in bad})
    assert (met["located_groups"], met["fallback_signatures"]) == (located, fallback), met


@pytest.mark.parametrize("kind", [ED, SR])
def test_chain_paths(bctx, kind):
    """One case through both chains of round 5: the batch equation (its
    Horner beside the helper workgroups that reduce every entry's k, then the
    failing groups re-verified one by one) and the per-entry pipeline (k
    reduced once by the prep's hash lane) -- each gives the oracle's vector.
    (Their switched-off forms were A/B knobs, now in -DTMV_AB builds only.)"""
    b, sig, bad = _bisect_case(kind, 64, n=20_000 + 37)
    if kind == ED:
        ok_o, ref = C.ed25519_verify_packed(b.pk, sig, b.msg, b.off, threads=16)
    else:
        ref = C.sr25519_status_packed(b.pk, sig, b.msg, b.off, threads=16)
    for flags in (BEQ, N.TMV_FLAG_PER_ENTRY):
        bctx.set_batch_options(seed=SEED, stats=True)
        s0 = bctx.batch_stats()
        ok, st = bctx.verify_batch_ex(kind, flags, b.pk, sig, b.msg, b.off)
        s1 = bctx.batch_stats()
        if kind == ED:
            assert ok == ok_o and np.array_equal(st.astype(np.uint8), ref), flags
        else:
            assert np.array_equal(st, ref), flags
        if flags == BEQ:
            assert s1["failed"] - s0["failed"] == len({i // 64 for i in bad if i < b.n})
