"""Every multi-GPU code path on GPU hardware, on the one-GPU box (VERDICT r03
next #1):

* RCCL: a world-size-1 "nccl" process group (torch.distributed over RCCL on
  the device) runs the collectives `bench.py --gpus N` issues --
  shard.all_gather_validity (packed bitmaps, sizes that are not multiples of
  8), shard.all_gather_statuses (int8 statuses with the sr25519 Add errors
  -1 / -2) and the MAX all-reduce of the timing -- on device tensors, each
  compared with the local vector.
* Multi-device contexts: tmv_open_logical(mask, 2 / 3) (test aid) gives
  GPU 0 to the context as 2 / 3 devices, each with its own streams, host
  lanes, workspaces and key cache, so run_batch's shard plan (one
  contiguous shard per device, chunks over each device's lanes, harvest in
  launch order) runs with real streams -- the in-process path C4's
  "commits sharded across 8 GPUs" takes (internal/blocksync/pool.go:32-35,
  internal/blocksync/reactor.go:582-586).  A C4 window (600 blocks x 175
  validators: 1,200 commit checks), a C3 light window (1,000 headers x 100
  validators) and a streamed 2.56 M C2 host batch each equal one device's
  results and the C oracle's.
"""
import os
import random
import socket
from concurrent.futures import ProcessPoolExecutor

import numpy as np
import pytest

import at_size as A
import chain_fixtures as CF
import light_ref as L
import oracle_c
from tendermint_amd import _native as N, host as H
from tendermint_amd.testing.factory import Batch, make_block_chain, make_c2_batch, make_light_chain

pytestmark = pytest.mark.gpu
CHAIN = "test_chain_id"


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_rccl_world1_gathers():
    """The first RCCL execution: a one-rank nccl group on cuda:0 gathers
    validity bitmaps and int8 statuses and reduces the timing as bench.py
    does; every gathered vector equals the local one."""
    import torch
    import torch.distributed as dist
    from tendermint_amd.shard import all_gather_statuses, all_gather_validity
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    assert dist.is_nccl_available()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=dev)
    try:
        assert dist.get_backend() == "nccl"
        g = torch.Generator().manual_seed(4)
        for n in (1, 7, 8, 9, 10_000, 10_003, 160_001):
            st = torch.randint(-2, 2, (n,), generator=g, dtype=torch.int8).to(dev)
            v = all_gather_validity(st, [n])
            assert v.device == dev and v.dtype == torch.uint8
            assert torch.equal(v, (st == 1).to(torch.uint8)), n
            s = all_gather_statuses(st, [n])
            assert torch.equal(s, st), n
            assert int((s < 0).sum()) == int((st < 0).sum())
        # a shorter local vector than the largest count pads, then trims
        st = torch.randint(0, 2, (999,), generator=g, dtype=torch.int8).to(dev)
        assert torch.equal(all_gather_statuses(st, [999]), st)
        t = torch.tensor([1.25], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        assert float(t.item()) == 1.25
        dist.barrier()
        torch.cuda.synchronize()
    finally:
        dist.destroy_process_group()


@pytest.fixture(scope="module")
def contexts():
    """One-device, two-device and three-device contexts on GPU 0."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    out = {}
    for k in (1, 2, 3):
        out[k] = N.Context(1, logical=k)  # tmv_open_logical (test aid)
        assert out[k].num_devices() == k
    yield out
    for c in out.values():
        c.close()


def test_logical_devices_have_own_key_caches(contexts):
    caps = {k: c.key_cache_stats()["capacity"] for k, c in contexts.items()}
    assert caps[2] == 2 * caps[1] and caps[3] == 3 * caps[1]


def test_c4_window_sharded(contexts):
    """A blocksync window of 600 blocks (1,200 jobs: the light check of each
    block's successor's LastCommit, then the full check of its own) through
    tmv_verify_commits on 1, 2 and 3 devices: identical results, equal to
    oracle/light_ref.py with the C oracle's signature verdicts."""
    vals, blocks, pv = make_block_chain(602, 175, packed=True)
    rng = random.Random(0x4C4)
    picks = sorted(rng.sample(range(1, 600), 8))
    for n_pick, c in enumerate(picks):
        i = rng.randrange(175)
        A.corrupt_sig(blocks[c + 1].last_commit, i, pv, int(pv.commit_off[c]) + i, rng, s_plus_l=(n_pick == 0))
    vec = A.oracle_vector(pv)
    jobs, want = [], []
    ov = CF.valset(vals)
    with L.signature_oracle(A.Verdicts(pv, vec)):
        for i in range(1, 601):
            f, s2 = blocks[i], blocks[i + 1]
            jobs.append(H.CommitJob(H.MODE_LIGHT, CHAIN, vals, f.block_id, f.height, s2.last_commit))
            e = L.verify_commit_light(CHAIN, ov, CF.block_id(f.block_id), f.height, CF.commit(s2.last_commit))
            want.append(None if e is None else e.text)
            jobs.append(H.CommitJob(H.MODE_FULL, CHAIN, vals, blocks[i - 1].block_id, f.height - 1, f.last_commit))
            e = L.verify_commit(CHAIN, ov, CF.block_id(blocks[i - 1].block_id), f.height - 1, CF.commit(f.last_commit))
            want.append(None if e is None else e.text)
    assert sum(w is not None for w in want) >= len(picks)
    for k, ctx in contexts.items():
        for _ in range(2):  # cold, then warm key caches
            got = H.verify_commits(ctx, jobs)
            diff = [j for j, (g, w) in enumerate(zip(got, want)) if g != w]
            assert not diff, f"{k} devices, jobs {diff[:4]}: {[got[j] for j in diff[:2]]} vs {[want[j] for j in diff[:2]]}"


def test_c3_window_sharded(contexts):
    """A light window of 1,000 headers x 100 validators (VerifyAdjacent each,
    one validator rotated per height) through tmv_light_verify_many on 1, 2
    and 3 devices: identical results, equal to the oracle's."""
    trusted, blocks, pv = make_light_chain(1000, 100, packed=True)
    now = (blocks[-1].signed_header.header.time[0] + 5, 0)
    rng = random.Random(0x3C3)
    picks = sorted(rng.sample(range(1, 1001), 8))
    for n_pick, c in enumerate(picks):
        i = rng.randrange(100)
        A.corrupt_sig(blocks[c - 1].signed_header.commit, i, pv, int(pv.commit_off[c]) + i, rng,
                      s_plus_l=(n_pick == 0))
    blocks[500].signed_header.header.app_hash = b"tampered"
    vec = A.oracle_vector(pv)
    conv = CF.OracleBlocks()
    now_ns = now[0] * L.NS + now[1]
    want = []
    with L.signature_oracle(A.Verdicts(pv, vec)):
        prev = conv(trusted)
        for lb in blocks:
            cur = conv(lb)
            e = L.verify_adjacent(prev.signed_header, cur.signed_header, cur.vals, A.PERIOD, now_ns, A.DRIFT)
            want.append((L.OK, None) if e is None else (e.kind, e.text))
            prev = cur
    jobs, prev = [], trusted
    for lb in blocks:
        jobs.append(H.LightJob(prev.signed_header, None, lb.signed_header, lb.vals, A.PERIOD, now, A.DRIFT,
                               mode=H.LIGHT_ADJACENT))
        prev = lb
    assert 500 in [h for h, w in enumerate(want) if w[0] != L.OK]
    for k, ctx in contexts.items():
        got = H.light_verify_many(ctx, jobs)
        diff = [h for h, (g, w) in enumerate(zip(got, want)) if g != w]
        assert not diff, f"{k} devices, headers {diff[:4]}: {[got[h] for h in diff[:2]]} vs {[want[h] for h in diff[:2]]}"


def _c2(seed):
    return make_c2_batch(10_000, seed=seed)


def test_streamed_c2_host_batch_sharded(contexts):
    """256 C2 batches (2.56 M host-resident signatures, 8 distinct batches
    repeated) through tmv_verify_batch_ex's streamed batch-equation path on
    1, 2 and 3 devices: identical vectors, equal to the C oracle's (each
    distinct batch checked by the oracle once)."""
    with ProcessPoolExecutor(8) as ex:
        base = list(ex.map(_c2, [0xD2 + j for j in range(8)]))
    want1 = [oracle_c.ed25519_verify_packed(b.pk, b.sig, b.msg, b.off, threads=16)[1] for b in base]
    hb = Batch.concat([base[j % 8] for j in range(256)])
    want = np.concatenate([want1[j % 8] for j in range(256)]).astype(np.int8)
    assert int(want.sum()) == 256 * 9950
    for k, ctx in contexts.items():
        _, st = ctx.verify_batch_ex(N.TMV_KIND_ED25519, N.TMV_FLAG_BATCH_EQUATION, hb.pk, hb.sig, hb.msg, hb.off)
        bad = np.flatnonzero(np.asarray(st, np.int8) != want)
        assert not len(bad), f"{k} devices: entries {bad[:8]} differ from the oracle"


def test_c5_mixed_host_batch_sharded(contexts):
    """A C5-shaped mixed ed25519 + sr25519 host batch (a 20k mixed base
    tiled to 200k, ~1% of each kind corrupted) through the batch equation on
    1, 2 and 3 devices: identical status vectors (sr25519 Add errors
    included), equal to the C oracle's statuses of the base, tiled."""
    from tendermint_amd.testing.factory import make_mixed_batch
    kind, base = make_mixed_batch(20_000)
    ed = np.flatnonzero(kind == 0)
    sr = np.flatnonzero(kind == 1)
    want1 = np.zeros(base.n, np.int8)
    be, bs = base.take(ed), base.take(sr)
    want1[ed] = oracle_c.ed25519_verify_packed(be.pk, be.sig, be.msg, be.off, threads=16)[1]
    want1[sr] = oracle_c.sr25519_status_packed(bs.pk, bs.sig, bs.msg, bs.off, threads=16)
    n = 200_000
    idx = np.arange(n) % base.n
    hb = base.take(idx)
    kinds = np.ascontiguousarray(kind[idx])
    want = want1[idx]
    assert (want < 0).any() and (want == 0).any()
    for k, ctx in contexts.items():
        _, st = ctx.verify_mixed_batch_ex(N.TMV_FLAG_BATCH_EQUATION, kinds, hb.pk, hb.sig, hb.msg, hb.off)
        bad = np.flatnonzero(np.asarray(st, np.int8) != want)
        assert not len(bad), f"{k} devices: entries {bad[:8]}: {np.asarray(st)[bad[:8]]} vs {want[bad[:8]]}"
