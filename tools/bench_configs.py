#!/usr/bin/env python3
"""Secondary measurements for BASELINE configs 1, 3, 4, 5 (one JSON line
each; the headline line is bench.py's C2).  Single GPU.

  C1  types.VerifyCommit, 150 validators: p50/p99 latency, cold + warm key cache
  C3  light sequential: H headers x 100 validators (VerifyAdjacent: header
      and validator-set hashes + VerifyCommitLight, 67 signatures read per
      header), window-batched through tmv_light_verify_many
  C4  blocksync replay: B blocks x 175 validators (light + full check per
      block = 292 reference verifications, 175 unique)
  (C3 / C4 native: one window at a time, and 2 / 3 windows in flight on
  caller threads -- chains.in_order, the drivers' default depth 2)
  C5  mixed ed25519 + sr25519 batch (kernel path, inputs resident)
"""
import argparse, json, os, statistics, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np
import torch
from tendermint_amd import _native as N, host as H, chains
from tendermint_amd.testing import factory as Fa

ap = argparse.ArgumentParser()
ap.add_argument("--headers", type=int, default=10_000)
ap.add_argument("--blocks", type=int, default=10_000)
ap.add_argument("--c5", type=int, default=1_000_000)
ap.add_argument("--only", default="1,3,4,5")
ap.add_argument("--c5-methods", default="", help="comma list of C5 method labels (default: all)")
ap.add_argument("--native-only", action="store_true", help="C3 / C4: only the C-ABI loop (no Python driver pass)")
a = ap.parse_args()
only = set(a.only.split(","))
ctx = N.Context(1)

if "1" in only:
    vals, bid, commit = Fa.make_c1_commit(150)
    call = H.PreparedCommitCall(ctx, H.MODE_FULL, "test_chain_id", vals, bid, 3, commit)
    t = time.perf_counter(); assert call() is None; cold = (time.perf_counter() - t) * 1e3
    lat = []
    for _ in range(500):
        t = time.perf_counter(); assert call() is None; lat.append((time.perf_counter() - t) * 1e3)
    lat.sort()
    print(json.dumps({"config": "C1 VerifyCommit 150 vals", "cold_ms": round(cold, 3),
                      "p50_ms": round(lat[250], 4), "p99_ms": round(lat[494], 4)}), flush=True)

if "3" in only:
    trusted, blocks = Fa.make_light_chain(a.headers, 100)
    period, now = 10**15, (blocks[-1].signed_header.header.time[0] + 1, 0)
    chains.verify_sequential(ctx, trusted, blocks[:50], period, now)  # warm
    n, dt = len(blocks), float("nan")
    if not a.native_only:
        t = time.perf_counter()
        n, err = chains.verify_sequential(ctx, trusted, blocks, period, now, window=1000)
        dt = time.perf_counter() - t
        assert err is None, err
    # the native part alone: C structs prepared outside the timed region
    pj = []
    for lo in range(0, len(blocks), 1000):
        prev = [trusted] + blocks[lo:lo + 999] if lo == 0 else blocks[lo - 1:lo + 999]
        pj.append(H.PreparedLightJobs([H.LightJob(p.signed_header, None, lb.signed_header, lb.vals, period, now,
                                                  mode=H.LIGHT_ADJACENT)
                                       for p, lb in zip(prev, blocks[lo:lo + 1000])]))
    L = H._setup_light(H._setup(N.lib()))
    t = time.perf_counter()
    for p in pj:
        res = H.run_light_jobs(L.tmv_light_verify_many, ctx.handle, p)
        assert all(k == 0 for k, _ in res)
    dn = time.perf_counter() - t
    line = {"config": f"C3 light sequential {a.headers} headers x 100 vals",
            "native_seconds": round(dn, 4), "native_headers_per_s": round(n / dn, 1)}
    # windows pipelined on caller threads (chains.in_order, the drivers' default depth 2)
    for depth in (2, 3):
        t = time.perf_counter()
        for res in chains.in_order(iter(pj), lambda p: H.run_light_jobs(L.tmv_light_verify_many, ctx.handle, p),
                                   depth):
            assert all(k == 0 for k, _ in res)
        line[f"native_depth{depth}_headers_per_s"] = round(n / (time.perf_counter() - t), 1)
    if not a.native_only:
        line.update({"seconds": round(dt, 4), "headers_per_s": round(n / dt, 1),
                     "verifies_per_s_ref_count": round(67 * n / dt)})
    print(json.dumps(line), flush=True)

if "4" in only:
    vals, blocks = Fa.make_block_chain(a.blocks, 175)
    chains.blocksync_replay(ctx, "test_chain_id", vals, blocks[:20], H.BlockID())  # warm (key table)
    applied, dt = len(blocks) - 2, float("nan")
    if not a.native_only:
        t = time.perf_counter()
        applied, err = chains.blocksync_replay(ctx, "test_chain_id", vals, blocks, H.BlockID(), window=600)
        dt = time.perf_counter() - t
        assert err is None, err
    jobs = []
    for i in range(1, len(blocks) - 1):
        f, s2 = blocks[i], blocks[i + 1]
        jobs.append(H.CommitJob(H.MODE_LIGHT, "test_chain_id", vals, f.block_id, f.height, s2.last_commit))
        jobs.append(H.CommitJob(H.MODE_FULL, "test_chain_id", vals, blocks[i - 1].block_id, f.height - 1,
                                f.last_commit))
    pj = [H.PreparedJobs(jobs[lo:lo + 1200]) for lo in range(0, len(jobs), 1200)]
    t = time.perf_counter()
    for p in pj:
        H.run_prepared_jobs(ctx, p)
    dn = time.perf_counter() - t
    line = {"config": f"C4 blocksync {a.blocks} blocks x 175 vals",
            "native_seconds": round(dn, 4), "native_blocks_per_s": round((len(blocks) - 2) / dn, 1)}
    for depth in (2, 3):
        t = time.perf_counter()
        for rc in chains.in_order(iter(pj), lambda p: H.run_prepared_jobs(ctx, p), depth):
            assert rc == 0
        line[f"native_depth{depth}_blocks_per_s"] = round((len(blocks) - 2) / (time.perf_counter() - t), 1)
    assert all(e is None for p in pj for e in p.decode())
    if not a.native_only:
        line.update({"seconds": round(dt, 4), "blocks_per_s": round(applied / dt, 1),
                     "verifies_per_s_ref_count": round(292 * applied / dt),
                     "unique_verifies_per_s": round(175 * applied / dt)})
    print(json.dumps(line), flush=True)

if "5" in only:
    # C5: 1M mixed ed25519 + sr25519 (20k distinct entries tiled; ~1% of each
    # kind corrupted as in make_mixed_batch), device-resident, per method
    kind, base = Fa.make_mixed_batch(20_000)
    reps = (a.c5 + base.n - 1) // base.n
    b = base.tile(a.c5)
    kind = np.tile(kind, reps)[:a.c5]
    dev = torch.device("cuda:0")
    t = lambda x: torch.from_numpy(x).to(dev)
    dk, dp, ds, dm = t(kind), t(b.pk), t(b.sig), t(b.msg)
    do = t(b.off.view(np.int32))
    st = torch.cuda.Stream()
    ref = None
    # "batch default": the runtime's own group sizes (ed25519 half 128 with the
    # located fallback, sr25519 half 64); "batch m=..": both halves forced
    c5_methods = [("per-entry", N.TMV_FLAG_PER_ENTRY, 0), ("batch default", N.TMV_FLAG_BATCH_EQUATION, 0),
                  ("batch m=32", N.TMV_FLAG_BATCH_EQUATION, 5),
                  ("batch m=64", N.TMV_FLAG_BATCH_EQUATION, 6), ("batch m=128", N.TMV_FLAG_BATCH_EQUATION, 7),
                  ("batch m=256", N.TMV_FLAG_BATCH_EQUATION, 8)]
    if a.c5_methods:
        c5_methods = [m for m in c5_methods if m[0] in a.c5_methods.split(",")]
    for label, flags, mlog in c5_methods:
        ctx.set_batch_options(group_log2=mlog)
        dst = torch.zeros(a.c5, dtype=torch.int8, device=dev)
        run = lambda: ctx.verify_batch_device_ex(0, N.TMV_KIND_MIXED, flags, dk.data_ptr(), dp.data_ptr(),
                                                 ds.data_ptr(), dm.data_ptr(), do.data_ptr(), a.c5, dst.data_ptr(),
                                                 st.cuda_stream)
        for _ in range(2):
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(3):
            run()
        e1.record(st); torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 3
        host = dst.cpu().numpy()
        if ref is None:
            ref = host
        print(json.dumps({"config": f"C5 mixed ed25519+sr25519 {a.c5} sigs, 1 GPU, kernel path, {label}",
                          "ms": round(ms, 3), "verifies_per_s": round(a.c5 / ms * 1e3),
                          "valid": int((host == 1).sum()), "same_vector": bool(np.array_equal(host, ref))}),
              flush=True)
