#!/usr/bin/env python3
"""C3 / C4 native loops with the caller pipelining windows (development
tool; GPU box): `seq` = one window at a time (bench_configs.py), `thr2` =
two caller threads take alternate windows, so one window's host phases
(convert, plan, sign-bytes, hashing) run while the other's engine call holds
the device; results are checked in window order.  `whole` (C4) = every job
in one tmv_verify_commits call (sliced by the library, TMV_HOST_SLICE).

  python tools/c34_pipeline.py --only 3,4 --modes seq,thr2,seq,thr2
"""
import argparse, json, os, sys, time
from concurrent.futures import ThreadPoolExecutor
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from tendermint_amd import _native as N, host as H, chains
from tendermint_amd.testing import factory as Fa

ap = argparse.ArgumentParser()
ap.add_argument("--headers", type=int, default=10_000)
ap.add_argument("--blocks", type=int, default=10_000)
ap.add_argument("--only", default="3,4")
ap.add_argument("--modes", default="seq,thr2,seq,thr2")
ap.add_argument("--python", action="store_true", help="also the Python drivers at depth 1 / 2")
ap.add_argument("--c3-window", type=int, default=1000, help="headers per tmv_light_verify_many call")
ap.add_argument("--c4-window", type=int, default=600, help="blocks per tmv_verify_commits call")
a = ap.parse_args()
only = set(a.only.split(","))
ctx = N.Context(1)


def py_driver(label, call, unit_n, unit):
    """the Python drivers (chains.*) at depth 1 / 2, then the same after
    gc.freeze() (the chain's objects out of the collector's full passes)"""
    import gc
    for frozen in (False, True):
        if frozen:
            gc.collect()
            gc.freeze()
        for depth in (1, 2, 1, 2):
            t = time.perf_counter()
            n, err = call(depth)
            dt = time.perf_counter() - t
            assert err is None, err
            print(json.dumps({"config": label, "mode": f"python depth{depth}" + (" gc.freeze" if frozen else ""),
                              "seconds": round(dt, 4), unit: round(unit_n / dt, 1)}), flush=True)
    gc.unfreeze()


def timed(run, windows, mode):
    t = time.perf_counter()
    if mode == "seq":
        res = [run(w) for w in windows]
    else:
        with ThreadPoolExecutor(int(mode[3:])) as ex:
            res = list(ex.map(run, windows))
    return time.perf_counter() - t, res


if "3" in only:
    trusted, blocks = Fa.make_light_chain(a.headers, 100)
    period, now = 10**15, (blocks[-1].signed_header.header.time[0] + 1, 0)
    chains.verify_sequential(ctx, trusted, blocks[:50], period, now)  # warm
    pj = []
    W3 = a.c3_window
    for lo in range(0, len(blocks), W3):
        prev = [trusted] + blocks[lo:lo + W3 - 1] if lo == 0 else blocks[lo - 1:lo + W3 - 1]
        pj.append(H.PreparedLightJobs([H.LightJob(p.signed_header, None, lb.signed_header, lb.vals, period, now,
                                                  mode=H.LIGHT_ADJACENT)
                                       for p, lb in zip(prev, blocks[lo:lo + W3])]))
    if a.python:
        py_driver("C3 python driver, windows of 1000",
                  lambda d: chains.verify_sequential(ctx, trusted, blocks, period, now, window=1000, depth=d),
                  len(blocks), "headers_per_s")
    L = H._setup_light(H._setup(N.lib()))
    run = lambda p: H.run_light_jobs(L.tmv_light_verify_many, ctx.handle, p)
    for mode in a.modes.split(","):
        if mode == "whole":
            continue
        dt, res = timed(run, pj, mode)
        assert all(k == 0 for r in res for k, _ in r)
        print(json.dumps({"config": f"C3 {len(blocks)} headers x 100 vals, windows of {W3}", "mode": mode,
                          "seconds": round(dt, 4), "headers_per_s": round(len(blocks) / dt, 1)}), flush=True)

if "4" in only:
    vals, blocks = Fa.make_block_chain(a.blocks, 175)
    chains.blocksync_replay(ctx, "test_chain_id", vals, blocks[:20], H.BlockID())  # warm (key table)
    if a.python:
        py_driver("C4 python driver, windows of 600 blocks",
                  lambda d: chains.blocksync_replay(ctx, "test_chain_id", vals, blocks, H.BlockID(), window=600,
                                                    depth=d),
                  len(blocks) - 2, "blocks_per_s")
    jobs = []
    for i in range(1, len(blocks) - 1):
        f, s2 = blocks[i], blocks[i + 1]
        jobs.append(H.CommitJob(H.MODE_LIGHT, "test_chain_id", vals, f.block_id, f.height, s2.last_commit))
        jobs.append(H.CommitJob(H.MODE_FULL, "test_chain_id", vals, blocks[i - 1].block_id, f.height - 1,
                                f.last_commit))
    W4 = 2 * a.c4_window
    pj = [H.PreparedJobs(jobs[lo:lo + W4]) for lo in range(0, len(jobs), W4)]
    whole = H.PreparedJobs(jobs)
    for mode in a.modes.split(","):
        if mode == "whole":
            dt, res = timed(lambda p: H.run_prepared_jobs(ctx, p), [whole], "seq")
            wins = [whole]
        else:
            dt, res = timed(lambda p: H.run_prepared_jobs(ctx, p), pj, mode)
            wins = pj
        assert all(e is None for p in wins for e in p.decode())
        print(json.dumps({"config": f"C4 {a.blocks} blocks x 175 vals, windows of {a.c4_window} blocks", "mode": mode,
                          "seconds": round(dt, 4), "blocks_per_s": round((len(blocks) - 2) / dt, 1)}), flush=True)
