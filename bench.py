#!/usr/bin/env python3
"""Benchmark: ed25519 ZIP-215 verification on MI355X (BASELINE.json metric).

  python bench.py --gpus N --steps K --warmup W

A *step* = one pass of the hot path over one synthetic C2 batch
(BASELINE.json configs[1]: 10,000 ed25519 signatures over commit-vote
sign-bytes, 1% corrupted / ZIP-215 edge cases) already resident in HBM,
producing that batch's exact validity vector.  Each rank holds K distinct
C2 batches; one launch (tmv_verify_batches_device) verifies K of them at once
(`--per-launch K`, default 32): the batches are gathered on the device, run
through one pipeline and each gets its own vector, as a node draining a
queue of batches does (a single 10k batch fills about one wave per SIMD and
is latency-bound).  `--inflight F` keeps F launches in flight
on F streams (default 4, the HIP hardware queues per process).  `--method batch` (default) uses the random-linear-combination
group check with per-entry fallback (voi's BatchVerifier.Verify, SURVEY rows
G-I); `--method per-entry` verifies every signature singly.  With N > 1 (one
process per GPU, torchrun) every rank verifies its own batches (weak
scaling) and the packed validity bitmaps are all-gathered over RCCL on one
communication stream, the only cross-GPU exchange the path has.

Printed (rank 0, one JSON line): value = verifies/s of the whole job
(kernel path, inputs resident), the single-batch latency and serial rate,
end-to-end (host buffers, PCIe included), p50/p99 of a 150-validator commit
through the host C-ABI, the roofline object and a CPU baseline (the C
oracle "port" on the host's cores; the Go reference cannot be built here).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time
from concurrent.futures import ProcessPoolExecutor

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from tendermint_amd import _native as N  # noqa: E402
from tendermint_amd.shard import all_gather_validity  # noqa: E402
from tendermint_amd import host as H  # noqa: E402
from tendermint_amd.testing.factory import Batch, make_c1_commit, make_c2_batch  # noqa: E402

METRIC = "ed25519 verifies/sec at 1/2/4/8 GPUs + p50 VerifyCommit latency, 150 vals"
# Canonical algorithmic work per verified signature:
# 2,700 field multiplications x 100 32x32->64 partial products.
MULS_PER_SIG = 2.7e5
# Peak 32x32->64 multiply-add rate of one MI355X, measured by
# tools/occbench.hip (v_mad_i64_i32, 16 waves/SIMD): profiles/occbench_r01.json.
PEAK_MUL_PER_S = 1.9686e13


def _load_peak() -> float:
    """Highest measured v_mad_i64_i32 rate: tools/mulbench.hip
    (profiles/mulbench_r01.json) and tools/occbench.hip at 16 waves/SIMD
    (profiles/occbench_r01.json)."""
    best = 0.0
    try:
        with open(os.path.join(REPO, "profiles", "mulbench_r01.json")) as f:
            best = max(best, float(json.load(f)["mad_i64_i32_per_s"]))
    except Exception:
        pass
    try:
        with open(os.path.join(REPO, "profiles", "occbench_r01.json")) as f:
            best = max([best] + [float(r["mad_per_s"]) for r in json.load(f)["rows"]])
    except Exception:
        pass
    return best or PEAK_MUL_PER_S


def _load_pmc(method: str):
    """PMC summary of a launch of 32 C2 batches from the committed passes
    (tools/profile_round.sh + tools/pmc_summary.py: FETCH_SIZE x2 gfx950
    correction + WRITE_SIZE; tools/pmc_derived.py: occupancy, VALU issue)."""
    path = (os.path.join(REPO, "profiles", "r01_close", "pmc_batch.json") if method == "batch"
            else os.path.join(REPO, "profiles", "r01_msm", "pmc_per_entry.json"))
    try:
        with open(path) as f:
            return json.load(f)
    except Exception:
        return {}


def _load_traffic(method: str):
    return _load_pmc(method).get("hbm_bytes_per_launch")


def _pmc_kernels(method: str):
    """Per-kernel occupancy (mean waves / SIMD) and VALU issue utilisation."""
    out = {}
    for name, k in _load_pmc(method).get("kernels", {}).items():
        d = k.get("derived")
        if d:
            out[name.replace("tmv::", "")] = {"occupancy": d["occupancy_waves_per_simd"],
                                              "valu_issue_util": d["valu_issue_util"]}
    return out or None


def cpu_baseline(batch, seconds_target: float = 12.0):
    """Oracle C port on the host cores, bounded sample (rank 0, N=1 only)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle_c  # noqa: E402  (test infrastructure; checker/baseline only)
    threads = int(os.environ.get("TMV_CPU_THREADS", min(16, os.cpu_count() or 1)))
    # calibrate on 1,000 sigs, then size the sample to ~seconds_target of CPU time
    sub = batch.off[:1001]
    t0 = time.perf_counter()
    oracle_c.ed25519_verify_packed(batch.pk[:32000], batch.sig[:64000], batch.msg, sub, threads=1)
    per_sig_cpu = (time.perf_counter() - t0) / 1000
    reps = max(1, int(seconds_target / (per_sig_cpu * batch.n)))
    t0 = time.perf_counter()
    for _ in range(reps):
        oracle_c.ed25519_verify_packed(batch.pk, batch.sig, batch.msg, batch.off, threads=threads)
    wall = time.perf_counter() - t0
    out = {"value": round(reps * batch.n / wall, 1), "unit": "verifies/s", "cores": threads, "kind": "port",
           "sample": f"C2 batch ({batch.n} sigs) x {reps} passes, oracle/c/ed25519_oracle.c, "
                     f"{threads} pthreads; Go/curve25519-voi not buildable here (no toolchain)"}
    out["openssl_proxy"] = _openssl_proxy(threads)
    return out


def _openssl_proxy(threads: int, seconds_target: float = 5.0):
    """SURVEY 8(d)'s strict-semantics CPU proxy when voi cannot run: OpenSSL 3
    Ed25519 single-verify/s on the same host threads, honest signatures only
    (RFC 8032 cofactorless verification disagrees with ZIP-215 on edge cases)."""
    import ctypes
    path = os.path.join(REPO, "oracle", "_build", "libopenssl_proxy.so")
    if not os.path.exists(path):
        return None
    L = ctypes.CDLL(path)
    honest = make_c1_commit_batch()  # 2,000 validators, one signature each
    b = honest.tile(20000)
    keys = honest.pk.copy()
    key_idx = (np.arange(b.n) % honest.n).astype(np.uint32)
    u8 = ctypes.POINTER(ctypes.c_uint8)
    u32 = ctypes.POINTER(ctypes.c_uint32)
    out = np.zeros(b.n, np.uint8)
    args = lambda: (b.pk.ctypes.data_as(u8), b.sig.ctypes.data_as(u8), b.msg.ctypes.data_as(u8),  # noqa: E731
                    b.off.ctypes.data_as(u32), b.n, out.ctypes.data_as(u8), threads, keys.ctypes.data_as(u8),
                    key_idx.ctypes.data_as(u32), honest.n)
    t0 = time.perf_counter()
    assert L.openssl_ed25519_verify_batch(*args()) == 1
    first = time.perf_counter() - t0
    reps = max(1, int(seconds_target / max(first, 1e-3)))
    t0 = time.perf_counter()
    for _ in range(reps):
        L.openssl_ed25519_verify_batch(*args())
    wall = time.perf_counter() - t0
    return {"value": round(reps * b.n / wall, 1), "unit": "verifies/s", "cores": threads,
            "kind": "openssl-proxy", "sample": f"{b.n} honest commit-vote sigs x {reps} passes (2,000 keys decoded "
                                               "once), OpenSSL 3 EVP Ed25519 verify (strict RFC 8032; not ZIP-215, "
                                               "not batched)"}


def make_c1_commit_batch():
    from tendermint_amd.testing.factory import make_commit_batch
    return make_commit_batch(2000)


def _c2(a):
    return make_c2_batch(a[0], seed=a[1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1536)
    ap.add_argument("--warmup", type=int, default=16)
    ap.add_argument("--batch", type=int, default=10_000)
    ap.add_argument("--per-launch", type=int, default=32,
                    help="independent batches per pipeline launch (tmv_verify_batches_device)")
    ap.add_argument("--inflight", type=int, default=4, help="launches in flight (streams)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--method", choices=["batch", "per-entry"], default="batch",
                    help="batch: random-linear-combination group check + per-entry fallback "
                         "(voi's BatchVerifier.Verify); per-entry: every signature verified singly")
    ap.add_argument("--group-log2", type=int, default=0)
    ap.add_argument("--window", type=int, default=0)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    K = max(1, min(64, args.per_launch))
    F = max(1, args.inflight)
    # K distinct C2 batches per rank (own keys / messages), generated on the
    # host before this process touches the GPU (worker processes are forked)
    with ProcessPoolExecutor(min(8, K)) as ex:
        batches = list(ex.map(_c2, [(args.batch, 0xED25519 + 1000 * rank + j) for j in range(K)]))
    if world > 1:
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)

    ctx = N.Context(1 << local_rank)
    ctx.set_batch_options(group_log2=args.group_log2, window_bits=args.window)
    flags = N.TMV_FLAG_BATCH_EQUATION if args.method == "batch" else N.TMV_FLAG_PER_ENTRY
    batch = batches[0]
    n = batch.n
    d_in = []
    for b in batches:
        d_in.append((torch.from_numpy(b.pk).to(dev), torch.from_numpy(b.sig).to(dev), torch.from_numpy(b.msg).to(dev),
                     torch.from_numpy(b.off.view(np.int32)).to(dev), int(b.off[-1] - b.off[0])))
    # one contiguous status vector per in-flight launch; batch j is a slice
    d_valid = [torch.zeros(K * n, dtype=torch.int8, device=dev) for _ in range(F)]
    refs = [[N.BatchRef(pk.data_ptr(), sig.data_ptr(), msg.data_ptr(), off.data_ptr(), n, mb,
                        d_valid[f][j * n:(j + 1) * n].data_ptr()) for j, (pk, sig, msg, off, mb) in enumerate(d_in)]
            for f in range(F)]
    streams = [torch.cuda.Stream(dev) for _ in range(F)]
    comm = torch.cuda.Stream(dev) if world > 1 else None

    def launch(i, kk=K, ev_pair=None):
        f = i % F
        st = streams[f]
        if ev_pair is not None:
            ev_pair[0].record(st)
        ctx.verify_batches_device(local_rank, N.TMV_KIND_ED25519, flags, refs[f][:kk], st.cuda_stream)
        if ev_pair is not None:
            ev_pair[1].record(st)
        if world > 1:
            # one collective per launch (the K vectors are contiguous), in
            # issue order on one stream, after this launch
            comm.wait_stream(st)
            with torch.cuda.stream(comm):
                all_gather_validity(d_valid[f][:kk * n], [kk * n] * world)
            st.wait_stream(comm)

    # single-batch latency (one batch per launch, one at a time), untimed for value
    lat_ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
    for _ in range(2):
        launch(0, 1)
    torch.cuda.synchronize(dev)
    for i in range(10):
        launch(0, 1, lat_ev[i])
        torch.cuda.synchronize(dev)
    batch_ms = statistics.median(a.elapsed_time(b) for a, b in lat_ev)

    launches = max(1, (args.steps + K - 1) // K)
    steps = launches * K
    # every stream's workspace is allocated by its first launch: warm all of them
    for i in range(max(2 * F, args.warmup // K)):
        launch(i)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(launches)]
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(launches):
        launch(i, K, evs[i])
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    launch_ms = statistics.mean(a.elapsed_time(b) for a, b in evs)
    valid = [int((d_valid[f][j * n:(j + 1) * n] == 1).sum().item()) for f in range(min(F, launches)) for j in range(K)]
    assert all(v == 9950 for v in valid), valid  # C2: 100 edge cases, 50 of them valid (factory.py)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    result = None
    if rank == 0:
        total = n * world * steps
        value = total / elapsed
        gpu_rate = n * steps / elapsed
        # end-to-end through the host C-ABI (pinned staging, H2D, kernels,
        # D2H): the K batches of one launch as one host-resident batch
        hb = Batch.concat(batches)
        e2e = []
        for _ in range(5):
            t1 = time.perf_counter()
            ctx.verify_batch_ex(N.TMV_KIND_ED25519, flags, hb.pk, hb.sig, hb.msg, hb.off)
            e2e.append(time.perf_counter() - t1)
        e2e_rate = hb.n / statistics.median(e2e)
        # p50 / p99 of types.VerifyCommit on a 150-validator commit (C1): the
        # C++ L3 path (sign-bytes, tally, batch verifier, error mapping) +
        # H2D + GPU kernels + D2H, through tmv_verify_commit.
        vals, bid, commit = make_c1_commit(150)
        call = H.PreparedCommitCall(ctx, H.MODE_FULL, "test_chain_id", vals, bid, 3, commit)
        assert call() is None
        lat = []
        for _ in range(200):
            t1 = time.perf_counter()
            err = call()
            lat.append((time.perf_counter() - t1) * 1e3)
            assert err is None
        lat.sort()
        peak = _load_peak()
        # canonical work per launch of K batches / its average
        # duration (HIP events on the launch stream)
        achieved = n * K * MULS_PER_SIG / (launch_ms * 1e-3)
        result = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "verifies/s",
            "n_gpus": world,
            "steps": steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic (deterministic C2 generator, OpenSSL-signed commit-vote sign-bytes)",
            "config": {"workload": "C2: 10k ed25519 ZIP-215 batch, 1% corrupted/edge-case sigs (BASELINE configs[1])",
                       "batch_per_step": n, "batches_per_launch": K, "launches_in_flight": F,
                       "method": args.method, "msg_bytes_avg": round(float(batch.msg.size) / n, 1),
                       "parallelism": f"shard{world}" if world > 1 else "single"},
            "valid_per_batch": valid[0],
            "batch_latency_ms": round(batch_ms, 4),
            "serial_verifies_per_s": round(n / (batch_ms * 1e-3), 1),
            "end_to_end_verifies_per_s": round(e2e_rate, 1),
            "end_to_end_note": f"{hb.n} host-resident signatures per call (pinned staging + PCIe + kernels + D2H)",
            "verify_commit_150_p50_ms": round(lat[len(lat) // 2], 4),
            "verify_commit_150_p99_ms": round(lat[int(len(lat) * 0.99) - 1], 4),
            "verify_commit_note": "types.VerifyCommit (C1: 150 validators) via tmv_verify_commit, host-resident commit",
            "roofline": {"bound": "valu-int-mul", "achieved": round(achieved / 1e12, 4),
                         "peak": round(peak / 1e12, 4), "unit": "Tmul/s", "frac": round(achieved / peak, 4),
                         "traffic": _load_traffic(args.method) if K == 32 else None,
                         "traffic_note": "HBM bytes per launch (PMC, profiles/r01_close/pmc_batch.json); algorithmic "
                                         "input bytes per launch = 32 x 10k x ~222 B = 71 MB",
                         "kernel": ("batch-equation pipeline k_prep..k_verify_quad" if args.method == "batch"
                                    else "k_prep + k_verify_quad"),
                         "launch_avg_ms": round(launch_ms, 4),
                         "aggregate_achieved": round(gpu_rate * MULS_PER_SIG / 1e12, 4),
                         "aggregate_frac": round(gpu_rate * MULS_PER_SIG / peak, 4),
                         "aggregate_note": f"{F} launches overlap, so each launch's own duration (above) is longer "
                                           "than the timed span / launches; aggregate = verifies/s x 2.7e5",
                         "achieved_from": f"{K} x {n} sigs x 2.7e5 canonical products / average launch "
                                          "duration (HIP events on the launch stream)",
                         "work_per_sig": "2.7e5 int32 products (SURVEY 8(d), single-verify equivalent)",
                         "pmc_kernels": _pmc_kernels(args.method) if K == 32 else None,
                         "pmc_note": "each kernel alone under --pmc: occupancy = mean resident waves per SIMD, "
                                     "valu_issue_util = share of SIMD cycles issuing VALU (tools/pmc_derived.py)"},
        }
        if world == 1 and not args.no_cpu_baseline:
            result["cpu_baseline"] = cpu_baseline(batch)
        else:
            result["cpu_baseline"] = None
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return result


if __name__ == "__main__":
    main()
