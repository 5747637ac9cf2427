#!/usr/bin/env python3
"""Benchmark: ed25519 ZIP-215 verification on MI355X (BASELINE.json metric).

  python bench.py --gpus N --steps K --warmup W

A *step* = one device launch (tmv_verify_batches_device) that verifies
`--batches-per-step` (default 256, TMV_MAX_BATCHES) synthetic C2 batches (BASELINE.json
configs[1]: 10,000 ed25519 signatures over commit-vote sign-bytes, 1%
corrupted / ZIP-215 edge cases each) already resident in HBM, producing every
batch's exact validity vector: the batches are gathered on the device, run
through one pipeline and each gets its own vector, as a node draining a queue
of batches does.  A single 10k batch fills about one wave per SIMD and ends
in two latency chains (Horner, per-entry fallback), so its
latency is reported beside the throughput (`batch_latency_ms`), not as it.
`--steps K` times exactly K such launches; `--inflight F` keeps F launches in
flight on F streams (default 4, the HIP hardware queues per process), so
the driver's `--steps 20` already measures the steady state.  `--method batch`
(default) uses the random-linear-combination group check with per-entry
fallback (voi's BatchVerifier.Verify); `--method per-entry`
verifies every signature singly.  With N > 1 (one process per GPU, torchrun)
every rank verifies its own batches (weak scaling) and the packed validity
bitmaps are all-gathered over RCCL on one communication stream, the only
cross-GPU exchange the path has.

Printed (rank 0, one JSON line): value = verifies/s of the whole job
(kernel path, inputs resident), the single-batch latency and serial rate,
end-to-end (host buffers, PCIe included), p50/p99 of a 150-validator commit
through the host C-ABI, the roofline object and a CPU baseline (the C
oracle "port" on the host's cores; the Go reference cannot be built here).
"""
from __future__ import annotations

import argparse
import contextlib
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
from tendermint_amd.shard import all_gather_statuses, all_gather_validity, shard_range  # noqa: E402
from tendermint_amd import host as H  # noqa: E402
from tendermint_amd.testing.factory import (Batch, C2_VALID_KINDS, c2_kinds, make_c1_commit, make_c2_batch,  # noqa: E402
                                             make_mixed_batch)

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


PMC_DIRS = ("r06", "r05", "r04", "r03", "r02_final", "r02_close", "r02", "r01_close")  # newest first


def _load_pmc(method: str, batches_per_step: int = 32):
    """PMC summary of the batch-equation (or per-entry) pipeline from the
    newest committed passes (tools/profile_round.sh + tools/pmc_summary.py:
    FETCH_SIZE x2 gfx950 correction + WRITE_SIZE; tools/pmc_derived.py:
    occupancy, VALU issue), normalised to one step (one launch of
    `batches_per_step` 10k C2 batches)."""
    name = "pmc_batch.json" if method == "batch" else "pmc_per_entry.json"
    for d in PMC_DIRS + ("r01_msm",):
        path = os.path.join(REPO, "profiles", d, name)
        if not os.path.exists(path):
            continue
        with open(path) as f:
            pmc = json.load(f)
        per_launch = pmc.get("batches_per_launch", 32)
        out = dict(pmc)
        if "hbm_bytes_per_launch" in pmc:
            out["hbm_bytes_per_step"] = int(pmc["hbm_bytes_per_launch"] * batches_per_step / per_launch)
            fac = pmc.get("fetch_factors")
            how = (f"FETCH_SIZE x calibrated factors {fac} (tools/fetchbench.hip)" if fac
                   else "FETCH_SIZE x2 gfx950 correction")
            out["note"] = (f"HBM bytes per step ({batches_per_step} x 10k signatures) from PMC (profiles/{d}/{name}: "
                           f"{how} + WRITE_SIZE, launches of {per_launch} batches); "
                           f"algorithmic input bytes per step = {batches_per_step} x 10k x ~222 B")
        out["source"] = f"profiles/{d}/{name}"
        return out
    return {}


def _pmc_kernels(method: str):
    """Per-kernel occupancy (mean waves / SIMD) and VALU issue utilisation."""
    out = {}
    for name, k in _load_pmc(method).get("kernels", {}).items():
        d = k.get("derived")
        if d:
            out[name.replace("tmv::", "")] = {"occupancy": d["occupancy_waves_per_simd"],
                                              "valu_issue_util": d["valu_issue_util"]}
    return out or None


TIMED_KERNELS = ("k_msm_accum", "k_msm_wpart", "k_prep_fused")
# k_msm_accum's algorithmic work: one mixed (Niels) addition per bucket entry,
# 7 field multiplications (ge_madd 3 + p1p1->p3 4) x 100 int32 products.
ACCUM_PRODUCTS_PER_ENTRY = 7 * 100


def accum_entries_per_sig(m: int = 64, c: int = 5, samples: int = 4000, seed: int = 1) -> float:
    """Expected bucket entries per signature of the batch equation (msm.h):
    the nonzero signed c-bit digits of a uniform 128-bit weight z (R term, 129
    bits of windows) and of a uniform scalar mod l (A term, 254 bits), plus
    the group's B scalar shared by m signatures -- simulated with the device's
    recoding (msm_kernels.hip window_digit)."""
    import random
    l_order = 2**252 + 27742317777372353535851937790883648493
    rng = random.Random(seed)

    def nonzero(x, windows):
        cnt, carry = 0, 0
        for w in range(windows):
            d = ((x >> (w * c)) & ((1 << c) - 1)) + carry
            if w + 1 < windows and d >= 1 << (c - 1):
                d -= 1 << c
                carry = 1
            else:
                carry = 0
            cnt += d != 0
        return cnt
    wr, w = -(-129 // c), -(-254 // c)
    tot = 0
    for _ in range(samples):
        tot += nonzero(rng.getrandbits(128), wr) + nonzero(rng.randrange(l_order), w)
    return tot / samples + nonzero(rng.randrange(l_order), w) / m


# Algorithmic int32 products of each pipeline kernel per launch (SURVEY 8(d)'s
# unit: a field multiplication = 100 32x32->64 products; a squaring needs 55).
FE_MUL, FE_SQ = 100, 55
# ge_decode_zip215 (255 squarings, 19 multiplications: y^2, d y^2, v^3, v^7,
# the (p-5)/8 power, the check, T) + the Niels / cached form of the point (1)
DECODE_PRODUCTS = 255 * FE_SQ + 20 * FE_MUL
BARRETT_PRODUCTS = 9 * 9 + 9 * 8  # sc_reduce512 (32x32 word products)
QDBL = 4 * FE_SQ + 4 * FE_MUL     # one point doubling (quad: a squaring + a multiply per lane)
QADD = 8 * FE_MUL                 # one point addition + conversion to extended
QCACHED = 4 * FE_MUL              # extended -> cached
QTABLE = QDBL + 6 * QADD + 8 * QCACHED  # (m+1) P, m < 8, cached
WPART_BUCKET = 17 * FE_MUL        # running sums per bucket: U += B (cached U: 9), T += U (8)


def kernel_products(n, m, c, fallback_entries=0, groups_failed=0, located=False, half_scalars=True):
    """Algorithmic products of each kernel of one batch-equation launch of n
    ed25519 entries (groups of m, c-bit windows): prep (two decodes + the
    Barrett reduction of the hash; SHA-512 has no products), bucket sums
    (one mixed addition per bucket entry), running sums (17 multiplications
    per bucket), Horner ((W-1) c + 3 doublings + W-1 additions per group), the
    per-entry fallback (half-size scalars: two 8-entry tables, 124 doublings,
    96 additions; full k: 252 doublings) and, located, the second MSM over
    the failing groups (the same bucket and running-sum work per group, the R
    weights a few bits longer)."""
    W, H = -(-254 // c), 1 << (c - 1)
    G = -(-n // m)
    e = accum_entries_per_sig(m=m, c=c)
    Gl = groups_failed if located else 0
    per_entry = 2 * QTABLE + QCACHED + ((124 + 3) * QDBL + 96 * QADD if half_scalars else (252 + 3) * QDBL + 96 * QADD)
    return {
        "k_prep_fused": n * (2 * DECODE_PRODUCTS + BARRETT_PRODUCTS),
        "k_msm_accum": (n + Gl * m) * e * 7 * FE_MUL,
        "k_msm_wpart": (G + Gl) * W * (H * WPART_BUCKET + FE_MUL),
        "k_msm_horner": G * (((W - 1) * c + 3) * QDBL + (W - 1) * QADD),
        "k_msm_horner_loc": Gl * (((W - 1) * c + 3) * QDBL + (W - 1) * QADD),  # the located pass's own Horner
        "fallback": fallback_entries * per_entry,
    }


def msm_shape(n_launch: int, group_log2: int = 0, window: int = 0, locate_min: int = 400_000):
    """The runtime's batch-equation shape for an uncached ed25519 launch of
    n_launch entries (tmverify_runtime.cpp msm_params): groups of 128 from
    the located-fallback size up, else 64; the window from the same cost
    model.  Returns (m, c)."""
    m_log2 = group_log2 or (7 if n_launch >= locate_min else 6)
    m = 1 << m_log2
    if window:
        return m, window
    best, c = None, 5
    for cc in range(4, 10):
        w, wr, h = -(-254 // cc), -(-129 // cc), 1 << (cc - 1)
        cost = m * (w + wr) + 3.0 * w * h  # tmverify_runtime.cpp kRunningSumWeight
        if best is None or cost < best:
            best, c = cost, cc
    return m, c


def host_cpu_info():
    """The cores this process may use (affinity and cgroup CPU quota), the
    machine's CPU count and model."""
    n = os.cpu_count() or 1
    try:
        n = min(n, len(os.sched_getaffinity(0)))
    except Exception:
        pass
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) // int(per)))
    except Exception:
        pass
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except Exception:
        pass
    usable = min(n, quota) if quota else n
    return {"usable_cores": usable, "machine_cpus": os.cpu_count(), "cgroup_quota_cores": quota, "model": model}


def cpu_baseline(batches, seconds_target: float = 4.0):
    """CPU baselines on all the host cores this process may use, bounded
    samples (rank 0, N=1 only); test infrastructure from oracle/ (never the
    measured path).

    value: the reference's own algorithm on this workload -- voi's
    BatchVerifier.Verify restated in C (oracle/c/ed25519_batch_cpu.c): one
    batch per C2 batch (verifyCommitBatch adds every signature, then
    Verify), one random linear combination, entry by entry when it fails
    (every C2 batch holds invalid signatures, so it always does).
    Also: the same verifier on honest signatures in batches of 1,024 (the
    CPU's best case), the per-entry C port, and OpenSSL single-verify."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle_c  # noqa: E402  (test infrastructure; checker/baseline only)
    info = host_cpu_info()
    threads = int(os.environ.get("TMV_CPU_THREADS", info["usable_cores"]))
    batch = batches[0]

    # voi semantics on C2: one BatchVerifier per 10k batch, `threads` batches at once
    hb = Batch.concat(batches[:max(1, min(len(batches), threads))])
    def voi():
        return oracle_c.ed25519_batch_verify_voi(hb.pk, hb.sig, hb.msg, hb.off, threads=threads, batch=batch.n)
    t0 = time.perf_counter()
    _, v, failed = voi()
    calib = time.perf_counter() - t0
    reps = max(1, int(seconds_target / max(calib, 1e-3)))
    t0 = time.perf_counter()
    for _ in range(reps):
        voi()
    wall = time.perf_counter() - t0
    out = {"value": round(reps * hb.n / wall, 1), "unit": "verifies/s", "cores": threads, "kind": "port",
           "host": info,
           "sample": f"{hb.n // batch.n} C2 batches ({batch.n} sigs each, one per thread) x {reps} passes through "
                     "oracle/c/ed25519_batch_cpu.c: curve25519-voi's BatchVerifier.Verify algorithm restated in "
                     f"plain C (radix 2^51), one batch per C2 batch -- {failed} of {hb.n // batch.n} batch equations "
                     f"failed (every C2 batch holds invalid signatures), then entry by entry, as voi; {threads} "
                     "pthreads = every core this process may use; Go/curve25519-voi not buildable here (no Go "
                     "toolchain, voi absent)"}
    # the CPU's best case: honest signatures, batches of 1,024
    honest = make_c1_commit_batch().tile(1024 * threads)
    t0 = time.perf_counter()
    oracle_c.ed25519_batch_verify_voi(honest.pk, honest.sig, honest.msg, honest.off, threads=threads, batch=1024)
    calib = time.perf_counter() - t0
    reps = max(1, int(seconds_target / max(calib, 1e-3)))
    t0 = time.perf_counter()
    for _ in range(reps):
        ok, _, f2 = oracle_c.ed25519_batch_verify_voi(honest.pk, honest.sig, honest.msg, honest.off,
                                                      threads=threads, batch=1024)
    wall = time.perf_counter() - t0
    out["all_valid_batch"] = {"value": round(reps * honest.n / wall, 1), "unit": "verifies/s", "cores": threads,
                              "sample": f"{honest.n} honest commit-vote sigs (2,000 keys) in batches of 1,024 x "
                                        f"{reps} passes, same C batch verifier ({f2} failed batches): the CPU's best "
                                        "case, not this workload"}
    # the per-entry C port (round-1 baseline)
    sub = batch.off[:1001]
    t0 = time.perf_counter()
    oracle_c.ed25519_verify_packed(batch.pk[:32000], batch.sig[:64000], batch.msg, sub, threads=1)
    per_sig_cpu = (time.perf_counter() - t0) / 1000
    reps = max(1, int(seconds_target * threads / (per_sig_cpu * batch.n)))
    t0 = time.perf_counter()
    for _ in range(reps):
        oracle_c.ed25519_verify_packed(batch.pk, batch.sig, batch.msg, batch.off, threads=threads)
    wall = time.perf_counter() - t0
    out["per_entry_port"] = {"value": round(reps * batch.n / wall, 1), "unit": "verifies/s", "cores": threads,
                             "sample": f"C2 batch x {reps} passes, oracle/c/ed25519_oracle.c per-entry verification"}
    out["openssl_proxy"] = _openssl_proxy(threads)
    out["verify_commit_150"] = _c1_cpu(oracle_c)
    return out


def mixed_oracle_statuses(kind, base) -> np.ndarray:
    """Checker only (never timed): the exact per-entry statuses of a mixed
    ed25519 + sr25519 batch from the C oracle (ed25519 1/0, sr25519 1/0/-1/-2),
    the known vector the strong mixed leg's gathered vector must equal."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle_c  # noqa: E402  (test infrastructure; checker role)
    threads = min(16, host_cpu_info()["usable_cores"])
    want = np.zeros(base.n, np.int8)
    ed, sr = np.flatnonzero(kind == 0), np.flatnonzero(kind == 1)
    if len(ed):
        be = base.take(ed)
        want[ed] = oracle_c.ed25519_verify_packed(be.pk, be.sig, be.msg, be.off, threads=threads)[1]
    if len(sr):
        bs = base.take(sr)
        want[sr] = oracle_c.sr25519_status_packed(bs.pk, bs.sig, bs.msg, bs.off, threads=threads)
    return want


def _c1_cpu(oracle_c, calls: int = 300):
    """BASELINE configs[0] on the CPU: types.VerifyCommit's signature work on
    the 150-validator C1 commit, one thread (the Go benchmark runs one
    goroutine, types/validator_set_test.go:1530-1556): every vote's
    sign-bytes, then one voi-style batch of 150 (oracle/c/ed25519_batch_cpu.c
    oracle_verify_commit_cpu).  p50 / p99 over `calls` calls."""
    from tendermint_amd.testing.bulk import commit_vote_head
    from tendermint_amd.types.canonical import BlockID, PartSetHeader
    vals, bid, commit = make_c1_commit(150)
    head = commit_vote_head(3, 0, BlockID(bid.hash, PartSetHeader(bid.psh_total, bid.psh_hash)))
    pk = np.frombuffer(b"".join(v.pub_key for v in vals.validators), np.uint8)
    sig = np.frombuffer(b"".join(cs.signature for cs in commit.signatures), np.uint8)
    call = oracle_c.CommitCPU(head, "test_chain_id", [cs.timestamp[0] for cs in commit.signatures],
                              [cs.timestamp[1] for cs in commit.signatures], pk, sig)
    assert call()
    lat = []
    for _ in range(calls):
        t1 = time.perf_counter()
        ok = call()
        lat.append((time.perf_counter() - t1) * 1e3)
        assert ok
    lat.sort()
    return {"p50_ms": round(lat[len(lat) // 2], 4), "p99_ms": round(lat[int(len(lat) * 0.99) - 1], 4),
            "calls": calls, "cores": 1, "kind": "port",
            "sample": "C1 commit (150 validators): 150 vote sign-bytes + one 150-entry voi-style batch verify, one "
                      "thread, oracle/c/ed25519_batch_cpu.c (plain-C restatement; NOT the reference: Go/voi are not "
                      "buildable here; voi's expanded-key cache not restated)"}


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


VALID_KINDS = C2_VALID_KINDS  # factory.make_c2_batch's valid entries


def _mixed(a):
    return make_mixed_batch(a[0], seed=a[1])


STRONG_SEED = 0xED25519  # batch j of the strong-scaling batch: make_c2_batch(n, STRONG_SEED + j), on every rank


class _HostStream:
    """--cpu-stub stand-in for torch.cuda.Stream (the control flow only)."""
    cuda_stream = 0

    def wait_stream(self, other):
        pass


class _HostEvent:
    def __init__(self, **_):
        self.t = None

    def record(self, stream=None):
        self.t = time.perf_counter()

    def elapsed_time(self, other):
        return (other.t - self.t) * 1e3


KFRACS_FILE = os.path.join("profiles", "r06", "kernel_fracs.json")


def _kernel_fracs():
    """Per-kernel fractions of single launches (tools/kernel_fracs.py over the
    committed kernel trace and PMC pass of tools/launch_alone.py --stats)."""
    try:
        with open(os.path.join(REPO, KFRACS_FILE)) as f:
            return json.load(f)
    except Exception:
        return {}


def _profile_build(d, build_digest):
    """(same_build, note) for a committed profile d: its executed counts
    describe this run's kernels only when it was taken on a library with
    this run's compiled source digest."""
    src = (d.get("source") or {}).get("src_digest") if isinstance(d.get("source"), dict) else d.get("src_digest")
    if src and build_digest and src == build_digest:
        return True, f"profile of this build (src={src})"
    return False, (f"ESTIMATE: the committed profile was taken on build src={src or 'unrecorded'}, this run's "
                   f"library is src={build_digest or 'unknown'}; the counts may not describe these kernels")


def _pipeline_roofline(gpu_rate, peak, pmc, launch_ms, method, n_launch=0, ms_per_step=0.0, build_digest=None):
    """The whole pipeline.  executed_mad_frac: the v_mad_i64_i32 lane-ops one
    launch of this size executes (PMC SQ_INSTS_VALU_INT64 per kernel x its
    static v_mad_i64_i32 share, tools/isa_mix.py; committed pass at this
    launch size) / this run's ms_per_step / the measured multiply peak -- a
    true fraction (each counted op is one issued multiply-add).  Also the
    per-kernel algorithmic fractions of single launches of this size and of
    the 125k shard (the 1/8 of the north_star's 1M batch), and
    canonical_ratio: verifies/s x SURVEY 8(d)'s 2.7e5 products per
    single-verify-equivalent signature / peak, which the batch equation
    exceeds (it does less work than single verifies): a ratio, never the
    roofline fraction."""
    out = {"canonical_ratio": round(gpu_rate * MULS_PER_SIG / peak, 4),
           "canonical_note": "verifies/s of this GPU x 2.7e5 canonical products per signature (SURVEY 8(d)) / peak: "
                             "the batch equation does less work than a single verify, so this ratio exceeds 1 and is "
                             "not a roofline fraction",
           "kernel": ("batch-equation pipeline k_prep..k_verify_quad" if method == "batch"
                      else "k_prep + k_verify_quad"),
           "launch_avg_ms": round(launch_ms, 4),
           "traffic_per_step": pmc.get("hbm_bytes_per_step"),
           "traffic_note": pmc.get("note"),
           "executed": pmc.get("executed"),
           "pmc_kernels": _pmc_kernels(method),
           "peak": round(peak / 1e12, 4), "unit": "Tmul/s"}
    kf = _kernel_fracs()
    by_n = {L["n"]: L for L in kf.get("launches", [])}
    if method == "batch" and n_launch in by_n:
        L = by_n[n_launch]
        mads = sum(k["int64_lane_ops"] * k["mad_share_static"] for k in L["kernels"].values()
                   if "int64_lane_ops" in k)
        if mads and ms_per_step:
            same, prov = _profile_build(kf, build_digest)
            key = "executed_mad_frac" if same else "executed_mad_frac_estimate"
            out[key] = round(mads / (ms_per_step * 1e-3) / peak, 4)
            out["executed_mad_note"] = (f"{mads:.4g} v_mad_i64_i32 lane-ops per launch of {n_launch} signatures (PMC "
                                        "SQ_INSTS_VALU_INT64 x 64 lanes x each kernel's static v_mad_i64_i32 share, "
                                        f"{KFRACS_FILE}) / this run's ms_per_step / peak; the same launch alone: "
                                        f"{L.get('pipeline_executed_mad_frac')}; {prov}")
    if kf:
        out["kernel_fracs"] = {
            str(L["n"]): {"launch_span_us": L["launch_span_us"], "verifies_per_s": L["verifies_per_s"],
                          "pipeline_algorithmic_frac": L["pipeline_algorithmic_frac"],
                          "pipeline_executed_mad_frac": L.get("pipeline_executed_mad_frac"),
                          "kernels": {k: {x: v[x] for x in ("us", "frac", "executed_mad_frac") if x in v}
                                      for k, v in L["kernels"].items()}}
            for L in kf.get("launches", [])}
        out["kernel_fracs_note"] = (f"single launches alone ({KFRACS_FILE}: rocprofv3 kernel trace + PMC of "
                                    "tools/launch_alone.py --stats): frac = the kernel's algorithmic products "
                                    "(bench.kernel_products: decodes, bucket entries, running sums, Horner, fallback "
                                    "entries of that launch) / its time / peak; executed_mad_frac = its executed "
                                    "v_mad_i64_i32 lane-ops / its time / peak")
    return out


DOMINANT_FILE = os.path.join("profiles", "r06", "dominant_kernel.json")


def _dominant_file():
    try:
        with open(os.path.join(REPO, DOMINANT_FILE)) as f:
            return json.load(f)
    except Exception:
        return {}


def _isa_mix():
    """Static instruction mix of k_msm_accum<16> (tools/isa_mix.py), newest
    committed profile first."""
    for d in ("r06", "r05"):
        path = os.path.join(REPO, "profiles", d, "isa_mix.json")
        if os.path.exists(path):
            with open(path) as f:
                m = json.load(f).get("kernels", {}).get("k_msm_accum<16>")
            if m and m.get("mad_share_of_int64"):
                m["source"] = f"profiles/{d}/isa_mix.json"
                return m
    for d in ("r04", "r03", "r02_close"):
        path = os.path.join(REPO, "profiles", d, "isa_mix_accum.json")
        if os.path.exists(path):
            with open(path) as f:
                m = json.load(f)
            if m.get("mad_share_of_int64"):
                m["source"] = f"profiles/{d}/isa_mix_accum.json"
                return m
    return None


def _dominant_roofline(ktimes, ktimes_alone, K, n, args, peak, steps, pipeline, ms_per_step, build_digest=None):
    """roofline for the dominant kernel, k_msm_accum<16> (bucket sums; the
    largest share of the pipeline's VALU work): its algorithmic products per
    launch (SURVEY 8(d)'s per-unit work: one mixed addition = 7 field
    multiplications x 100 int32 products per bucket entry, x the expected
    entries per signature x the launch's signatures) over its own launch
    duration -- the five launches run alone after the timed region, bracketed
    by HIP events on their stream (tmv_kernel_timing), so no other launch
    shares the chip -- against the measured v_mad_i64_i32 peak.  The
    committed rocprofv3 --kernel-trace --stats of bench.py --inflight 1 (one
    launch at a time) gives the same kernel's average dispatch
    (profiles/r06/dominant_kernel.json); traffic = its HBM bytes per launch
    from PMC passes at this launch size (256 x 10k)."""
    m_grp, c_win = msm_shape(K * n, args.group_log2, args.window)
    per_launch = K * n * accum_entries_per_sig(m=m_grp, c=c_win) * ACCUM_PRODUCTS_PER_ENTRY
    alone = ktimes_alone.get("k_msm_accum", (0, 0))
    ov_ms, ov_cnt = ktimes["k_msm_accum"]
    own_ms = alone[0] / alone[1] if alone[1] else None
    dfile = _dominant_file()
    rp = dfile.get("rocprof_alone")
    if own_ms is None and rp:  # --no-extras: the committed rocprof figure
        own_ms = rp["avg_ms"]
    achieved = per_launch / (own_ms * 1e-3) if own_ms else None
    r = {"bound": "valu-int-mul",
         "kernel": "k_msm_accum<16>",
         "achieved": round(achieved / 1e12, 4) if achieved else None,
         "peak": round(peak / 1e12, 4), "unit": "Tmul/s",
         "frac": round(achieved / peak, 4) if achieved else None,
         # PMC bytes of a launch of the profiled size; omitted at other sizes
         "traffic": dfile.get("traffic_bytes_per_launch") if K == dfile.get("batches_per_launch", 256) else None,
         "traffic_note": dfile.get("traffic_note"),
         "avg_launch_ms": round(own_ms, 4) if own_ms else None,
         "ms_per_step": round(ms_per_step, 4),
         "timing": "HIP events on the stream of each k_msm_accum launch, five launches of the bench's size run alone "
                   "after the timed region (tmv_kernel_timing); one per step, so its own time per step is "
                   "avg_launch_ms <= ms_per_step",
         "algorithmic_products_per_launch": round(per_launch),
         "msm_shape": {"group": m_grp, "window_bits": c_win},
         "algorithmic_note": f"{K} x {n} signatures x expected bucket entries per signature (nonzero signed "
                             f"{c_win}-bit digits of z and z k mod l, + the group's B scalar over {m_grp}; simulated "
                             "recoding) x 7 field multiplications x 100 int32 products (SURVEY 8(d) unit)",
         "peak_from": "measured v_mad_i64_i32 rate, 16 waves/SIMD (tools/occbench.hip, profiles/occbench_r01.json)",
         "rocprof": rp,
         "rocprof_inflight4": dfile.get("rocprof_inflight4"),
         "under_overlap": {"avg_launch_ms": round(ov_ms / ov_cnt, 4), "launches": ov_cnt,
                           "note": f"the timed region's launches ({args.inflight} in flight share the chip, so a "
                                   "launch's span is stretched; not the kernel's own time)"},
         "other_kernels_alone_ms": {k: round(v[0] / v[1], 4) for k, v in ktimes_alone.items()
                                    if v[1] and k != "k_msm_accum"},
         "pipeline": pipeline}
    ex = dfile.get("executed_int64_lane_ops_per_launch")
    prof_k = dfile.get("batches_per_launch", 256)
    mix = _isa_mix()
    if ex and own_ms and mix and K == prof_k:
        # only the v_mad_i64_i32 share of the 64-bit lane-ops is priced
        # against the v_mad_i64_i32 peak (the carry adds / shifts are other
        # instructions): PMC INT64 lane-ops x the kernel's static mad share
        mads = ex * mix["mad_share_of_int64"]
        same, prov = _profile_build(dfile, build_digest)
        r["executed_mad_frac" if same else "executed_mad_frac_estimate"] = round(mads / (own_ms * 1e-3) / peak, 4)
        r["executed_note"] = (f"PMC SQ_INSTS_VALU_INT64 lane-ops per launch (profiled at {prof_k} batches per launch) "
                              f"x the kernel's static v_mad_i64_i32 share of its 64-bit VALU instructions "
                              f"({mix['mad_share_of_int64']}, {mix['source']}) / own duration / peak "
                              f"v_mad_i64_i32 rate; {prov}")
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=48, help="timed steps (device launches of --batches-per-step "
                                                           "C2 batches)")
    ap.add_argument("--warmup", type=int, default=8, help="untimed steps before timing (at least --inflight)")
    ap.add_argument("--batch", type=int, default=10_000)
    ap.add_argument("--batches-per-step", "--per-launch", dest="per_step", type=int, default=256,
                    help="C2 batches per step (one tmv_verify_batches_device launch, <= 256)")
    ap.add_argument("--inflight", type=int, default=4, help="launches in flight (streams)")
    ap.add_argument("--resident", type=int, default=64,
                    help="distinct C2 batches held in HBM per rank (a step's batches cycle through them)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip latency / end-to-end / C1 measurements")
    ap.add_argument("--method", choices=["batch", "per-entry"], default="batch",
                    help="batch: random-linear-combination group check + per-entry fallback "
                         "(voi's BatchVerifier.Verify); per-entry: every signature verified singly")
    ap.add_argument("--group-log2", type=int, default=0)
    ap.add_argument("--window", type=int, default=0)
    ap.add_argument("--strong-n", type=int, default=1_000_000,
                    help="signatures of the strong-scaling batch split over the ranks (north_star: 1M; 0 = skip)")
    ap.add_argument("--strong-mixed", type=int, default=1,
                    help="also run the strong-scaling leg on the C5 mixed ed25519 + sr25519 batch")
    ap.add_argument("--strong-reps", type=int, default=5, help="timed repetitions of each strong-scaling leg")
    ap.add_argument("--cpu-stub", action="store_true",
                    help="CI only: run the launch / gather / timing control flow on the CPU (gloo) with a stub "
                         "engine that writes the known statuses; no GPU, no verification, not a measurement")
    args = ap.parse_args()
    stub = args.cpu_stub
    t_main = time.perf_counter()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    gpu = local_rank  # this rank's HIP device (one process per GPU)
    if not args.cpu_stub and torch.cuda.device_count() <= local_rank:
        gpu = 0  # the launcher exposed one device per process
    F = max(1, args.inflight)
    R = max(1, min(256, args.resident))
    K = max(1, min(256, args.per_step))
    sizes = [K] * max(1, args.steps)
    nb = args.batch
    # R distinct C2 batches per rank (own keys / messages), generated on the
    # host before this process touches the GPU (worker processes are forked).
    # The strong-scaling batch is the same on every rank: batch j of it is
    # make_c2_batch(nb, STRONG_SEED + j); a rank generates only the batches
    # its shard touches (rank 0's own batches carry the same seeds).
    own = [0xED25519 + 1000 * rank + j for j in range(R)]
    strong_n = 0 if args.no_extras else max(0, args.strong_n)
    s_lo, s_hi = shard_range(strong_n, world, rank)
    strong_js = list(range(s_lo // nb, (s_hi - 1) // nb + 1)) if s_hi > s_lo else []
    extra = [STRONG_SEED + j for j in strong_js if STRONG_SEED + j not in own]
    mixed_n = 2_000 if stub else 20_000
    with ProcessPoolExecutor(min(8, R + len(extra))) as ex:
        fut_mixed = ex.submit(_mixed, (mixed_n, 0xC5)) if strong_n and args.strong_mixed else None
        gen = dict(zip(own + extra, ex.map(_c2, [(nb, sd) for sd in own + extra])))
        mixed_base = fut_mixed.result() if fut_mixed else None
    batches = [gen[sd] for sd in own]
    strong_batches = [gen[STRONG_SEED + j] for j in strong_js]
    del gen
    if stub:
        if world > 1:
            dist.init_process_group("gloo")
        dev = torch.device("cpu")
        ctx = None
        sync = lambda d=None: None  # noqa: E731
        Stream, Event, stream_ctx = (lambda d: _HostStream()), _HostEvent, (lambda st: contextlib.nullcontext())
    else:
        if world > 1:
            torch.cuda.set_device(gpu)
            # RCCL; TMV_BENCH_BACKEND=gloo rehearses N ranks on a one-GPU box
            backend = os.environ.get("TMV_BENCH_BACKEND", "nccl")
            if backend == "nccl":
                dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
            else:
                dist.init_process_group(backend)
        dev = torch.device("cuda", gpu)
        torch.cuda.set_device(dev)
        ctx = N.Context(1 << gpu)
        ctx.set_batch_options(group_log2=args.group_log2, window_bits=args.window)
        sync = torch.cuda.synchronize
        Stream, Event, stream_ctx = torch.cuda.Stream, torch.cuda.Event, torch.cuda.stream
    flags = N.TMV_FLAG_BATCH_EQUATION if args.method == "batch" else N.TMV_FLAG_PER_ENTRY
    key_kind = N.TMV_KIND_ED25519
    # the exchange: packed bitmaps where statuses are 0 / 1 (ed25519); kinds
    # whose statuses carry deferred Add errors (sr25519: -1 / -2) gather the
    # int8 statuses themselves (shard.all_gather_statuses)
    gather_fn = all_gather_validity if key_kind == N.TMV_KIND_ED25519 else all_gather_statuses
    batch = batches[0]
    n = batch.n
    expect_valid = [sum(k in VALID_KINDS for k in b.kinds) for b in batches]
    d_in = []
    for b in batches:
        d_in.append((torch.from_numpy(b.pk).to(dev), torch.from_numpy(b.sig).to(dev), torch.from_numpy(b.msg).to(dev),
                     torch.from_numpy(b.off.view(np.int32)).to(dev), int(b.off[-1] - b.off[0])))
    # one contiguous status vector per stream; the j-th batch of a launch is a slice
    d_valid = [torch.zeros(K * n, dtype=torch.int8, device=dev) for _ in range(F)]

    def refs(f, first, kk):
        out = []
        for j in range(kk):
            pk, sig, msg, off, mb = d_in[(first + j) % R]
            out.append(N.BatchRef(pk.data_ptr(), sig.data_ptr(), msg.data_ptr(), off.data_ptr(), n, mb,
                                  d_valid[f][j * n:(j + 1) * n].data_ptr()))
        return out
    streams = [Stream(dev) for _ in range(F)]
    comm = Stream(dev) if world > 1 else None
    # every resident batch's known vector (factory kinds: 9,950 valid of 10k);
    # the timed launches' vectors are compared with it entry by entry
    want_status = [torch.tensor([1 if k in VALID_KINDS else 0 for k in b.kinds], dtype=torch.int8, device=dev)
                   for b in batches]
    if stub:  # the statuses the engine would write, per resident batch
        stub_status = want_status
    gathered = {}

    def launch(i, first, kk, ev_pair=None, gather=True):
        f = i % F
        st = streams[f]
        if ev_pair is not None:
            ev_pair[0].record(st)
        if stub:
            for j in range(kk):
                d_valid[f][j * n:(j + 1) * n] = stub_status[(first + j) % R]
        else:
            ctx.verify_batches_device(gpu, key_kind, flags, refs(f, first, kk), st.cuda_stream)
        if ev_pair is not None:
            ev_pair[1].record(st)
        if world > 1 and gather:
            # one collective per launch (its kk vectors are contiguous), in
            # issue order on one stream, after this launch
            comm.wait_stream(st)
            with stream_ctx(comm):
                gathered[f] = gather_fn(d_valid[f][:kk * n], [kk * n] * world)
            st.wait_stream(comm)

    def run(sizes_, evs=None):
        first = 0
        for i, kk in enumerate(sizes_):
            launch(i, first, kk, evs[i] if evs else None)
            first += kk
        return first

    # warmup: every stream's workspace is allocated by its first launch, at
    # the largest launch size of the timed region
    run([K] * max(args.warmup, F))
    sync(dev)
    if world > 1:
        dist.barrier()
    evs = [(Event(enable_timing=True), Event(enable_timing=True)) for _ in sizes]
    sync(dev)
    if ctx is not None:  # live HIP-event timing of the hot kernels (roofline.dominant_kernel)
        for k in TIMED_KERNELS:
            ctx.kernel_timing_read(k)  # drop earlier records
        ctx.kernel_timing(True)
    t0 = time.perf_counter()
    n_batches = run(sizes, evs)
    steps = len(sizes)
    sync(dev)
    ktimes = {}
    if ctx is not None:
        ctx.kernel_timing(False)
        ktimes = {k: ctx.kernel_timing_read(k) for k in TIMED_KERNELS}
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    launch_ms = statistics.mean(a.elapsed_time(b) for a, b in evs)
    # the last launch on each stream left its vectors: every C2 batch's vector
    # equals its factory-known per-entry kinds (9,950 of 10k valid: 100 edge
    # cases, 50 of them valid under ZIP-215)
    valid, first = [], 0
    for i, kk in enumerate(sizes):
        f = i % F
        if i >= len(sizes) - F:
            for j in range(kk):
                got = d_valid[f][j * n:(j + 1) * n]
                assert torch.equal(got, want_status[(first + j) % R]), \
                    f"launch {i} batch {j}: vector differs from the factory's known per-entry kinds"
                v = int((got == 1).sum().item())
                assert v == expect_valid[(first + j) % R], (v, expect_valid[(first + j) % R])
                valid.append(v)
            if world > 1:  # the gathered vector holds every rank's copy of this launch
                assert gathered[f].numel() == world * kk * n
        first += kk
    build_digest = None if stub else (N.build_info() or {}).get("src_digest_compiled")

    def max_over_ranks(x):
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    elapsed = max_over_ranks(elapsed)
    # SCALE-run readiness: host setup (batch generation, H2D, workspaces,
    # warmup) before the timed region, and the device memory in use after it
    setup_s = max_over_ranks(t0 - t_main)
    dev_used_gib = 0.0
    if not stub:
        free_b, total_b = torch.cuda.mem_get_info(dev)
        dev_used_gib = max_over_ranks((total_b - free_b) / 2**30)

    def timed_reps(fn, reps, warm=2):
        """fn() `reps` times, each bracketed by a barrier and device syncs;
        per repetition the max over ranks of its wall time (seconds)."""
        for _ in range(warm):
            fn()
        out, last = [], None
        for _ in range(reps):
            if world > 1:
                dist.barrier()
            sync(dev)
            t1 = time.perf_counter()
            last = fn()
            sync(dev)
            out.append(max_over_ranks(time.perf_counter() - t1))
        return out, last

    def strong_leg(n_total, key_kind_s, local, kind_local, want_full, statuses, proxies):
        """One batch of n_total signatures split over the ranks by
        shard_range (contiguous): every rank verifies its shard
        and the validity vectors are all-gathered (RCCL), so every rank holds
        the exact full vector, which must equal want_full.  Kernel only:
        inputs resident in HBM, the gathered vector left on the device; end
        to end: the shard from host buffers through the host C-ABI, the
        gathered vector copied back to the host (one rank: the call's own
        host vector, nothing to gather).  Wall time per repetition =
        the max over ranks (barrier + device syncs around it)."""
        counts = [b - a for a, b in (shard_range(n_total, world, r) for r in range(world))]
        lo, hi = shard_range(n_total, world, rank)
        nl = hi - lo
        st = streams[0]
        flags_s = N.TMV_FLAG_BATCH_EQUATION if args.method == "batch" else N.TMV_FLAG_PER_ENTRY
        gather = all_gather_statuses if statuses else all_gather_validity
        tdev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
        d_pk, d_sig, d_off = tdev(local.pk), tdev(local.sig), tdev(local.off.view(np.int32))
        d_msg = tdev(local.msg if local.msg.size else np.zeros(1, np.uint8))
        d_kind = tdev(kind_local) if kind_local is not None else None
        out = torch.zeros(max(nl, 1), dtype=torch.int8, device=dev)
        want_dev = tdev(want_full)
        want_local = want_dev[lo:hi].to(torch.int8)

        def full(v):  # this rank's vector -> the whole job's, on the device
            if world == 1:
                return v if statuses else (v == 1).to(torch.uint8)
            return gather(v, counts)

        def launch_shard(m):
            if stub:
                out[:m].copy_(want_local[:m])
            else:
                ctx.verify_batch_device_ex(gpu, key_kind_s, flags_s, d_kind.data_ptr() if d_kind is not None else 0,
                                           d_pk.data_ptr(), d_sig.data_ptr(), d_msg.data_ptr(), d_off.data_ptr(), m,
                                           out.data_ptr(), st.cuda_stream)

        def kernel_only():
            with stream_ctx(st):
                launch_shard(nl)
                return full(out[:nl])

        def end_to_end():
            if stub:
                v = want_full[lo:hi].astype(np.int8)
            elif kind_local is None:
                v = ctx.verify_batch_ex(key_kind_s, flags_s, local.pk, local.sig, local.msg, local.off)[1]
            else:
                v = ctx.verify_mixed_batch_ex(flags_s, kind_local, local.pk, local.sig, local.msg, local.off)[1]
            v = np.asarray(v, np.int8)
            if world == 1:  # the call already returned the whole vector on the host: nothing to gather
                return torch.from_numpy(v if statuses else (v == 1).astype(np.uint8))
            with stream_ctx(st):
                return full(tdev(v)).cpu()

        k_t, g = timed_reps(kernel_only, args.strong_reps)
        assert torch.equal(g, want_dev), "strong scaling: gathered vector differs from the known one (kernel path)"
        h_t, gh = timed_reps(end_to_end, args.strong_reps, warm=1)
        assert torch.equal(gh, want_dev.cpu()), "strong scaling: gathered vector differs (end to end)"
        km, hm = statistics.median(k_t), statistics.median(h_t)
        res = {"signatures": n_total, "ranks": world, "shard_per_rank": counts, "method": args.method,
               "kernel_only": {"ms": round(km * 1e3, 4), "verifies_per_s": round(n_total / km, 1),
                               "ms_reps": [round(x * 1e3, 4) for x in k_t]},
               "end_to_end": {"ms": round(hm * 1e3, 4), "verifies_per_s": round(n_total / hm, 1),
                              "ms_reps": [round(x * 1e3, 4) for x in h_t]},
               "exact_vector_on_every_rank": True,
               "note": (f"one {n_total}-signature batch split over {world} rank(s) (contiguous shards), every rank "
                        "verifies its shard and the vectors are all-gathered"
                        + (f" ({'RCCL' if dist.get_backend() == 'nccl' else dist.get_backend()})"
                           if world > 1 and not stub and dist.is_initialized() else "")
                        + "; every rank's full vector equals the "
                        "known one; wall time = max over ranks, median of the repetitions; kernel_only: inputs "
                        "resident in HBM, vector left on the device; end_to_end: host buffers through the C-ABI, "
                        "vector back on the host")}
        if proxies and world == 1 and not stub:
            # the shard one GPU of an N-GPU job would verify, launched alone
            prox = {}
            for parts in (1, 2, 4, 8):
                m = n_total // parts
                lat = []
                for r_ in range(7):
                    e = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                    e[0].record(st)
                    launch_shard(m)
                    e[1].record(st)
                    torch.cuda.synchronize(dev)
                    if r_ >= 2:
                        lat.append(e[0].elapsed_time(e[1]))
                ms = statistics.median(lat)
                prox[f"n{parts}"] = {"shard": m, "launch_alone_ms": round(ms, 4),
                                     "verifies_per_s": round(m / (ms * 1e-3), 1)}
            res["single_gpu_shard_proxy"] = dict(
                prox, note="single-GPU proxy, NOT scaling: the 1/N shard of this batch launched alone on one GPU "
                           "(HIP events, median of 5); an N-GPU run adds the all-gather and the max over ranks")
        return res

    def strong_leg_ed(n_total):
        """north_star target: C2-shaped ed25519 (1% corrupted / ZIP-215
        edge cases), batch j = make_c2_batch(nb, STRONG_SEED + j)."""
        j0 = strong_js[0] if strong_js else 0
        loc = Batch.concat(strong_batches).take(np.arange(s_lo - j0 * nb, s_hi - j0 * nb)) if strong_js else \
            Batch.from_entries([])
        n_bat = -(-n_total // nb)
        want = np.fromiter((k in VALID_KINDS for j in range(n_bat) for k in c2_kinds(nb, STRONG_SEED + j)),
                           np.uint8, count=n_bat * nb)[:n_total]
        r = strong_leg(n_total, N.TMV_KIND_ED25519, loc, None, want, False, True)
        r["workload"] = (f"C2-shaped: {n_total} ed25519 signatures = {n_bat} distinct C2 batches of {nb} (1% "
                         "corrupted / ZIP-215 edge cases each); known vector from the generator's per-entry kinds")
        return r

    def strong_leg_mixed(n_total):
        """C5 (BASELINE configs[4]): mixed ed25519 + sr25519, a 20k base
        tiled; the known vector is the base's per-entry statuses (sr25519
        Add errors included) from the C oracle (checker role, set up outside
        the timed region), tiled."""
        kind_b, base = mixed_base
        idx = np.arange(s_lo, s_hi) % base.n
        loc = base.take(idx)
        if stub:
            want_b = np.array([0 if ("bitflip" in k or "flip" in k or "plus" in k or "undec" in k) else 1
                               for k in base.kinds], np.int8)
        else:
            want_b = mixed_oracle_statuses(kind_b, base)
        want = np.asarray(want_b, np.int8)[np.arange(n_total) % base.n]
        r = strong_leg(n_total, N.TMV_KIND_MIXED, loc, np.ascontiguousarray(kind_b[idx]), want, True, False)
        r["workload"] = (f"C5-shaped: {n_total} mixed ed25519 + sr25519 signatures (a {base.n}-entry mixed base "
                         "tiled, ~1% of each kind corrupted); known vector = C oracle (oracle/c: ed25519 ZIP-215 "
                         "and sr25519 statuses of the base, computed at setup as the checker), tiled")
        return r

    extras = {}
    ktimes_alone = {}
    if not args.no_extras:
        # end to end on every rank at once: each rank streams its own host
        # batch (the timed region's launch size, TMV_BENCH_E2E_BATCHES
        # resident batches as one host-resident batch) through the host C-ABI
        # (staging / the caller's pages pinned and DMA'd, kernels, D2H);
        # whole-job rate = all ranks' signatures / the max over ranks
        KE = max(1, min(K, int(os.environ.get("TMV_BENCH_E2E_BATCHES", str(K)))))
        hb = Batch.concat([batches[j % R] for j in range(KE)])
        want_e2e = sum(expect_valid[j % R] for j in range(KE))
        stub_e2e = np.concatenate([want_status[j % R].cpu().numpy() for j in range(KE)]) if stub else None

        def e2e_call():
            if stub:
                return stub_e2e
            return ctx.verify_batch_ex(key_kind, flags, hb.pk, hb.sig, hb.msg, hb.off)[1]
        e2e_t, st_e2e = timed_reps(e2e_call, 5, warm=1)
        assert int((np.asarray(st_e2e) == 1).sum()) == want_e2e
        e2e_s = statistics.median(e2e_t)
        extras["end_to_end_verifies_per_s"] = round(world * hb.n / e2e_s, 1)
        h2d = hb.pk.nbytes + hb.sig.nbytes + hb.msg.nbytes + hb.off.nbytes
        extras["end_to_end_h2d_bytes_per_sig"] = round(h2d / hb.n, 1)
        extras["end_to_end_h2d_GBps"] = round(world * h2d / e2e_s / 1e9, 2)
        extras["end_to_end_note"] = (f"every rank at once: {hb.n} host-resident signatures per rank per call (the "
                                     "caller's pages pinned part by part and DMA'd directly, TMV_REGISTER; + kernels "
                                     f"+ D2H), {world} x {hb.n} / the max over ranks of the call's wall time (median "
                                     "of 5); never the headline value")
        del hb
        if strong_n:
            extras["strong_1m"] = strong_leg_ed(strong_n)
            if mixed_base is not None:
                extras["strong_1m_mixed"] = strong_leg_mixed(strong_n)
    if rank == 0 and not args.no_extras and not stub:
        # one launch of K batches alone on one stream (no overlap): the
        # pipeline's own duration, HIP events on its stream
        alone = []
        ctx.kernel_timing(True)
        for _ in range(5):
            e = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            launch(0, 0, K, e, gather=False)  # rank 0 alone: no collective
            torch.cuda.synchronize(dev)
            alone.append(e[0].elapsed_time(e[1]))
        ctx.kernel_timing(False)
        ktimes_alone.update({k: ctx.kernel_timing_read(k) for k in TIMED_KERNELS})
        extras["launch_alone_ms"] = round(statistics.median(alone), 4)
        # sustained: the timed region's pattern (F launches in flight) for
        # ~TMV_BENCH_SUSTAIN_S seconds -- a steadier rate than K steps, and a
        # GPU busy long enough for an outside utilisation sampler to see
        sustain_s = float(os.environ.get("TMV_BENCH_SUSTAIN_S", "3"))
        if sustain_s > 0:
            sync(dev)
            t1, nl = time.perf_counter(), 0
            while True:
                for _ in range(4 * F):
                    launch(nl, (nl * K) % R, K, gather=False)
                    nl += 1
                sync(dev)
                if time.perf_counter() - t1 >= sustain_s:
                    break
            dt = time.perf_counter() - t1
            extras["sustained_verifies_per_s"] = round(nl * K * n / dt, 1)
            extras["sustained_seconds"] = round(dt, 3)
            extras["sustained_note"] = (f"{nl} launches of {K} C2 batches, {F} in flight, one device sync per "
                                        f"{4 * F} launches (rank 0, after the timed region; not the headline value)")
        # single-batch latency (one 10k batch per launch, one at a time), with
        # the runtime's own choice for a batch this size (flags 0: per entry
        # below TMV_MSM_MIN) and through the batch equation
        def one_batch_ms(fl):
            lat = []
            for _ in range(12):
                e = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                e[0].record(streams[0])
                ctx.verify_batches_device(gpu, N.TMV_KIND_ED25519, fl, refs(0, 0, 1), streams[0].cuda_stream)
                e[1].record(streams[0])
                torch.cuda.synchronize(dev)
                lat.append(e[0].elapsed_time(e[1]))
            return statistics.median(lat[2:])
        batch_ms = one_batch_ms(0)
        extras["batch_latency_ms"] = round(batch_ms, 4)
        extras["batch_latency_note"] = "one C2 batch alone, runtime default method (per entry at 10k)"
        extras["batch_latency_ms_batch_equation"] = round(one_batch_ms(flags), 4)
        extras["serial_verifies_per_s"] = round(n / (batch_ms * 1e-3), 1)
        # the same KE batches as one resident launch alone on rank 0: the
        # end-to-end rate over it isolates staging + PCIe + D2H
        if world == 1:
            KE = max(1, min(K, int(os.environ.get("TMV_BENCH_E2E_BATCHES", str(K)))))
            same = []
            for _ in range(3):
                e = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                launch(0, 0, KE, e, gather=False)
                torch.cuda.synchronize(dev)
                same.append(e[0].elapsed_time(e[1]))
            extras["end_to_end_vs_same_call_kernels"] = round(
                extras["end_to_end_verifies_per_s"] / (KE * n / (statistics.median(same) * 1e-3)), 3)
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
        extras["verify_commit_150_p50_ms"] = round(lat[len(lat) // 2], 4)
        extras["verify_commit_150_p99_ms"] = round(lat[int(len(lat) * 0.99) - 1], 4)
        extras["verify_commit_note"] = "types.VerifyCommit (C1: 150 validators) via tmv_verify_commit, host-resident commit"

    result = None
    if rank == 0:
        total = n * world * n_batches
        value = total / elapsed
        gpu_rate = n * n_batches / elapsed  # this rank
        peak = _load_peak()
        pmc = _load_pmc(args.method, K)
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
                       "step": f"one device launch verifying {K} C2 batches ({n:,} signatures each) to their exact "
                               "validity vectors",
                       "batch": n, "batches_per_step": K, "signatures_per_step": K * n,
                       "launches_in_flight": F, "resident_batches": R,
                       "method": args.method, "msg_bytes_avg": round(float(batch.msg.size) / n, 1),
                       "parallelism": (f"shard{world} ({dist.get_backend()}, process group world size "
                                       f"{dist.get_world_size()})" if world > 1 and dist.is_initialized()
                                       else "single")},
            "valid_per_batch": valid[0],
            "run_timing": {"setup_s_max_over_ranks": round(setup_s, 2),
                           "device_mem_in_use_gib_max_over_ranks": round(dev_used_gib, 2),
                           "note": "setup = process start to the timed region (C2 generation, H2D of the resident "
                                   "batches, context / workspaces, warmup); device memory = total - free on the "
                                   "rank's GPU after the timed region (every process on that GPU)"},
            **extras,
            "roofline": _pipeline_roofline(gpu_rate, peak, pmc, launch_ms, args.method, K * n, elapsed / steps * 1e3,
                                           build_digest),
        }
        if ktimes.get("k_msm_accum", (0, 0))[1] and args.method == "batch":
            result["roofline"] = _dominant_roofline(ktimes, ktimes_alone, K, n, args, peak, steps,
                                                    result["roofline"], elapsed / steps * 1e3, build_digest)
        if "end_to_end_verifies_per_s" in result:
            result["end_to_end_vs_headline"] = round(result["end_to_end_verifies_per_s"] / value, 4)
        if not stub:
            result["build"] = N.build_info()
        if stub:
            result["data"] = "CPU STUB (--cpu-stub): control-flow check only, no verification, not a measurement"
        if world == 1 and not args.no_cpu_baseline and not stub:
            result["cpu_baseline"] = cpu_baseline(batches)
            c1 = result["cpu_baseline"].get("verify_commit_150") or {}
            if "verify_commit_150_p50_ms" in result and c1:
                # beside the GPU's C1 latency: the CPU restatement, labelled
                result["verify_commit_150_cpu_p50_ms"] = c1["p50_ms"]
                result["verify_commit_150_cpu_p99_ms"] = c1["p99_ms"]
                result["verify_commit_150_cpu_note"] = "CPU port, one thread, not the reference (cpu_baseline.verify_commit_150)"
        else:
            result["cpu_baseline"] = None
        result["run_timing"]["process_start_to_print_s_rank0"] = round(time.perf_counter() - t_main, 2)
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return result


if __name__ == "__main__":
    main()
