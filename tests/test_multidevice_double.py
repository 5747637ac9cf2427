"""A multi-device context without GPUs: the CPU test
double (tests/native/commit_check.cpp) runs every engine batch through the
runtime's own shard plan and launch / harvest order (host/shard_plan.h,
host/shard_run.h -- what tmv_open(mask) with several devices executes in
tmverify_runtime.cpp run_batch) over simulated devices, under the product's
host layer (tm_host_abi.cpp, tm_light_abi.cpp).  tmv_verify_commits
(blocksync windows) and tmv_light_verify_many (a light window) sharded over
2 and 3 devices return exactly what one device returns, every entry is
launched once, each device gets one contiguous shard, and a lane's chunk is
harvested before the lane is reused."""
import ctypes

import numpy as np
import pytest

import commit_fixtures as F
from tendermint_amd import host as H
from tendermint_amd.testing.factory import make_block_chain, make_light_chain

PERIOD = 14 * 24 * 3600 * 10**9
DRIFT = 10 * 10**9


@pytest.fixture()
def fake():
    fb = F.FakeBackend()
    fb.real_signatures(True)
    L = fb.L
    L.commitcheck_set_devices.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]
    L.commitcheck_steps.restype = ctypes.c_uint32
    L.commitcheck_steps.argtypes = [ctypes.POINTER(ctypes.c_uint32), ctypes.c_uint32]
    yield fb
    L.commitcheck_set_devices(1, 262144, 2)
    fb.real_signatures(False)


def _steps(fb):
    buf = (ctypes.c_uint32 * (5 * 100000))()
    n = fb.L.commitcheck_steps(buf, 100000)
    return np.frombuffer(buf, np.uint32, count=5 * n).reshape(n, 5)


def _check_placement(steps, n_dev):
    """Per engine batch (a run of steps whose launches cover [0, n)): each
    entry launched once, device d's launches form one contiguous range and
    the devices' ranges are in order; every launch harvested once, and a
    lane is harvested before it is launched again."""
    batches, cur = [], []
    for st in steps:
        cur.append(tuple(int(x) for x in st))
        launched = sorted((lo, hi) for k, _, _, lo, hi in cur if k == 0)
        harvested = sorted((lo, hi) for k, _, _, lo, hi in cur if k == 1)
        if launched and launched == harvested and launched[0][0] == 0 and \
                all(a[1] == b[0] for a, b in zip(launched, launched[1:])):
            batches.append(cur)
            cur = []
    assert not cur, "steps left over after the last complete batch"
    multi = 0
    for b in batches:
        n = max(hi for _, _, _, _, hi in b)
        by_dev = {}
        for k, d, _, lo, hi in b:
            if k == 0:
                by_dev.setdefault(d, []).append((lo, hi))
        ranges = []
        for d in sorted(by_dev):
            r = sorted(by_dev[d])
            assert all(a[1] == b2[0] for a, b2 in zip(r, r[1:])), f"device {d} shard not contiguous"
            ranges.append((r[0][0], r[-1][1]))
        assert ranges[0][0] == 0 and ranges[-1][1] == n
        assert all(a[1] == b2[0] for a, b2 in zip(ranges, ranges[1:]))
        assert len(by_dev) <= n_dev
        multi += len(by_dev) > 1
        busy = {}
        for k, d, lane, lo, hi in b:
            if k == 0:
                assert (d, lane) not in busy, "lane launched again before its chunk was harvested"
                busy[(d, lane)] = (lo, hi)
            else:
                assert busy.pop((d, lane)) == (lo, hi)
        assert not busy
    return len(batches), multi


@pytest.mark.parametrize("n_dev,chunk", [(2, 2048), (3, 2048)])
def test_verify_commits_sharded_equals_one_device(fake, n_dev, chunk):
    vals, blocks = make_block_chain(64, 160, seed=5)
    for i, c in ((9, 3), (30, 159), (31, 0)):
        cm = blocks[i].last_commit
        s = cm.signatures[c]
        b = bytearray(s.signature)
        b[7] ^= 2
        cm.signatures[c] = H.CommitSig(s.block_id_flag, s.validator_address, s.timestamp, bytes(b))
    jobs = []
    for i in range(1, len(blocks) - 1):
        f, s2 = blocks[i], blocks[i + 1]
        jobs.append(H.CommitJob(H.MODE_LIGHT, "test_chain_id", vals, f.block_id, f.height, s2.last_commit))
        jobs.append(H.CommitJob(H.MODE_FULL, "test_chain_id", vals, blocks[i - 1].block_id, f.height - 1,
                                f.last_commit))
    fake.L.commitcheck_set_devices(1, 262144, 2)
    one = F.fake_verify_commits(fake, jobs)
    _steps(fake)
    fake.L.commitcheck_set_devices(n_dev, chunk, 2)
    many = F.fake_verify_commits(fake, jobs)
    steps = _steps(fake)
    assert many == one and sum(e is not None for e in one) == 5  # light + full of two commits, full of one
    n_batches, multi = _check_placement(steps, n_dev)
    assert n_batches >= 1 and multi >= 1
    assert len({(d, lane) for k, d, lane, _, _ in steps if k == 0}) > n_dev  # several chunks per device


def test_light_window_sharded_equals_one_device(fake):
    trusted, blocks = make_light_chain(120, 40, seed=9)
    now = (blocks[-1].signed_header.header.time[0] + 5, 0)
    cm = blocks[70].signed_header.commit
    s = cm.signatures[5]
    cm.signatures[5] = H.CommitSig(s.block_id_flag, s.validator_address, s.timestamp, bytes(64))
    jobs, prev = [], trusted
    for lb in blocks:
        jobs.append(H.LightJob(prev.signed_header, None, lb.signed_header, lb.vals, PERIOD, now, DRIFT,
                               mode=H.LIGHT_ADJACENT))
        prev = lb
    fake.L.commitcheck_set_devices(1, 262144, 2)
    one = fake.light_verify_many(jobs)
    _steps(fake)
    fake.L.commitcheck_set_devices(2, 2048, 2)
    many = fake.light_verify_many(jobs)
    steps = _steps(fake)
    assert many == one and [k for k, (c, _) in enumerate(one) if c != H.LIGHT_OK] == [70]
    n_batches, multi = _check_placement(steps, 2)
    assert multi >= 1
