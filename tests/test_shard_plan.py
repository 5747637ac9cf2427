"""Shard and chunk plan of host-buffer batches (tendermint_amd/csrc/host/
shard_plan.h, used by the runtime's run_batch): one contiguous shard per
device of a tmv_open(mask) context (tiny batches on one device), each shard
cut into chunks that rotate over the device's lanes.  The results of chunk
[lo, hi) land at out[lo:hi], so the plan is the per-device result placement.
CPU, through the harness build (tests/native/commit_check.cpp)."""
import ctypes

import numpy as np
import pytest

import commit_fixtures as F


@pytest.fixture(scope="module")
def plan():
    L = F.FakeBackend().L
    L.commitcheck_shard_plan.restype = ctypes.c_uint32
    L.commitcheck_shard_plan.argtypes = [ctypes.c_uint32] * 3 + [ctypes.POINTER(ctypes.c_uint32), ctypes.c_uint32]

    def run(n, ndev, chunk=262144):
        k = L.commitcheck_shard_plan(n, ndev, chunk, None, 0)
        buf = np.zeros(4 * max(1, k), np.uint32)
        assert L.commitcheck_shard_plan(n, ndev, chunk, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), k) == k
        return buf[:4 * k].reshape(-1, 4)
    return run


@pytest.mark.parametrize("n,ndev,chunk", [
    (1, 8, 262144), (1023, 8, 262144), (1024, 8, 262144), (5000, 8, 262144), (10_000, 3, 2048),
    (320_000, 1, 262144), (320_000, 8, 262144), (1_000_000, 8, 262144), (1_000_003, 7, 131072),
    (4_000_000, 8, 262144), (70_000, 2, 65536), (2**32 - 1 - 7, 8, 262144)])
def test_plan_partitions_batch(plan, n, ndev, chunk):
    p = plan(n, ndev, chunk)
    shards = max(1, min(ndev, n // 1024))
    dev = p[:, 0]
    assert set(dev.tolist()) == set(range(shards))
    # every entry in exactly one chunk; per device the chunks are contiguous, in order
    order = np.lexsort((p[:, 3], dev))
    q = p[order]
    assert q[0, 1] == 0 and q[-1, 2] == n
    assert (q[1:, 1] == q[:-1, 2]).all() and (q[:, 2] > q[:, 1]).all()
    # equal contiguous shards (sizes differ by at most one)
    sizes = [int(q[q[:, 0] == s][:, 2].max() - q[q[:, 0] == s][:, 1].min()) for s in range(shards)]
    assert max(sizes) - min(sizes) <= 1
    # launch order: chunk k of every shard before chunk k + 1 of any
    assert (np.diff(p[:, 3].astype(np.int64)) >= 0).all()
    # chunk sizes: at least half a chunk (unless the shard is smaller), at most ~1 chunk + rounding
    c = max(2048, chunk)
    for s in range(shards):
        cs = q[q[:, 0] == s]
        lens = cs[:, 2] - cs[:, 1]
        if sizes[s] >= c // 2:
            assert lens.min() >= c // 2 - 1
        assert len(cs) == 1 or len(cs) <= max(4, sizes[s] // c)


def test_placement_roundtrip(plan):
    """Executing the plan (each chunk writes its own results at out[lo:hi])
    reassembles the whole vector for any device count."""
    n = 777_777
    want = (np.arange(n) * 2654435761 % 7 == 0).astype(np.uint8)
    for ndev in range(1, 9):
        out = np.full(n, 0xEE, np.uint8)
        for d, lo, hi, k in plan(n, ndev, 131072):
            out[lo:hi] = want[lo:hi]
        assert np.array_equal(out, want)
