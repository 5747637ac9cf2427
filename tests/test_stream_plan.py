"""Streamed host-buffer chunks (tendermint_amd/csrc/host/stream_plan.h, used
by the runtime's stage_and_launch / batch_check / mixed_check_streamed): the
part schedule (a short first part, parts doubling up to TMV_STREAM_PART,
group edges for one-kind launches, a part cap for mixed chunks) and the
caller-page locking (two locked ranges per span, only whole pages inside the
caller's bytes, the rest staged, a failed lock staging the span for the rest
of the chunk).  CPU, through the harness build (tests/native/commit_check.cpp)."""
import ctypes
import random

import numpy as np
import pytest

import commit_fixtures as F

PAGE = 4096


@pytest.fixture(scope="module")
def L():
    lib = F.FakeBackend().L
    lib.commitcheck_stream_parts.restype = ctypes.c_uint32
    lib.commitcheck_stream_parts.argtypes = [ctypes.c_uint32] * 4 + [ctypes.c_int, ctypes.c_int, ctypes.c_uint32,
                                                                      ctypes.POINTER(ctypes.c_uint32), ctypes.c_uint32]
    lib.commitcheck_pin_walk.restype = ctypes.c_uint32
    lib.commitcheck_pin_walk.argtypes = [ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint32,
                                         ctypes.c_uint64, ctypes.c_int, ctypes.c_uint64,
                                         ctypes.POINTER(ctypes.c_uint64)]
    return lib


def parts(L, n, m=128, first=32768, part=131072, ramp=True, mixed=False, max_parts=512):
    k = L.commitcheck_stream_parts(n, m, first, part, int(ramp), int(mixed), max_parts, None, 0)
    buf = np.zeros(max(1, k), np.uint32)
    assert L.commitcheck_stream_parts(n, m, first, part, int(ramp), int(mixed), max_parts,
                                      buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), k) == k
    return [int(x) for x in buf[:k]]


def test_default_schedule_ramps_to_the_part_size(L):
    b = parts(L, 2_560_000)
    sizes = np.diff(b)
    assert b[0] == 0 and b[-1] == 2_560_000
    assert list(sizes[:4]) == [32768, 65536, 131072, 131072]
    assert all(s <= 131072 for s in sizes)
    assert all(x % 128 == 0 for x in b[:-1])
    # without the ramp: 32k, then 128k parts (rounds 2-5)
    nr = np.diff(parts(L, 2_560_000, ramp=False))
    assert list(nr[:3]) == [32768, 131072, 131072]


@pytest.mark.parametrize("n,m,first,part", [(200_000, 64, 32768, 131072), (40_000, 64, 32768, 131072),
                                            (150_091, 128, 1000, 3000), (1, 64, 32768, 131072),
                                            (4_000_000, 128, 8192, 262144), (12_345, 32, 100, 100)])
@pytest.mark.parametrize("ramp", [True, False])
def test_one_kind_parts_are_whole_groups(L, n, m, first, part, ramp):
    b = parts(L, n, m, first, part, ramp)
    assert b[0] == 0 and b[-1] == n and all(x < y for x, y in zip(b, b[1:]))
    assert all(x % m == 0 for x in b[:-1])  # every part starts on a group edge; only the last may end off one
    sizes = np.diff(b)
    cap = -(-max(first, part) // m) * m
    assert all(s <= cap for s in sizes[:-1])
    if ramp:  # doubling, never more than twice the previous request (+ group rounding)
        want = first
        for s in sizes[:-1]:
            assert s == -(-want // m) * m or s >= want
            want = min(part, 2 * want)


@pytest.mark.parametrize("n", [1, 1000, 1_000_000, 4_194_304, 60_000_000])
@pytest.mark.parametrize("ramp", [True, False])
def test_mixed_parts_respect_the_part_cap(L, n, ramp):
    b = parts(L, n, mixed=True, ramp=ramp, max_parts=512)
    assert b[0] == 0 and b[-1] == n and all(x < y for x, y in zip(b, b[1:]))
    assert len(b) - 1 <= 512


def pin_walk(L, base, lens, fail_at=-1, min_len=4 * PAGE):
    arr = (ctypes.c_uint64 * len(lens))(*lens)
    out = (ctypes.c_uint64 * (3 * len(lens) + 16))()
    k = L.commitcheck_pin_walk(base, arr, len(lens), PAGE, fail_at, min_len, out)
    per = [(out[3 * i], out[3 * i + 1], out[3 * i + 2]) for i in range(len(lens))]
    rng = [(out[3 * len(lens) + 2 * j], out[3 * len(lens) + 2 * j + 1]) for j in range(k)]
    return per, rng


def check_walk(base, lens, per, rng, fail_at=-1):
    end = base + sum(lens)
    assert len(rng) <= 2
    for r0, r1 in rng:  # whole pages, inside the caller's span
        assert r0 % PAGE == 0 and r1 % PAGE == 0 and r1 > r0
        assert base <= r0 and r1 <= end
    for (a0, a1), (b0, b1) in zip(rng, rng[1:]):  # disjoint, contiguous
        assert a1 == b0
    locked = lambda x0, x1: any(r0 <= x0 and x1 <= r1 for r0, r1 in rng)  # noqa: E731
    s0 = base
    for ln, (d0, d1, cut) in zip(lens, per):
        assert 0 <= d0 <= cut <= d1 <= ln
        if d1 > d0:
            # each DMA piece lies inside one locked range
            if cut > d0:
                assert locked(s0 + d0, s0 + cut)
            if d1 > cut:
                assert locked(s0 + cut, s0 + d1)
            # the split is exactly at the boundary between the two ranges
            if cut < d1:
                assert len(rng) == 2 and s0 + cut == rng[1][0]
        s0 += ln


def test_two_ranges_cover_every_whole_page(L):
    base = 0x7F00_0000_0010  # a numpy-like data pointer: 16 bytes past a page
    lens = [32768 * 64, 65536 * 64, 131072 * 64, 131072 * 64, 131072 * 64 + 320]
    per, rng = pin_walk(L, base, lens)
    check_walk(base, lens, per, rng)
    assert len(rng) == 2
    end = base + sum(lens)
    assert rng[0][0] == -(-base // PAGE) * PAGE and rng[1][1] == end // PAGE * PAGE
    # only part 0's head and tail and the last part's tail are staged
    staged = [ln - (d1 - d0) for ln, (d0, d1, _) in zip(lens, per)]
    assert staged[1:-1] == [0] * (len(lens) - 2)
    assert 0 < staged[0] < 2 * PAGE and 0 < staged[-1] < PAGE


@pytest.mark.parametrize("seed", range(40))
def test_random_spans(L, seed):
    rnd = random.Random(seed)
    base = rnd.randrange(1 << 30, 1 << 40)
    lens = [rnd.choice([rnd.randrange(1, 3 * PAGE), rnd.randrange(4 * PAGE, 64 * PAGE), rnd.randrange(1, 200 * PAGE)])
            for _ in range(rnd.randrange(1, 12))]
    per, rng = pin_walk(L, base, lens)
    check_walk(base, lens, per, rng)


@pytest.mark.parametrize("fail_at", [0, 1])
def test_a_failed_lock_stages_the_rest(L, fail_at):
    base = 0x10_0000_0123
    lens = [40 * PAGE, 80 * PAGE, 160 * PAGE, 160 * PAGE]
    per, rng = pin_walk(L, base, lens, fail_at=fail_at)
    check_walk(base, lens, per, rng)
    assert len(rng) == fail_at
    # after the failure nothing more is DMA'd from the caller's pages
    first_failed = 0 if fail_at == 0 else 1
    for d0, d1, _ in per[first_failed:]:
        assert d1 == d0
