"""Failure handling: a device wait is bounded
(TMV_DEVICE_TIMEOUT_MS -> TMV_ERR_TIMEOUT, tendermint_amd/csrc/host/wait.h
used by every wait in tmverify_runtime.cpp), and an infrastructure error of
the engine surfaces from every host-layer entry point as an error (< 0 /
NativeError), never as a verdict, so the Go shim can re-verify on the CPU
(INTEGRATION.md).  CPU harness: tests/native/commit_check.cpp."""
import ctypes

import pytest

import commit_fixtures as F
from tendermint_amd import host as H
from tendermint_amd._native import NativeError

TMV_ERR_TIMEOUT = -5
READY, ERROR, TIMEOUT = 0, 1, 2


@pytest.fixture(scope="module")
def fake():
    fb = F.FakeBackend()
    fb.L.commitcheck_poll.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.POINTER(ctypes.c_double)]
    fb.L.commitcheck_fail_next.argtypes = [ctypes.c_int]
    fb.L.commitcheck_ctx.restype = ctypes.c_void_p
    yield fb
    fb.L.commitcheck_fail_next(0)


def _poll(fake, ready_after, fail, timeout_ms):
    el = ctypes.c_double()
    r = fake.L.commitcheck_poll(ready_after, fail, timeout_ms, ctypes.byref(el))
    return r, el.value


def test_poll_until(fake):
    assert _poll(fake, 0, 0, 1000)[0] == READY
    assert _poll(fake, 5000, 0, 5000)[0] == READY      # finishes after many polls
    r, ms = _poll(fake, -1, 0, 50)                      # never finishes
    assert r == TIMEOUT and 50 <= ms < 1000
    assert _poll(fake, -1, 1, 50)[0] == ERROR            # the query reports a device error
    r, ms = _poll(fake, 3, 0, 0)                         # 0 = unbounded
    assert r == READY


def test_timeout_surfaces_from_verify_commit(fake):
    vals, signers = F.rand_val_set("fake", 4, 10)
    bid = F.random_block_id(3)
    commit = F.make_commit(signers, "c", 3, 0, bid)
    assert fake.verify_commit("c", vals, bid, 3, commit) is None
    fake.L.commitcheck_fail_next(TMV_ERR_TIMEOUT)
    with pytest.raises(NativeError):
        fake.verify_commit("c", vals, bid, 3, commit)
    assert fake.verify_commit("c", vals, bid, 3, commit) is None  # the double recovered; the engine would not


def test_timeout_surfaces_from_batch_verifier(fake):
    v = H.create_batch_verifier(fake.L.commitcheck_ctx(), H.TMV_KIND_ED25519, fake.L)
    v.add(H.TMV_KIND_ED25519, bytes(32), b"m", bytes(64))
    fake.L.commitcheck_fail_next(TMV_ERR_TIMEOUT)
    with pytest.raises(NativeError):
        v.verify()


def test_timeout_surfaces_from_light_verify(fake):
    from tendermint_amd.testing.factory import make_light_chain
    trusted, blocks = make_light_chain(3, 4)
    now = (blocks[-1].signed_header.header.time[0] + 1, 0)
    job = H.LightJob(trusted.signed_header, None, blocks[0].signed_header, blocks[0].vals, 10**15, now,
                     mode=H.LIGHT_ADJACENT)
    fake.real_signatures(True)
    try:
        assert fake.light_verify_many([job]) == [(H.LIGHT_OK, None)]
        fake.L.commitcheck_fail_next(TMV_ERR_TIMEOUT)
        with pytest.raises(NativeError):
            fake.light_verify_many([job])
    finally:
        fake.real_signatures(False)


def test_sliced_call_error_reaches_caller_thread(fake, monkeypatch):
    """a sliced call (TMV_HOST_SLICE) whose failing slice ran on
    the partner thread still returns that slice's infrastructure error, with
    its message as the caller thread's last error and in errs[0] (copied
    after every slice has finished, so no slice's own error text races it)."""
    import numpy as np
    monkeypatch.setenv("TMV_HOST_SLICE", "4")
    fake.L.tmv_last_error.restype = ctypes.c_char_p
    L = fake.L
    L.commitcheck_verify_commits.argtypes = [ctypes.POINTER(H.CCommitJob), ctypes.c_uint32,
                                             ctypes.POINTER(ctypes.c_int32), ctypes.c_char_p, ctypes.c_size_t]
    L.commitcheck_verify_commits.restype = ctypes.c_int
    jobs = F.random_jobs("fake", 32, seed=11)
    pj = H.PreparedJobs(jobs)
    seen = set()
    for _ in range(12):  # the failing call lands on either thread; both must report it
        fake.L.commitcheck_fail_next(TMV_ERR_TIMEOUT)
        rc = L.commitcheck_verify_commits(pj.arr, pj.n, pj.results, pj.errs, pj.stride)
        assert rc == TMV_ERR_TIMEOUT
        msg = fake.L.tmv_last_error().decode()
        assert msg.startswith("fake infrastructure error on thread"), msg
        raw = ctypes.string_at(pj.errs, pj.stride)
        assert raw.split(b"\0")[0].decode() == msg
        seen.add(msg)
    # a clean call after the failures: results equal a one-slice run's
    ok = L.commitcheck_verify_commits(pj.arr, pj.n, pj.results, pj.errs, pj.stride)
    sliced = pj.decode()
    monkeypatch.setenv("TMV_HOST_SLICE", "0")
    pj1 = H.PreparedJobs(jobs)
    assert L.commitcheck_verify_commits(pj1.arr, pj1.n, pj1.results, pj1.errs, pj1.stride) == ok >= 0
    assert pj1.decode() == sliced
    assert len(seen) >= 1 and np.all(np.asarray([len(s) for s in seen]) > 0)


def test_random_source_failure_is_an_error_not_a_spin():
    """A getrandom failure while drawing a launch's weights key returns
    TMV_ERR_RANDOM with the errno in tmv_last_error (it
    used to loop forever); EINTR and short reads are retried
    (crypto/ed25519/ed25519.go:232 surfaces rand.Reader errors)."""
    import errno
    from tendermint_amd import _native
    L = _native.lib()
    L.tmv_internal_random_fault.argtypes = [ctypes.c_int, ctypes.c_int]
    L.tmv_internal_draw_key.argtypes = [ctypes.c_void_p]
    L.tmv_last_error.restype = ctypes.c_char_p
    key = (ctypes.c_uint8 * 32)()
    try:
        assert L.tmv_internal_draw_key(key) == 0
        assert any(key)
        for err in (errno.ENOSYS, errno.EPERM):
            L.tmv_internal_random_fault(err, -1)  # every call fails
            assert L.tmv_internal_draw_key(key) == -6  # TMV_ERR_RANDOM, returned at once
            assert L.tmv_last_error().decode().startswith("getrandom: ")
        L.tmv_internal_random_fault(errno.EINTR, 3)  # interrupted three times, then fine
        assert L.tmv_internal_draw_key(key) == 0
    finally:
        L.tmv_internal_random_fault(0, 0)


def test_mixed_stream_chunk_fits_device_memory():
    """a streamed mixed chunk's workspaces (both kinds'
    per-entry scratch and MSM workspaces, per host lane) are sized from the
    device memory free at the call (~20 KB per entry and lane: 3.5M+ entries
    on an idle 288 GB MI355X, so the bench's 1M mixed batch stays one chunk),
    smaller chunks on a smaller device instead of TMV_ERR_NOMEM."""
    from tendermint_amd import _native
    L = _native.lib()
    L.tmv_internal_mixed_stream_chunk.restype = ctypes.c_int64
    L.tmv_internal_mixed_stream_chunk.argtypes = [ctypes.c_uint64]
    gib = 1 << 30
    big = L.tmv_internal_mixed_stream_chunk(280 * gib)
    assert 3 << 20 <= big <= 1 << 22
    prev = 0
    for free in (1, 8, 16, 32, 64, 128, 280):
        c = L.tmv_internal_mixed_stream_chunk(free * gib)
        assert 65536 <= c <= 1 << 22 and c % 65536 == 0 and c >= prev
        prev = c
    c32 = L.tmv_internal_mixed_stream_chunk(32 * gib)
    assert 65536 < c32 < big // 4
