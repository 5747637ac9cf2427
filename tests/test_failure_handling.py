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
