"""Host side of device sign-bytes (CPU): the C++ encoder and the template
split (tmv_vote_template_encode) against the sign-bytes mirror, which is
pinned by the reference's KAT vectors (types/vote_test.go:81-179).  The
product library's host layer is exercised through libcommitcheck.so
(tests/native), which links the same tm_host_abi.cpp."""
import ctypes
import random

import pytest

import vote_cases as V
from commit_fixtures import CHECK_SO
from tendermint_amd import host as H
from tendermint_amd.types.canonical import Timestamp


@pytest.fixture(scope="module")
def hostlib():
    return ctypes.CDLL(CHECK_SO)


def test_cpp_encoder_kat(golden, hostlib):
    for v in golden("signbytes_vectors.json")["vectors"]:
        got = H.vote_sign_bytes(v["chain_id"], v["type"], v["height"], v["round"], None, tuple(v["timestamp"]),
                                lib=hostlib)
        assert got.hex() == v["want"]


def test_cpp_encoder_random(hostlib):
    rng = random.Random(41)
    for _ in range(400):
        t = V.random_template(rng)
        ts = V.random_ts(rng)
        got = H.vote_sign_bytes(t["chain_id"], t["vtype"], t["height"], t["round_"], V.host_block_id(t["block_id"]),
                                ts, lib=hostlib)
        assert got == V.expected(t, True, ts), t


def test_template_assembly(hostlib):
    """Every template x (with / without field 4) x edge timestamps assembles to
    the reference's sign-bytes."""
    rng = random.Random(42)
    for _ in range(200):
        t = V.random_template(rng)
        seg = V.segments(t, lib=hostlib)
        for ts in V.EDGE_TS[:6] + [V.random_ts(rng)]:
            for wb in (True, False):
                assert V.assemble(seg, wb, ts) == V.expected(t, wb, ts), (t, ts, wb)


def test_template_segments_shape(hostlib):
    """A nil BlockID gives an empty block segment; the chain segment is field 6."""
    from tendermint_amd.types.canonical import BlockID
    t = dict(chain_id="test_chain_id", vtype=2, height=3, round_=0, block_id=BlockID())
    head, block, chain = V.segments(t, lib=hostlib)
    assert head == b"\x08\x02\x11\x03" + b"\x00" * 7 and block == b"" and chain == b"\x32\x0dtest_chain_id"
    assert V.assemble((head, block, chain), True, (0, 0)) == V.expected(t, False, (0, 0))
    from tendermint_amd.types.canonical import vote_sign_bytes
    assert V.assemble((head, block, chain), False, (5, 6)) == vote_sign_bytes("test_chain_id", 2, 3, 0, None,
                                                                             Timestamp(5, 6))


@pytest.mark.parametrize("threshold", ["1", "1000000000"])
def test_commit_suite_both_message_paths(threshold):
    """The CPU commit suite with every batch on the device-template path
    (threshold 1) and every batch on host-encoded messages."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, TMV_DEVICE_SIGNBYTES_MIN=threshold)
    out = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-m", "not gpu", "-p", "no:cacheprovider",
                          os.path.join(root, "tests", "test_commit_verify.py")], env=env, cwd=root,
                         capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-2000:]
