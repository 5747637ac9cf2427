"""GPU parity: libtmgpu.so (k_ed25519_verify on gfx950, through the C-ABI)
vs the CPU oracle and the committed golden vectors.  Bit-exact validity
vectors are required (integer work)."""
import hashlib

import numpy as np
import pytest

import oracle_c as C
from tendermint_amd.testing.factory import make_c2_batch, make_commit_batch

pytestmark = pytest.mark.gpu


def _pack(vs):
    return C.pack([(bytes.fromhex(v["pk"]), bytes.fromhex(v["msg"]), bytes.fromhex(v["sig"])) for v in vs])


def test_rfc8032(ctx, golden):
    for v in golden("ed25519_rfc8032.json")["vectors"]:
        assert ctx.ed25519_verify(bytes.fromhex(v["pk"]), bytes.fromhex(v["msg"]), bytes.fromhex(v["sig"]))


def test_golden_vectors(ctx, golden):
    vs = golden("ed25519_vectors.json")["vectors"]
    ok, vec = ctx.ed25519_verify_batch(*_pack(vs))
    assert [bool(x) for x in vec] == [v["valid"] for v in vs]
    assert ok is False


def test_zip215_small_order_matrix(ctx, golden):
    g = golden("zip215_small_order.json")
    msg = bytes.fromhex(g["msg"])
    ents = [(bytes.fromhex(a), msg, bytes.fromhex(r) + bytes(32)) for a, r in g["pairs_all_valid_with_S0"]]
    ok, vec = ctx.ed25519_verify_batch(*C.pack(ents))
    assert ok and vec.all() and len(vec) == 196


def test_c2_full_size_bit_exact(ctx, golden):
    g = golden("c2_expected.json")
    b = make_c2_batch()
    ok, vec = ctx.ed25519_verify_batch(b.pk, b.sig, b.msg, b.off)
    bits = np.packbits(vec.astype(np.uint8), bitorder="little").tobytes().hex()
    assert bits == g["valid_bits_hex"] and not ok
    assert int(vec.sum()) == 9950


def test_random_vs_oracle(ctx):
    b = make_c2_batch(3000, seed=99, edge_scale=5.0)
    ok, vec = ctx.ed25519_verify_batch(b.pk, b.sig, b.msg, b.off)
    ok_o, ref = C.ed25519_verify_packed(b.pk, b.sig, b.msg, b.off, threads=8)
    assert np.array_equal(vec, ref) and ok == ok_o


def test_all_valid_commit(ctx):
    b = make_commit_batch(150)
    ok, vec = ctx.ed25519_verify_batch(b.pk, b.sig, b.msg, b.off)
    assert ok and vec.all()


def test_empty_batch_false(ctx):
    ok, vec = ctx.ed25519_verify_batch(np.zeros(0, np.uint8), np.zeros(0, np.uint8), np.zeros(0, np.uint8),
                                       np.zeros(1, np.uint32))
    assert ok is False and len(vec) == 0


def test_single_verify_length_rules(ctx, golden):
    v = golden("ed25519_rfc8032.json")["vectors"][1]
    pk, m, s = bytes.fromhex(v["pk"]), bytes.fromhex(v["msg"]), bytes.fromhex(v["sig"])
    assert ctx.ed25519_verify(pk, m, s)
    assert not ctx.ed25519_verify(pk, m, s[:63])          # crypto/ed25519/ed25519.go:175-177
    assert not ctx.ed25519_verify(pk, m, s + b"\0")
    b = bytearray(s); b[7] ^= 1                            # crypto/ed25519/ed25519_test.go:25-29
    assert not ctx.ed25519_verify(pk, m, bytes(b))


def test_message_lengths_and_block_boundaries(ctx):
    """Messages whose R||A||M straddles SHA-512 block boundaries (0..300 B)."""
    from tendermint_amd.testing._openssl import Ed25519Signer
    ents = []
    for n in list(range(0, 70)) + [110, 111, 112, 113, 127, 128, 129, 175, 176, 177, 239, 240, 241, 300]:
        s = Ed25519Signer(hashlib.sha256(b"len %d" % n).digest())
        m = bytes((i * 7 + n) & 255 for i in range(n))
        ents.append((s.public_key, m, s.sign(m)))
    ok, vec = ctx.ed25519_verify_batch(*C.pack(ents))
    assert ok and vec.all()


def test_unaligned_device_path(ctx):
    """Odd-offset device pointers take the unaligned-load path."""
    import torch
    b = make_c2_batch(500, seed=5)
    dev = torch.device("cuda:0")
    raw_pk = torch.zeros(b.pk.size + 1, dtype=torch.uint8, device=dev)
    raw_sig = torch.zeros(b.sig.size + 1, dtype=torch.uint8, device=dev)
    raw_pk[1:] = torch.from_numpy(b.pk).to(dev)
    raw_sig[1:] = torch.from_numpy(b.sig).to(dev)
    d_msg = torch.from_numpy(b.msg).to(dev)
    d_off = torch.from_numpy(b.off.view(np.int32)).to(dev)
    out = torch.zeros(b.n, dtype=torch.uint8, device=dev)
    s = torch.cuda.Stream()
    ctx.ed25519_verify_batch_device(0, raw_pk.data_ptr() + 1, raw_sig.data_ptr() + 1, d_msg.data_ptr(),
                                    d_off.data_ptr(), b.n, out.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    _, ref = C.ed25519_verify_packed(b.pk, b.sig, b.msg, b.off, threads=4)
    assert np.array_equal(out.cpu().numpy(), ref)


@pytest.mark.parametrize("tiles", [1, 6], ids=["quad", "single"])
def test_both_kernels_c2(ctx, golden, tiles):
    """Per-entry verification picks its kernel by size: up to 49,152 entries
    the quad kernel (4 lanes per signature), above it the single-lane one.
    The C2 batch once (quad) and tiled 6x = 60k entries (single lane): every
    tile reproduces the committed C2 vector bit for bit."""
    from tendermint_amd import _native as N
    from tendermint_amd.testing.factory import Batch
    b1 = make_c2_batch()
    b = Batch.concat([b1] * tiles)
    _, st = ctx.verify_batch_ex(N.TMV_KIND_ED25519, N.TMV_FLAG_PER_ENTRY, b.pk, b.sig, b.msg, b.off)
    want = golden("c2_expected.json")["valid_bits_hex"]
    for t in range(tiles):
        v = (st[t * b1.n:(t + 1) * b1.n] == 1).astype(np.uint8)
        assert np.packbits(v, bitorder="little").tobytes().hex() == want, t


def test_random_failure_fails_the_call_not_the_vector(ctx, golden):
    """A batch-equation call whose weights key cannot be drawn (getrandom
    failing, injected through tmv_internal_random_fault) returns
    TMV_ERR_RANDOM before anything is launched, so the caller sees an error,
    never a vector; per-entry calls draw nothing and are unaffected; the
    next batch-equation call after the fault clears verifies normally
    (crypto/ed25519/ed25519.go:232: rand.Reader errors reach the caller)."""
    import ctypes
    import errno
    from tendermint_amd import _native as N
    L = N.lib()
    L.tmv_internal_random_fault.argtypes = [ctypes.c_int, ctypes.c_int]
    b = make_c2_batch()
    want = golden("c2_expected.json")["valid_bits_hex"]
    bits = lambda st: np.packbits((st == 1).astype(np.uint8), bitorder="little").tobytes().hex()  # noqa: E731
    try:
        L.tmv_internal_random_fault(errno.ENOSYS, -1)
        with pytest.raises(N.NativeError, match=r"\(-6\).*getrandom"):
            ctx.verify_batch_ex(N.TMV_KIND_ED25519, N.TMV_FLAG_BATCH_EQUATION, b.pk, b.sig, b.msg, b.off)
        _, st = ctx.verify_batch_ex(N.TMV_KIND_ED25519, N.TMV_FLAG_PER_ENTRY, b.pk, b.sig, b.msg, b.off)
        assert bits(st) == want
    finally:
        L.tmv_internal_random_fault(0, 0)
    _, st = ctx.verify_batch_ex(N.TMV_KIND_ED25519, N.TMV_FLAG_BATCH_EQUATION, b.pk, b.sig, b.msg, b.off)
    assert bits(st) == want
