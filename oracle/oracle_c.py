"""TEST INFRASTRUCTURE ONLY — ctypes loader for the C oracle (oracle/_build/liboracle.so).

Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as
the *checker*.  The product path (tendermint_amd) never imports this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _SO


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = ctypes.CDLL(_SO)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        L.oracle_ed25519_verify.argtypes = [u8p, u8p, ctypes.c_size_t, u8p]
        L.oracle_ed25519_verify_batch.argtypes = [u8p, u8p, u8p, ctypes.POINTER(ctypes.c_uint32),
                                                  ctypes.c_size_t, u8p, ctypes.c_int]
        L.oracle_sr25519_status_batch.argtypes = [u8p, u8p, u8p, ctypes.POINTER(ctypes.c_uint32),
                                                  ctypes.c_size_t, ctypes.POINTER(ctypes.c_int8), ctypes.c_int]
        L.oracle_sr25519_verify.argtypes = [u8p, u8p, ctypes.c_size_t, u8p]
        L.oracle_sr25519_add_check.argtypes = [u8p, u8p]
        L.oracle_sha512.argtypes = [u8p, ctypes.c_size_t, u8p]
        L.oracle_sc_reduce64.argtypes = [u8p, u8p]
        L.oracle_merlin_test.argtypes = [u8p]
        L.oracle_ge_decode_lax.argtypes = [u8p, u8p, u8p]
        L.oracle_ristretto_decode.argtypes = [u8p, u8p, u8p]
        _lib = L
    return _lib


def _p(a: np.ndarray, t=ctypes.c_uint8):
    return a.ctypes.data_as(ctypes.POINTER(t))


def _buf(b: bytes):
    a = np.frombuffer(b, dtype=np.uint8).copy() if len(b) else np.zeros(1, np.uint8)
    return a


def ed25519_verify(pk: bytes, msg: bytes, sig: bytes) -> bool:
    if len(sig) != 64 or len(pk) != 32:
        return False
    a, m, s = _buf(pk), _buf(msg), _buf(sig)
    return bool(lib().oracle_ed25519_verify(_p(a), _p(m), len(msg), _p(s)))


def ed25519_verify_packed(pk: np.ndarray, sig: np.ndarray, msg: np.ndarray, off: np.ndarray,
                          threads: int = 1):
    """Packed layout (see include/tmverify.h).  Returns (ok, uint8 vector)."""
    n = len(off) - 1
    out = np.zeros(max(n, 1), np.uint8)
    msg = msg if len(msg) else np.zeros(1, np.uint8)
    ok = lib().oracle_ed25519_verify_batch(_p(pk), _p(sig), _p(msg), _p(off, ctypes.c_uint32), n,
                                           _p(out), threads)
    return bool(ok), out[:n]


def ed25519_batch_verify_voi(pk: np.ndarray, sig: np.ndarray, msg: np.ndarray, off: np.ndarray,
                             threads: int = 1, batch: int = 1024, seed: int = 1):
    """voi-style batch verification (c/ed25519_batch_cpu.c): one random
    linear combination per `batch` entries, entry-by-entry on failure.
    Returns (ok, uint8 vector, batches whose equation failed)."""
    L = lib()
    if not getattr(L, "_batch_voi", False):
        L.oracle_ed25519_batch_verify_voi.argtypes = [ctypes.c_void_p] * 4 + [
            ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_uint64,
            ctypes.POINTER(ctypes.c_size_t)]
        L._batch_voi = True
    n = len(off) - 1
    out = np.zeros(max(n, 1), np.uint8)
    msg = msg if len(msg) else np.zeros(1, np.uint8)
    failed = ctypes.c_size_t(0)
    ok = L.oracle_ed25519_batch_verify_voi(pk.ctypes.data, sig.ctypes.data, msg.ctypes.data,
                                           np.ascontiguousarray(off, np.uint32).ctypes.data, n, out.ctypes.data,
                                           threads, batch, seed, ctypes.byref(failed))
    return bool(ok), out[:n], failed.value


class CommitCPU:
    """types.VerifyCommit's signature work for one commit on the CPU, one
    thread (c/ed25519_batch_cpu.c oracle_verify_commit_cpu: every vote's
    sign-bytes, then one voi-style batch): bench.py's C1 CPU baseline.
    Arrays are prepared once; __call__() verifies the commit again."""

    def __init__(self, head: bytes, chain_id: str, secs, nanos, pk: np.ndarray, sig: np.ndarray):
        L = lib()
        if not getattr(L, "_commit_cpu", False):
            L.oracle_verify_commit_cpu.restype = ctypes.c_int
            L.oracle_verify_commit_cpu.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_uint32,
                                                   ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                   ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                                   ctypes.c_uint64]
            L._commit_cpu = True
        self.L = L
        self.head, self.chain = head, chain_id.encode()
        self.secs = np.ascontiguousarray(secs, np.int64)
        self.nanos = np.ascontiguousarray(nanos, np.int32)
        self.pk, self.sig = np.ascontiguousarray(pk, np.uint8), np.ascontiguousarray(sig, np.uint8)
        self.n = len(self.secs)
        self.out = np.zeros(max(self.n, 1), np.uint8)
        self.seed = 1

    def __call__(self) -> bool:
        self.seed += 1
        return bool(self.L.oracle_verify_commit_cpu(self.head, len(self.head), self.chain, len(self.chain),
                                                    self.secs.ctypes.data, self.nanos.ctypes.data,
                                                    self.pk.ctypes.data, self.sig.ctypes.data, self.n,
                                                    self.out.ctypes.data, self.seed))


def sr25519_status_packed(pk, sig, msg, off, threads: int = 1) -> np.ndarray:
    n = len(off) - 1
    out = np.zeros(max(n, 1), np.int8)
    msg = msg if len(msg) else np.zeros(1, np.uint8)
    lib().oracle_sr25519_status_batch(_p(pk), _p(sig), _p(msg), _p(off, ctypes.c_uint32), n,
                                      _p(out, ctypes.c_int8), threads)
    return out[:n]


def sr25519_verify(pk: bytes, msg: bytes, sig: bytes) -> bool:
    if len(sig) != 64 or len(pk) != 32:
        return False
    a, m, s = _buf(pk), _buf(msg), _buf(sig)
    return bool(lib().oracle_sr25519_verify(_p(a), _p(m), len(msg), _p(s)))


def sha512(m: bytes) -> bytes:
    out = np.zeros(64, np.uint8)
    lib().oracle_sha512(_p(_buf(m)), len(m), _p(out))
    return out.tobytes()


def merlin_test_vector() -> bytes:
    out = np.zeros(32, np.uint8)
    lib().oracle_merlin_test(_p(out))
    return out.tobytes()


L_ORDER = 2**252 + 27742317777372353535851937790883648493


def ed25519_prechecks(pk: np.ndarray, sig: np.ndarray) -> np.ndarray:
    """Per entry: A and R decode (ZIP-215 lax) and S < l — the entries a
    random-linear-combination batch check includes (test infrastructure: the
    expected group verdicts follow from these and the validity vector)."""
    L = lib()
    n = len(pk) // 32
    out = np.zeros(n, bool)
    x, y = np.zeros(32, np.uint8), np.zeros(32, np.uint8)
    for i in range(n):
        a = np.ascontiguousarray(pk[32 * i:32 * i + 32])
        r = np.ascontiguousarray(sig[64 * i:64 * i + 32])
        s = int.from_bytes(sig[64 * i + 32:64 * i + 64].tobytes(), "little")
        out[i] = (s < L_ORDER and bool(L.oracle_ge_decode_lax(_p(a), _p(x), _p(y)))
                  and bool(L.oracle_ge_decode_lax(_p(r), _p(x), _p(y))))
    return out


def sr25519_prechecks(pk: np.ndarray, sig: np.ndarray) -> np.ndarray:
    """As ed25519_prechecks for sr25519: A and R Ristretto-decode, the
    schnorrkel marker is set and the cleared scalar is < l."""
    L = lib()
    n = len(pk) // 32
    out = np.zeros(n, bool)
    x, y = np.zeros(32, np.uint8), np.zeros(32, np.uint8)
    for i in range(n):
        a = np.ascontiguousarray(pk[32 * i:32 * i + 32])
        r = np.ascontiguousarray(sig[64 * i:64 * i + 32])
        sb = bytearray(sig[64 * i + 32:64 * i + 64].tobytes())
        marker = bool(sb[31] & 0x80)
        sb[31] &= 0x7F
        out[i] = (marker and int.from_bytes(bytes(sb), "little") < L_ORDER
                  and bool(L.oracle_ristretto_decode(_p(a), _p(x), _p(y)))
                  and bool(L.oracle_ristretto_decode(_p(r), _p(x), _p(y))))
    return out


def failing_groups(precheck: np.ndarray, valid: np.ndarray, m: int) -> int:
    """Groups of m consecutive entries that must fail the batch equation:
    those holding an entry that passes the pre-checks but is invalid."""
    bad = precheck & ~valid.astype(bool)
    n = len(bad)
    return int(sum(bad[g:g + m].any() for g in range(0, n, m)))


def pack(entries):
    """[(pk, msg, sig)] -> (pk[n*32], sig[n*64], msg[], off[n+1]) numpy arrays."""
    n = len(entries)
    pk = np.frombuffer(b"".join(e[0] for e in entries), np.uint8).copy() if n else np.zeros(0, np.uint8)
    sig = np.frombuffer(b"".join(e[2] for e in entries), np.uint8).copy() if n else np.zeros(0, np.uint8)
    msgs = [e[1] for e in entries]
    off = np.zeros(n + 1, np.uint32)
    if n:
        off[1:] = np.cumsum([len(m) for m in msgs])
    msg = np.frombuffer(b"".join(msgs), np.uint8).copy() if sum(len(m) for m in msgs) else np.zeros(0, np.uint8)
    return pk, sig, msg, off
