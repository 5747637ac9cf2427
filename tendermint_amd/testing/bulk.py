"""Bulk input generation for chain-sized workloads (BASELINE C3 / C4: 1-2 M
commit signatures): commit-vote messages and RFC 8032 signatures built in
native code (_build/libtmfactory.so: OpenSSL 3 on a thread pool), so a
10,000-header chain is generated in seconds instead of minutes.  The bytes
are the ones the per-signature path (factory.commit_vote_message +
_openssl.Ed25519Signer) produces (tests/test_factory.py): RFC 8032 signing
is deterministic, and the factory's own signer is pinned to OpenSSL's.  Input generation
only; never used to verify.
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Sequence, Tuple

import numpy as np

from ..types.canonical import PRECOMMIT_TYPE, canonical_vote_head
from .sr25519_factory import _load as _load_factory

_ready = False


def _lib():
    global _ready
    L = _load_factory()
    if not _ready:
        L.tmf_vote_messages.restype = ctypes.c_size_t
        L.tmf_vote_messages.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_uint32,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                        ctypes.c_void_p]
        L.tmf_ed25519_sign_fast.restype = ctypes.c_int
        L.tmf_ed25519_sign_fast.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int]
        L.tmf_ed25519_sign_many.restype = ctypes.c_int
        L.tmf_ed25519_sign_many.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_int]
        _ready = True
    return L


def threads() -> int:
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def commit_vote_head(height: int, round_: int, block_id) -> bytes:
    """CanonicalVote fields before the timestamp of a precommit for block_id."""
    return canonical_vote_head(PRECOMMIT_TYPE, height, round_, block_id)


def vote_messages(head: bytes, chain_id: str, secs: Sequence[int], nanos: Sequence[int]
                  ) -> Tuple[np.ndarray, np.ndarray]:
    """Sign-bytes of the votes of one commit (all fields but the timestamp
    shared): (messages concatenated, n + 1 offsets)."""
    s = np.ascontiguousarray(secs, np.int64)
    ns = np.ascontiguousarray(nanos, np.int32)
    n = len(s)
    chain = chain_id.encode()
    out = np.empty(n * (len(head) + len(chain) + 48), np.uint8)
    off = np.empty(n + 1, np.uint32)
    total = _lib().tmf_vote_messages(head, len(head), chain, len(chain), s.ctypes.data, ns.ctypes.data, n,
                                     out.ctypes.data, off.ctypes.data)
    return out[:total], off


def public_keys(seeds: List[bytes]) -> List[bytes]:
    """Ed25519 public keys of 32-byte seeds."""
    if not seeds:
        return []
    sd = b"".join(seeds)
    pk = np.empty(32 * len(seeds), np.uint8)
    z = np.zeros(1, np.uint32)
    rc = _lib().tmf_ed25519_sign_many(sd, len(seeds), z.ctypes.data, z.ctypes.data, z.ctypes.data, 0,
                                      pk.ctypes.data, pk.ctypes.data, 1)
    if rc != 0:
        raise RuntimeError("tmf_ed25519_sign_many failed")
    raw = pk.tobytes()
    return [raw[32 * i:32 * i + 32] for i in range(len(seeds))]


def sign_many(seeds: List[bytes], key_idx: np.ndarray, msg: np.ndarray, off: np.ndarray,
              openssl: bool = False) -> np.ndarray:
    """Signature of message i by seeds[key_idx[i]], n x 64 bytes: the
    factory's own RFC 8032 signer, or OpenSSL's (openssl=True; the same
    bytes, several times slower)."""
    ki = np.ascontiguousarray(key_idx, np.uint32)
    m = np.ascontiguousarray(msg, np.uint8)
    o = np.ascontiguousarray(off, np.uint32)
    n = len(ki)
    sig = np.empty(64 * max(n, 1), np.uint8)
    if n:
        if openssl:
            rc = _lib().tmf_ed25519_sign_many(b"".join(seeds), len(seeds), ki.ctypes.data, m.ctypes.data,
                                              o.ctypes.data, n, sig.ctypes.data, None, threads())
        else:
            rc = _lib().tmf_ed25519_sign_fast(b"".join(seeds), len(seeds), ki.ctypes.data, m.ctypes.data,
                                              o.ctypes.data, n, sig.ctypes.data, threads())
        if rc != 0:
            raise RuntimeError("tmf_ed25519_sign_many failed")
    return sig[:64 * n]
