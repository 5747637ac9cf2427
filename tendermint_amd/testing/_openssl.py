"""Minimal OpenSSL 3 (libcrypto) Ed25519 signer for synthetic inputs.

RFC 8032 deterministic signing — byte-identical to curve25519-voi
ed25519.Sign, which the reference uses (crypto/ed25519/ed25519.go:88-91).
Input generation only; never used to verify.
"""
from __future__ import annotations

import ctypes
import ctypes.util

_EVP_PKEY_ED25519 = 1087
_lib = None


def _load():
    global _lib
    if _lib is None:
        name = ctypes.util.find_library("crypto") or "libcrypto.so.3"
        L = ctypes.CDLL(name)
        L.EVP_PKEY_new_raw_private_key.restype = ctypes.c_void_p
        L.EVP_PKEY_new_raw_private_key.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t]
        L.EVP_PKEY_get_raw_public_key.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_size_t)]
        L.EVP_PKEY_free.argtypes = [ctypes.c_void_p]
        L.EVP_MD_CTX_new.restype = ctypes.c_void_p
        L.EVP_MD_CTX_free.argtypes = [ctypes.c_void_p]
        L.EVP_DigestSignInit.argtypes = [ctypes.c_void_p] * 5
        L.EVP_DigestSign.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_size_t),
                                     ctypes.c_char_p, ctypes.c_size_t]
        _lib = L
    return _lib


class Ed25519Signer:
    """A private key held as an EVP_PKEY (seed = 32 bytes)."""

    def __init__(self, seed: bytes):
        L = _load()
        self._L = L
        self._pk = L.EVP_PKEY_new_raw_private_key(_EVP_PKEY_ED25519, None, seed, 32)
        if not self._pk:
            raise RuntimeError("EVP_PKEY_new_raw_private_key failed")
        out = ctypes.create_string_buffer(32)
        n = ctypes.c_size_t(32)
        if L.EVP_PKEY_get_raw_public_key(self._pk, out, ctypes.byref(n)) != 1:
            raise RuntimeError("EVP_PKEY_get_raw_public_key failed")
        self.public_key = out.raw
        self._sig = ctypes.create_string_buffer(64)

    def sign(self, msg: bytes) -> bytes:
        L = self._L
        ctx = L.EVP_MD_CTX_new()
        try:
            if L.EVP_DigestSignInit(ctx, None, None, None, self._pk) != 1:
                raise RuntimeError("EVP_DigestSignInit failed")
            n = ctypes.c_size_t(64)
            if L.EVP_DigestSign(ctx, self._sig, ctypes.byref(n), msg, len(msg)) != 1:
                raise RuntimeError("EVP_DigestSign failed")
            return self._sig.raw
        finally:
            L.EVP_MD_CTX_free(ctx)

    def __del__(self):
        try:
            self._L.EVP_PKEY_free(self._pk)
        except Exception:
            pass
