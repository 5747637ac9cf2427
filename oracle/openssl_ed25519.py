"""TEST INFRASTRUCTURE ONLY — independent cross-check for the oracle.

ctypes binding to the system OpenSSL 3 ``libcrypto`` Ed25519 (RFC 8032).
Signing is deterministic and byte-identical to voi ``ed25519.Sign`` for the
same seed, so it pins honest golden vectors.  Its verifier is the *strict*
(cofactorless, canonical-encoding) variant, so it agrees with ZIP-215 only on
honest and randomly corrupted inputs — never use it for edge cases.
"""
from __future__ import annotations

import ctypes
import ctypes.util

EVP_PKEY_ED25519 = 1087

_lib = None


def available() -> bool:
    return _load() is not None


def _load():
    global _lib
    if _lib is not None:
        return _lib
    name = ctypes.util.find_library("crypto")
    if not name:
        return None
    try:
        lib = ctypes.CDLL(name)
    except OSError:
        return None
    lib.EVP_PKEY_new_raw_private_key.restype = ctypes.c_void_p
    lib.EVP_PKEY_new_raw_private_key.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t]
    lib.EVP_PKEY_new_raw_public_key.restype = ctypes.c_void_p
    lib.EVP_PKEY_new_raw_public_key.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t]
    lib.EVP_PKEY_get_raw_public_key.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_size_t)]
    lib.EVP_PKEY_free.argtypes = [ctypes.c_void_p]
    lib.EVP_MD_CTX_new.restype = ctypes.c_void_p
    lib.EVP_MD_CTX_free.argtypes = [ctypes.c_void_p]
    lib.EVP_DigestSignInit.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    lib.EVP_DigestSign.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_size_t), ctypes.c_char_p, ctypes.c_size_t]
    lib.EVP_DigestVerifyInit.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    lib.EVP_DigestVerify.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t]
    _lib = lib
    return lib


def public_key(seed: bytes) -> bytes:
    lib = _load()
    pk = lib.EVP_PKEY_new_raw_private_key(EVP_PKEY_ED25519, None, seed, 32)
    out = ctypes.create_string_buffer(32)
    n = ctypes.c_size_t(32)
    assert lib.EVP_PKEY_get_raw_public_key(pk, out, ctypes.byref(n)) == 1
    lib.EVP_PKEY_free(pk)
    return out.raw


def sign(seed: bytes, msg: bytes) -> bytes:
    lib = _load()
    pk = lib.EVP_PKEY_new_raw_private_key(EVP_PKEY_ED25519, None, seed, 32)
    ctx = lib.EVP_MD_CTX_new()
    assert lib.EVP_DigestSignInit(ctx, None, None, None, pk) == 1
    out = ctypes.create_string_buffer(64)
    n = ctypes.c_size_t(64)
    assert lib.EVP_DigestSign(ctx, out, ctypes.byref(n), msg, len(msg)) == 1
    lib.EVP_MD_CTX_free(ctx)
    lib.EVP_PKEY_free(pk)
    return out.raw


def verify_strict(pub: bytes, msg: bytes, sig: bytes) -> bool:
    lib = _load()
    pk = lib.EVP_PKEY_new_raw_public_key(EVP_PKEY_ED25519, None, pub, 32)
    if not pk:
        return False
    ctx = lib.EVP_MD_CTX_new()
    ok = lib.EVP_DigestVerifyInit(ctx, None, None, None, pk) == 1
    ok = ok and lib.EVP_DigestVerify(ctx, sig, len(sig), msg, len(msg)) == 1
    lib.EVP_MD_CTX_free(ctx)
    lib.EVP_PKEY_free(pk)
    return bool(ok)
