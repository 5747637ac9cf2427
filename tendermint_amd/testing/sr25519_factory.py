"""sr25519 key generation / signing for synthetic inputs (ctypes over
_build/libtmfactory.so, built from tendermint_amd/testing/csrc/factory.cpp).

Keys follow GenPrivKeyFromSecret (crypto/sr25519/privkey.go:157-170:
mini secret = SHA-256(secret)).  Input generation only.
"""
from __future__ import annotations

import ctypes
import hashlib
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(os.path.dirname(_HERE), "_build", "libtmfactory.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", os.path.join(_HERE, "csrc")], check=True)


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = ctypes.CDLL(_SO)
        L.tmf_sr25519_public_key.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
        L.tmf_sr25519_sign.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p,
                                       ctypes.c_size_t, ctypes.c_char_p]
        _lib = L
    return _lib


def mini_from_secret(secret: bytes) -> bytes:
    return hashlib.sha256(secret).digest()


class Sr25519Signer:
    def __init__(self, mini: bytes):
        self.mini = mini
        out = ctypes.create_string_buffer(32)
        _load().tmf_sr25519_public_key(mini, out)
        self.public_key = out.raw

    def sign(self, msg: bytes, nonce_seed: bytes = b"") -> bytes:
        out = ctypes.create_string_buffer(64)
        _load().tmf_sr25519_sign(self.mini, msg, len(msg), nonce_seed, len(nonce_seed), out)
        return out.raw
