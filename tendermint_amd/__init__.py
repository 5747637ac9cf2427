"""tendermint_amd — MI355X-native signature-verification engine for
Tendermint's commit/vote validation path (ed25519 ZIP-215 and sr25519 behind
crypto.BatchVerifier).  See DESIGN.md.

The compute path is libtmgpu.so (HIP kernels for gfx950 + C-ABI,
include/tmverify.h).  There is no CPU fallback in this package: if the native
library or a GPU is missing, the verifier raises.
"""
__version__ = "0.1.0"
