"""The production knobs' thresholds move entries between
paths; every setting must keep the oracle's vector: the batch equation never
(TMV_MSM_MIN=0), the key-cached batches never on the fused latency kernel
(TMV_CACHED_FUSED_MAX=0), the located fallback for every launch
(TMV_LOCATE_MIN=1); and a large host batch (4M signatures, chunked over both
lanes) whose honest entries must all pass.  Each setting runs in its own
process (the knobs are read once).  The A/B switches (knobs.h) exist only in
-DTMV_AB builds; tools/gpu_ab_so.sh runs the GPU tests on such builds."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

CODE = r"""
import sys, numpy as np
sys.path.insert(0, '.'); sys.path.insert(0, 'oracle'); sys.path.insert(0, 'tests')
import oracle_c as C
from tendermint_amd import _native as N
from tendermint_amd.testing.factory import make_c2_batch, make_sr25519_batch
from test_gpu_fuzz import _ed_corpus
ctx = N.Context(1)
b = _ed_corpus(4000, 123)
_, ref = C.ed25519_verify_packed(b.pk, b.sig, b.msg, b.off, threads=8)
for flags in (N.TMV_FLAG_PER_ENTRY, N.TMV_FLAG_BATCH_EQUATION, N.TMV_FLAG_KEY_CACHE | N.TMV_FLAG_BATCH_EQUATION):
    ok, st = ctx.verify_batch_ex(N.TMV_KIND_ED25519, flags, b.pk, b.sig, b.msg, b.off)
    assert np.array_equal(st.astype(np.uint8), ref), flags
s = make_sr25519_batch(1500, seed=124, bad_frac=0.05)
sref = C.sr25519_status_packed(s.pk, s.sig, s.msg, s.off, threads=8)
for flags in (N.TMV_FLAG_PER_ENTRY, N.TMV_FLAG_BATCH_EQUATION):
    ok, st = ctx.verify_batch_ex(N.TMV_KIND_SR25519, flags, s.pk, s.sig, s.msg, s.off)
    assert np.array_equal(st, sref), flags
print("ok")
"""


@pytest.mark.parametrize("env", [{}, {"TMV_MSM_MIN": "0"}, {"TMV_CACHED_FUSED_MAX": "0"}, {"TMV_LOCATE_MIN": "1"}],
                         ids=["default", "msm-min-0", "fused-max-0", "locate-min-1"])
def test_variant_matches_oracle(env):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, "-c", CODE], env=dict(os.environ, **env), cwd=root, capture_output=True,
                         text=True, timeout=600)
    assert out.returncode == 0, (env, out.stdout[-2000:], out.stderr[-3000:])
    assert "ok" in out.stdout


def test_large_host_batch_all_valid(ctx):
    """4M honest signatures (2,000 keys, tiled) through the host API: chunked
    over both lanes, key-merged with the cache and plain batch equation."""
    import numpy as np
    from tendermint_amd import _native as N
    from tendermint_amd.testing.factory import make_commit_batch
    b = make_commit_batch(2000).tile(4_000_000)
    for flags in (N.TMV_FLAG_KEY_CACHE, 0):
        ok, st = ctx.verify_batch_ex(N.TMV_KIND_ED25519, flags, b.pk, b.sig, b.msg, b.off)
        assert ok and int((st == 1).sum()) == b.n, flags
