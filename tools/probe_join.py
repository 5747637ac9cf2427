"""Determinism probe: the located + sub-group check case 4 times in one process, vector vs oracle each time."""
import sys, numpy as np
sys.path.insert(0, '.'); sys.path.insert(0, 'oracle'); sys.path.insert(0, 'tests')
import os
os.environ["TMV_LOC_SUBCHECK"] = "1"; os.environ["TMV_LOCATE_MIN"] = "150000"
import oracle_c as C
from tendermint_amd import _native as N
from test_gpu_batch_equation import _located_case
ctx = N.Context(1)
b, sig, singles, pairs = _located_case(m=128)
ok_o, ref = C.ed25519_verify_packed(b.pk, sig, b.msg, b.off, threads=16)
for it in range(4):
    ctx.set_batch_options(group_log2=7, window_bits=6, seed=bytes(range(32)), stats=True)
    ctx.metrics_reset()
    ok, st = ctx.verify_batch_ex(N.TMV_KIND_ED25519, N.TMV_FLAG_BATCH_EQUATION, b.pk, sig, b.msg, b.off)
    met = ctx.metrics()
    bad = np.nonzero(st.astype(np.uint8) != ref)[0]
    print(it, "ok" if len(bad) == 0 and ok == ok_o else f"MISMATCH {len(bad)} {bad[:10].tolist()}", met, flush=True)
    if len(bad):
        break
