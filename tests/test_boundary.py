"""The C-ABI library builds, loads without a GPU, and exports every
function include/tmverify.h declares (no compute calls here)."""
import ctypes
import os
import re

from tendermint_amd import _native


def _declared():
    src = "".join(open(p).read() for p in _native.HEADER_PATHS)
    return sorted(set(re.findall(r"\b(tmv_[a-z0-9_]+)\s*\(", src)))


def test_header_symbols_exported():
    assert os.path.exists(_native.LIB_PATH), "run __graft_entry__.build() first"
    lib = ctypes.CDLL(_native.LIB_PATH)
    declared = _declared()
    assert declared, "no declarations parsed"
    missing = [s for s in declared if not hasattr(lib, s)]
    assert not missing, f"declared but not exported: {missing}"
    assert sorted(_native.EXPORTS) == declared


def test_version_and_no_device_error():
    lib = _native.lib()
    assert b"gfx950" in lib.tmv_version()


def test_no_cpu_fallback_in_product_sources():
    """The product path must not reach the oracle (or any CPU verifier)."""
    root = os.path.dirname(_native.__file__)
    for dirpath, _, files in os.walk(root):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h")):
                txt = open(os.path.join(dirpath, f)).read()
                assert "oracle" not in re.sub(r"(#|//).*", "", txt).lower() or f == "_native.py", f
