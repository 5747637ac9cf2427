#!/usr/bin/env python3
"""Static 64-bit VALU instruction mix of a kernel (gfx950 ISA from hipcc -S):
the share of its 64-bit integer VALU instructions that are v_mad_i64_i32
(the field-multiply products) versus 64-bit adds / shifts of the carry
chains.  bench.py scales the PMC SQ_INSTS_VALU_INT64 rate by this share to
report the multiply-only fraction of the dominant kernel.

  python tools/isa_mix.py [kernel_prefix] > profiles/r02_close/isa_mix_accum.json
"""
import collections
import json
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "tendermint_amd", "csrc", "msm_kernels.hip")


def main():
    prefix = sys.argv[1] if len(sys.argv) > 1 else "_ZN3tmv11k_msm_accumILi16E"
    with tempfile.TemporaryDirectory() as d:
        asm = os.path.join(d, "k.s")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only",
                        "-S", "-o", asm, SRC], check=True, capture_output=True)
        lines = open(asm).read().split("\n")
    st = next(k for k, l in enumerate(lines) if l.startswith(prefix) and l.rstrip().endswith(":") or
              (l.startswith(prefix) and ":" in l and "@" in l))
    en = st
    while "s_endpgm" not in lines[en]:
        en += 1
    ops = [l.split()[0] for l in lines[st + 1:en] if l.strip() and not l.strip().startswith((".", ";"))
           and not l.strip().split()[0].endswith(":")]
    c = collections.Counter(ops)
    i64 = {k: v for k, v in c.items() if k.startswith("v_") and re.search(r"_(i64|u64|b64)", k)}
    mads = c.get("v_mad_i64_i32", 0)
    tot = sum(i64.values())
    print(json.dumps({"kernel": lines[st].split(":")[0], "source": "tendermint_amd/csrc/msm_kernels.hip (hipcc -O3 gfx950)",
                      "instructions": len(ops), "int64_ops": tot, "v_mad_i64_i32": mads,
                      "mad_share_of_int64": round(mads / tot, 4) if tot else None,
                      "int64_mix": dict(sorted(i64.items(), key=lambda x: -x[1]))}, indent=1))


if __name__ == "__main__":
    main()
