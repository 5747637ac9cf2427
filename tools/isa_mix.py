#!/usr/bin/env python3
"""Static 64-bit VALU instruction mix of the pipeline's kernels (gfx950 ISA
from hipcc -S): per kernel, the share of its 64-bit integer VALU instructions
that are v_mad_i64_i32 (the field-multiply products) against the 64-bit
adds / shifts of the carry chains.  bench.py prices each kernel's PMC
SQ_INSTS_VALU_INT64 lane-ops by this share against the v_mad_i64_i32 peak
(roofline.pipeline.executed_mad_frac).  The share is static (instructions in
the code, not executed): exact for a kernel whose time is one loop body
(k_msm_accum), an estimate for kernels with several loops (k_prep_fused's
square-root chains and SHA-512 rounds).

  python tools/isa_mix.py > profiles/r06/isa_mix.json          # every kernel
  python tools/isa_mix.py accum > profiles/r05/isa_mix_accum.json  # one (old format)
"""
import collections
import json
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "tendermint_amd", "csrc")

# name -> (source, mangled-name prefix)
KERNELS = {
    "k_msm_accum<16>": ("msm_kernels.hip", "_ZN3tmv11k_msm_accumILi16E"),
    "k_msm_wpart": ("msm_kernels.hip", "_ZN3tmv11k_msm_wpartE"),
    "k_msm_wsum": ("msm_kernels.hip", "_ZN3tmv10k_msm_wsumE"),
    "k_msm_join_list": ("msm_kernels.hip", "_ZN3tmv15k_msm_join_listE"),
    "k_msm_horner<false, false, false>": ("msm_kernels.hip", "_ZN3tmv12k_msm_hornerILb0ELb0ELb0E"),
    "k_msm_horner<false, false, true>": ("msm_kernels.hip", "_ZN3tmv12k_msm_hornerILb0ELb0ELb1E"),
    "k_msm_horner_helped<false>": ("msm_kernels.hip", "_ZN3tmv19k_msm_horner_helpedILb0E"),
    "k_msm_sort<false, false, 64, false>": ("msm_kernels.hip", "_ZN3tmv10k_msm_sortILb0ELb0ELi64ELb0E"),
    "k_msm_sort<false, false, 64, true>": ("msm_kernels.hip", "_ZN3tmv10k_msm_sortILb0ELb0ELi64ELb1E"),
    "k_msm_sort<false, false, 256, false>": ("msm_kernels.hip", "_ZN3tmv10k_msm_sortILb0ELb0ELi256ELb0E"),
    "k_loc_search<false>": ("msm_kernels.hip", "_ZN3tmv12k_loc_searchILb0E"),
    "k_prep_fused<false>": ("verify_kernels.hip", "_ZN3tmv12k_prep_fusedILb0E"),
    "k_prep_fused<true>": ("verify_kernels.hip", "_ZN3tmv12k_prep_fusedILb1E"),
    "k_verify_quad<false, true>": ("verify_kernels.hip", "_ZN3tmv13k_verify_quadILb0ELb1E"),
    "k_verify_quad<false, false>": ("verify_kernels.hip", "_ZN3tmv13k_verify_quadILb0ELb0E"),
    "k_verify_quad_list<false>": ("verify_kernels.hip", "_ZN3tmv18k_verify_quad_listILb0E"),
    "k_gather": ("gather_kernels.hip", "_ZN3tmv8k_gatherE"),
}


def asm_of(src, d):
    out = os.path.join(d, src + ".s")
    if not os.path.exists(out):
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only",
                        "-S", "-o", out, os.path.join(CSRC, src)], check=True, capture_output=True)
    return open(out).read().split("\n")


def mix(lines, prefix):
    try:
        st = next(k for k, ln in enumerate(lines) if ln.startswith(prefix) and ln.split()[0].endswith(":"))
    except StopIteration:
        return None
    en = st + 1  # to the function's end label (a kernel may hold several s_endpgm)
    while not lines[en].startswith(".Lfunc_end"):
        en += 1
    ops = [ln.split()[0] for ln in lines[st + 1:en] if ln.strip() and not ln.strip().startswith((".", ";"))
           and not ln.strip().split()[0].endswith(":")]
    c = collections.Counter(ops)
    i64 = {k: v for k, v in c.items() if k.startswith("v_") and re.search(r"_(i64|u64|b64)", k)}
    mads = c.get("v_mad_i64_i32", 0)
    tot = sum(i64.values())
    return {"symbol": lines[st].split(":")[0], "instructions": len(ops), "int64_ops": tot, "v_mad_i64_i32": mads,
            "mad_share_of_int64": round(mads / tot, 4) if tot else None,
            "int64_mix": dict(sorted(i64.items(), key=lambda x: -x[1]))}


def main():
    only = sys.argv[1] if len(sys.argv) > 1 else None
    with tempfile.TemporaryDirectory() as d:
        if only == "accum":
            src, pre = KERNELS["k_msm_accum<16>"]
            m = mix(asm_of(src, d), pre)
            m["source"] = f"tendermint_amd/csrc/{src} (hipcc -O3 gfx950)"
            m["kernel"] = m.pop("symbol")
            print(json.dumps(m, indent=1))
            return
        out = {"note": "static counts in the gfx950 code object (hipcc -O3); mad_share_of_int64 = v_mad_i64_i32 / "
                       "all 64-bit integer VALU instructions of the kernel", "kernels": {}}
        for name, (src, pre) in KERNELS.items():
            m = mix(asm_of(src, d), pre)
            if m:
                m["source"] = f"tendermint_amd/csrc/{src}"
                out["kernels"][name] = m
        print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
