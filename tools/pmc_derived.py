#!/usr/bin/env python3
"""Derived per-kernel figures from a tools/pmc_summary.py json (in place):
  kernel_cycles      = GRBM_GUI_ACTIVE / 8           (rocprofv3 sums the 8 XCDs)
  occupancy          = SQ_WAVE_CYCLES x 4 / (kernel_cycles x 1024 SIMDs)
                       mean resident waves per SIMD (SQ_* count quad-cycles)
  valu_issue_util    = SQ_ACTIVE_INST_VALU x 4 / (kernel_cycles x 1024)
                       share of SIMD cycles issuing VALU work
  valu_per_wave_cyc  = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES (one wave's VALU share)
MI355X_MICROARCH.md: SQ_WAVE_CYCLES / SQ_ACTIVE_INST_* count quad-cycles;
GRBM_GUI_ACTIVE is the sum over the 8 XCDs.  Dispatches run one at a time
under --pmc, so the figures are per kernel, alone on the chip.

  python tools/pmc_derived.py profiles/r01_msm/pmc_batch.json [...]
"""
import json
import sys

SIMDS = 256 * 4

for path in sys.argv[1:]:
    d = json.load(open(path))
    for name, k in d["kernels"].items():
        g = k.get("GRBM_GUI_ACTIVE")
        if not g:
            continue
        cyc = g / 8.0
        k["derived"] = {
            "kernel_cycles": round(cyc),
            "occupancy_waves_per_simd": round(k.get("SQ_WAVE_CYCLES", 0) * 4 / (cyc * SIMDS), 3),
            "valu_issue_util": round(k.get("SQ_ACTIVE_INST_VALU", 0) * 4 / (cyc * SIMDS), 3),
            "valu_share_of_wave_cycles": round(k.get("SQ_ACTIVE_INST_VALU", 0) / max(1, k.get("SQ_WAVE_CYCLES", 1)), 3),
        }
    d["derived_note"] = ("occupancy = SQ_WAVE_CYCLES*4/(GRBM_GUI_ACTIVE/8*1024); valu_issue_util = "
                         "SQ_ACTIVE_INST_VALU*4/(GRBM_GUI_ACTIVE/8*1024); SQ counters in quad-cycles, GRBM summed "
                         "over 8 XCDs (MI355X_MICROARCH.md)")
    json.dump(d, open(path, "w"), indent=1)
    for name, k in sorted(d["kernels"].items(), key=lambda x: -x[1].get("SQ_INSTS_VALU", 0)):
        if "derived" in k:
            print(f"{path.split('/')[-1]:22s} {name:36s} occ {k['derived']['occupancy_waves_per_simd']:5.2f}  "
                  f"valu {k['derived']['valu_issue_util']:5.2f}")
