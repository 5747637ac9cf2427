#!/usr/bin/env python3
"""Per-kernel PMC counters of single launches (tools/launch_alone.py under
rocprofv3 --pmc, one pass; tools/profile_r05.sh alone_pmc): for each launch
size, the median over its launches (the first --skip dropped as warmup) of
each kernel's counters summed over that launch's dispatches, plus the
derived figures of tools/pmc_derived.py -- occupancy (mean resident waves
per SIMD), VALU issue share and the executed v_mad_i64_i32 fraction
(SQ_INSTS_VALU_INT64 x 64 lanes x the kernel's static v_mad share,
profiles/r05/isa_mix.json, over its GRBM_GUI_ACTIVE time at 2.4 GHz, against
the peak of bench._load_peak()).

  python tools/pmc_launch.py COUNTERS.csv --n 125000 [--isa profiles/r05/isa_mix.json] > profiles/r05/pmc_125k.json
"""
import gzip
import argparse
import csv
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))
import bench  # noqa: E402
from kernel_fracs import short  # noqa: E402

CLOCK_HZ = 2.4e9  # MI355X_MICROARCH.md: peak engine clock (GRBM_GUI_ACTIVE counts it per XCD)



def _open(path):  # a committed .csv.gz reads like the .csv
    return gzip.open(path, "rt") if path.endswith(".gz") else open(path)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--n", type=int, required=True)
    ap.add_argument("--skip", type=int, default=1)
    ap.add_argument("--isa", default=os.path.join(REPO, "profiles", "r05", "isa_mix.json"))
    a = ap.parse_args()
    grid = (-(-2 * a.n // 256) + -(-a.n // 256)) * 256  # k_prep_fused's grid marks a launch of n entries
    rows = sorted(csv.DictReader(_open(a.csv)), key=lambda r: (int(r["Start_Timestamp"]), r["Counter_Name"]))
    launches, cur = [], None
    for r in rows:
        nm = short(r["Kernel_Name"])
        if nm.startswith("__amd") or nm.startswith("at::"):
            continue
        if nm.startswith("k_prep") and r["Counter_Name"] == rows[0]["Counter_Name"]:
            cur = {} if int(r["Grid_Size"]) == grid else None
            if cur is not None:
                launches.append(cur)
        if cur is None:
            continue
        k = cur.setdefault(nm, {})
        k[r["Counter_Name"]] = k.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    launches = launches[a.skip:]
    if not launches:
        sys.exit(f"no launch of {a.n} entries in {a.csv}")
    isa = json.load(open(a.isa))["kernels"] if os.path.exists(a.isa) else {}
    peak = bench._load_peak()
    out = {"n": a.n, "launches": len(launches), "source": a.csv, "kernels": {},
           "note": "medians over the launches of each kernel's counters summed over its dispatches in the launch; "
                   "GRBM_GUI_ACTIVE sums the 8 XCDs (time = /8 / 2.4 GHz); SQ_* cycle counters in quad-cycles"}
    names = sorted({k for L in launches for k in L})
    for nm in names:
        cnt = {c: statistics.median(L.get(nm, {}).get(c, 0.0) for L in launches)
               for c in sorted({c for L in launches for c in L.get(nm, {})})}
        d = {"counters": {c: int(v) for c, v in cnt.items()}}
        cyc = cnt.get("GRBM_GUI_ACTIVE", 0) / 8
        if cyc:
            d["us"] = round(cyc / CLOCK_HZ * 1e6, 1)
            if "SQ_WAVE_CYCLES" in cnt:
                d["occupancy_waves_per_simd"] = round(cnt["SQ_WAVE_CYCLES"] * 4 / (cyc * 1024), 2)
            if "SQ_ACTIVE_INST_VALU" in cnt:
                d["valu_issue_util"] = round(cnt["SQ_ACTIVE_INST_VALU"] * 4 / (cyc * 1024), 3)
            share = (isa.get(nm) or {}).get("mad_share_of_int64")
            if share is not None and "SQ_INSTS_VALU_INT64" in cnt:
                d["executed_mad_frac"] = round(cnt["SQ_INSTS_VALU_INT64"] * 64 * share / (cyc / CLOCK_HZ) / peak, 4)
        out["kernels"][nm] = d
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
