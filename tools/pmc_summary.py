#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes of tools/pmc_driver.py into per-launch
figures: HBM bytes (FETCH_SIZE doubled — on gfx950 it reports half the
bytes of wide coalesced reads, MI355X_MICROARCH.md §HBM — plus WRITE_SIZE),
per-kernel shares, VALU instruction and cycle counters.

  python tools/pmc_summary.py gpurun_out/prof_<tag> <launches> > profiles/.../pmc.json
"""
import collections
import csv
import glob
import json
import os
import sys


def load(d, tag):
    f = glob.glob(os.path.join(d, tag, "*counter_collection.csv"))
    if not f:
        return {}
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f[0])):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        acc[name][r["Counter_Name"]] += float(r["Counter_Value"])
    return acc


def main():
    d, launches = sys.argv[1], int(sys.argv[2])
    fetch, write, valu, busy = (load(d, t) for t in ("fetch", "write", "valu", "busy"))
    # FETCH_SIZE calibration of tools/fetchbench.hip (profile_r03.sh's fetchcal
    # pass), when present: k_msm_wpart's runs of 160-B points and k_msm_accum's
    # scattered 160-B point gathers get their measured factors; the rest keep
    # the guide's x2 for coalesced reads
    cal = {}
    fc, known = load(d, "fetchcal"), {}
    log = os.path.join(d, "fetchcal.log")
    if os.path.exists(log):
        for line in open(log):
            if line.startswith("{"):
                known = json.loads(line)
    for k, extra in (("k_runs160", 0), ("k_gather160", known.get("k_gather160_idx_bytes", 0))):
        got = fc.get("tmv::" + k, fc.get(k, {})).get("FETCH_SIZE", 0.0) * 1024
        if got and f"{k}_bytes" in known:
            cal[k] = (known[f"{k}_bytes"] + extra) / got
    factor = lambda name: (cal.get("k_runs160", 2.0) if "k_msm_wpart" in name else  # noqa: E731
                           cal.get("k_gather160", 2.0) if "k_msm_accum" in name else 2.0)
    kernels = sorted(set(fetch) | set(write) | set(valu))
    per = {}
    tot_r = tot_w = 0.0
    for k in kernels:
        if not k.startswith("tmv::"):
            continue
        rd = factor(k) * fetch.get(k, {}).get("FETCH_SIZE", 0.0) * 1024 / launches
        wr = write.get(k, {}).get("WRITE_SIZE", 0.0) * 1024 / launches
        v = {c: x / launches for c, x in valu.get(k, {}).items()}
        b = {c: x / launches for c, x in busy.get(k, {}).items()}
        tot_r += rd
        tot_w += wr
        per[k] = {"hbm_read_bytes": round(rd), "hbm_write_bytes": round(wr), **{c: round(x) for c, x in v.items()},
                  **{c: round(x) for c, x in b.items()}}
    print(json.dumps({"launches": launches, "hbm_bytes_per_launch": round(tot_r + tot_w),
                      "hbm_read_bytes_per_launch": round(tot_r), "hbm_write_bytes_per_launch": round(tot_w),
                      "note": "FETCH_SIZE x factor + WRITE_SIZE, KB units x 1024, per launch of the profiled "
                              "driver; factor = the guide's x2 gfx950 correction for coalesced reads, or the "
                              "tools/fetchbench.hip calibration for k_msm_wpart (runs of 160-B points) and "
                              "k_msm_accum (scattered 160-B gathers) when the profile holds it; SQ counters summed "
                              "over dispatches / launches",
                      "fetch_factors": {"k_msm_wpart": round(cal.get("k_runs160", 2.0), 4),
                                        "k_msm_accum": round(cal.get("k_gather160", 2.0), 4), "other": 2.0},
                      "kernels": per}, indent=1))


if __name__ == "__main__":
    main()
