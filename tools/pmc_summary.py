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
    kernels = sorted(set(fetch) | set(write) | set(valu))
    per = {}
    tot_r = tot_w = 0.0
    for k in kernels:
        if not k.startswith("tmv::"):
            continue
        rd = 2 * fetch.get(k, {}).get("FETCH_SIZE", 0.0) * 1024 / launches
        wr = write.get(k, {}).get("WRITE_SIZE", 0.0) * 1024 / launches
        v = {c: x / launches for c, x in valu.get(k, {}).items()}
        b = {c: x / launches for c, x in busy.get(k, {}).items()}
        tot_r += rd
        tot_w += wr
        per[k] = {"hbm_read_bytes": round(rd), "hbm_write_bytes": round(wr), **{c: round(x) for c, x in v.items()},
                  **{c: round(x) for c, x in b.items()}}
    print(json.dumps({"launches": launches, "hbm_bytes_per_launch": round(tot_r + tot_w),
                      "hbm_read_bytes_per_launch": round(tot_r), "hbm_write_bytes_per_launch": round(tot_w),
                      "note": "FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE, KB units x 1024, per launch "
                              "of the profiled driver; SQ counters summed over dispatches / launches",
                      "kernels": per}, indent=1))


if __name__ == "__main__":
    main()
