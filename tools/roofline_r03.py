#!/usr/bin/env python3
"""Dominant-kernel roofline inputs from a round-3 profile directory
(tools/profile_r03.sh) -> profiles/r03/dominant_kernel.json, read by
bench.py's roofline object:

  rocprof_alone   rocprofv3 --kernel-trace --stats of bench.py --inflight 1:
                  k_msm_accum<16>'s average dispatch with one launch at a time
  fetch_calibration  FETCH_SIZE of tools/fetchbench against its known byte
                  counts (stream / wpart-like runs of 160-B points / scattered
                  160-B points): the gfx950 correction per access pattern
  traffic         k_msm_accum's HBM bytes per launch at the bench's launch
                  size (PMC passes over tools/pmc_driver.py --per-launch 256):
                  FETCH_SIZE x the scattered-point correction + WRITE_SIZE
  executed        SQ_INSTS_VALU_INT64 lane-ops per launch

  python tools/roofline_r03.py gpurun_out/prof_r03 > profiles/r03/dominant_kernel.json
"""
import collections
import csv
import glob
import json
import os
import sys

KERNEL = "k_msm_accum<16>"
PMC_LAUNCHES = 4  # tools/pmc_driver.py --launches 2: 2 warm-up + 2


def _csv(d, pattern):
    f = sorted(glob.glob(os.path.join(d, "**", pattern), recursive=True))
    return list(csv.DictReader(open(f[0]))) if f else []


def _short(name):
    return name.split("(")[0].replace("void ", "").replace("tmv::", "").strip()


def counters(d, tag):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in _csv(os.path.join(d, tag), "*counter_collection.csv"):
        acc[_short(r["Kernel_Name"])][r["Counter_Name"]] += float(r["Counter_Value"])
    return acc


def main():
    d = sys.argv[1]
    out = {"source": d, "kernel": KERNEL}
    stats = {_short(r["Name"]): r for r in _csv(os.path.join(d, "trace_alone"), "*kernel_stats.csv")}
    if KERNEL in stats:
        r = stats[KERNEL]
        out["rocprof_alone"] = {"command": "bench.py --steps 20 --warmup 5 --inflight 1 --no-cpu-baseline --no-extras",
                                "avg_ms": round(float(r["AverageNs"]) / 1e6, 4), "dispatches": int(r["Calls"]),
                                "total_ms": round(float(r["TotalDurationNs"]) / 1e6, 3),
                                "file": "rocprof --stats (trace_alone)"}
    # FETCH_SIZE calibration: known bytes / counted bytes per kernel
    cal = {}
    known = {}
    log = os.path.join(d, "fetchcal.log")
    if os.path.exists(log):
        for line in open(log):
            if line.startswith("{"):
                known = json.loads(line)
    fc = counters(d, "fetchcal")
    for k in ("k_stream", "k_runs160", "k_gather160"):
        if k in fc and f"{k}_bytes" in known:
            counted = fc[k]["FETCH_SIZE"] * 1024
            want = known[f"{k}_bytes"] + (known.get("k_gather160_idx_bytes", 0) if k == "k_gather160" else 0)
            cal[k] = {"fetch_size_bytes": round(counted), "known_bytes": want, "factor": round(want / counted, 4)}
    out["fetch_calibration"] = cal
    f, w = counters(d, "fetch"), counters(d, "write")
    busy = counters(d, "busy")
    if KERNEL in f:
        fetch = f[KERNEL]["FETCH_SIZE"] * 1024 / PMC_LAUNCHES
        write = w.get(KERNEL, {}).get("WRITE_SIZE", 0.0) * 1024 / PMC_LAUNCHES
        fac = cal.get("k_gather160", {}).get("factor", 2.0)
        out["traffic_bytes_per_launch"] = round(fetch * fac + write)
        out["traffic_raw"] = {"fetch_size_bytes": round(fetch), "write_size_bytes": round(write),
                              "fetch_factor": fac}
        out["traffic_note"] = (f"PMC at the bench's launch size (256 x 10k signatures), {KERNEL}: FETCH_SIZE x {fac} "
                               "(tools/fetchbench.hip calibration of scattered 160-B point loads, the kernel's "
                               "Niels-point gathers) + WRITE_SIZE, per launch")
    if KERNEL in busy and busy[KERNEL].get("SQ_INSTS_VALU_INT64"):
        out["executed_int64_lane_ops_per_launch"] = round(busy[KERNEL]["SQ_INSTS_VALU_INT64"] * 64 / PMC_LAUNCHES)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
