#!/usr/bin/env python3
"""Dominant-kernel roofline inputs from a round-3 profile directory
(tools/profile_round_pmc.sh, round 3: profile_r03.sh) -> profiles/r03/dominant_kernel.json, read by
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


def primary_counters(d, tag, kernel):
    """Counter sums over the kernel's PRIMARY dispatches only: a batch-equation
    launch dispatches the bucket kernels twice (the throughput pass, then the
    located fallback's pass over the failing groups, same grid), so per queue
    in dispatch order the first of each pair is the primary one.  Returns
    (sums, primary dispatches)."""
    disp = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in _csv(os.path.join(d, tag), "*counter_collection.csv"):
        if _short(r["Kernel_Name"]) == kernel:
            disp[(r["Queue_Id"], int(r["Dispatch_Id"]))][r["Counter_Name"]] += float(r["Counter_Value"])
    by_q = collections.defaultdict(list)
    for (q, i) in disp:
        by_q[q].append(i)
    acc = collections.defaultdict(float)
    n = 0
    for q, ids in by_q.items():
        for k, i in enumerate(sorted(ids)):
            if k % 2 == 0:
                n += 1
                for c, v in disp[(q, i)].items():
                    acc[c] += v
    return acc, n


def primary_trace(d, tag, kernel, skip=5, take=20):
    """Durations of the kernel's primary dispatches in a --kernel-trace csv
    (first of each pair per stream, as above), in start order, bench warmup
    skipped: the same launches bench.py times live with HIP events."""
    rows = [r for r in _csv(os.path.join(d, tag), "*kernel_trace.csv") if _short(r["Kernel_Name"]) == kernel]
    by_s = collections.defaultdict(list)
    for r in rows:
        by_s[r.get("Stream_Id", r.get("Queue_Id"))].append(
            (int(r["Dispatch_Id"]), int(r["Start_Timestamp"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6))
    prim, loc = [], []
    for v in by_s.values():
        v.sort()
        for i, (_, t0, ms) in enumerate(v):
            (prim if i % 2 == 0 else loc).append((t0, ms))
    prim = [ms for _, ms in sorted(prim)][skip:skip + take]
    loc = [ms for _, ms in sorted(loc)][skip:skip + take]
    return prim, loc


def main():
    d = sys.argv[1]
    out = {"source": d, "kernel": KERNEL}
    stats = {_short(r["Name"]): r for r in _csv(os.path.join(d, "trace_alone"), "*kernel_stats.csv")}
    prim, loc = primary_trace(d, "trace_alone", KERNEL)
    if prim:
        r = stats.get(KERNEL, {})
        out["rocprof_alone"] = {"command": "bench.py --steps 20 --warmup 5 --inflight 1 --no-cpu-baseline --no-extras",
                                "avg_ms": round(sum(prim) / len(prim), 4), "dispatches": len(prim),
                                "located_pass_avg_ms": round(sum(loc) / max(1, len(loc)), 4),
                                "stats_all_dispatches": {"calls": int(r.get("Calls", 0)),
                                                         "avg_ms": round(float(r.get("AverageNs", 0)) / 1e6, 4)},
                                "note": "primary k_msm_accum dispatch of each of the 20 timed launches (kernel trace, "
                                        "first of each launch's pair; the second is the located pass over the "
                                        "failing groups); --stats averages both",
                                "file": "rocprof --kernel-trace (trace_alone)"}
    # the driver's command (4 launches in flight): the same primary
    # dispatches, against the live under-overlap figure of that traced run
    prim4, _ = primary_trace(d, "trace", KERNEL)
    if prim4:
        live = None
        log = os.path.join(d, "trace.log")
        if os.path.exists(log):
            for line in open(log):
                if line.startswith("{"):
                    live = json.loads(line).get("roofline", {}).get("under_overlap", {}).get("avg_launch_ms")
        out["rocprof_inflight4"] = {"command": "bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras",
                                    "avg_ms": round(sum(prim4) / len(prim4), 4), "dispatches": len(prim4),
                                    "live_under_overlap_ms": live,
                                    "note": "primary k_msm_accum dispatches of the timed launches with 4 in flight "
                                            "(stretched by sharing the chip) against the bench's own HIP-event "
                                            "figure of the same run"}
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
    f, nf = primary_counters(d, "fetch", KERNEL)
    w, _ = primary_counters(d, "write", KERNEL)
    busy, nb = primary_counters(d, "busy", KERNEL)
    if nf:
        fetch = f["FETCH_SIZE"] * 1024 / nf
        write = w.get("WRITE_SIZE", 0.0) * 1024 / nf
        fac = cal.get("k_gather160", {}).get("factor", 2.0)
        out["traffic_bytes_per_launch"] = round(fetch * fac + write)
        out["traffic_raw"] = {"fetch_size_bytes": round(fetch), "write_size_bytes": round(write),
                              "fetch_factor": fac, "primary_dispatches": nf}
        out["traffic_note"] = (f"PMC at the bench's launch size (256 x 10k signatures), {KERNEL}, primary dispatches "
                               f"only: FETCH_SIZE x {fac} (tools/fetchbench.hip calibration of scattered 160-B point "
                               "loads, the kernel's Niels-point gathers) + WRITE_SIZE, per launch")
    if nb and busy.get("SQ_INSTS_VALU_INT64"):
        out["executed_int64_lane_ops_per_launch"] = round(busy["SQ_INSTS_VALU_INT64"] * 64 / nb)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
