#!/usr/bin/env python3
"""Per-launch breakdown of a rocprofv3 --kernel-trace of tools/launch_alone.py.

A launch starts at its k_prep* dispatch; every later dispatch up to the next
k_prep belongs to it.  Launches are grouped by the prep kernel's grid size
(one group per --n), the first `--skip` launches of a group (warmup) dropped.
Prints, per group: the median launch span (first start to last end), the sum
of kernel time, the idle gaps between dispatches, and each kernel's median
time per launch (dispatches of one name inside a launch summed).

  python tools/launch_trace.py gpurun_out/NAME/trace_K/run_kernel_trace.csv [--skip 3] [--csv out.csv]
"""
import gzip
import argparse
import csv
import re
import statistics
from collections import defaultdict



def _open(path):  # a committed .csv.gz reads like the .csv
    return gzip.open(path, "rt") if path.endswith(".gz") else open(path)


def short(name: str) -> str:
    name = re.sub(r"\(.*", "", name).replace("void ", "").replace("tmv::", "")
    return name


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--skip", type=int, default=3)
    ap.add_argument("--csv", default="")
    a = ap.parse_args()
    rows = [r for r in csv.DictReader(_open(a.trace)) if r["Kind"] == "KERNEL_DISPATCH"]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    launches = []
    for r in rows:
        nm = short(r["Kernel_Name"])
        if nm.startswith("__amd") or nm.startswith("at::"):
            continue
        if nm.startswith("k_prep"):
            launches.append({"grid": int(r["Grid_Size_X"]), "k": []})
        if launches:
            launches[-1]["k"].append((nm, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    groups = defaultdict(list)
    for L in launches:
        groups[L["grid"]].append(L)
    out_rows = []
    for grid, Ls in groups.items():
        Ls = Ls[a.skip:] or Ls
        span = statistics.median((L["k"][-1][2] - L["k"][0][1]) / 1e3 for L in Ls)
        busy = statistics.median(sum(e - s for _, s, e in L["k"]) / 1e3 for L in Ls)
        per = defaultdict(list)
        for L in Ls:
            acc = defaultdict(float)
            for nm, s, e in L["k"]:
                acc[nm] += (e - s) / 1e3
            for nm, v in acc.items():
                per[nm].append(v)
        print(f"prep grid {grid}: {len(Ls)} launches, span {span:.1f} us, kernels {busy:.1f} us, "
              f"gaps {span - busy:.1f} us")
        for nm, v in sorted(per.items(), key=lambda kv: -statistics.median(kv[1])):
            med = statistics.median(v)
            print(f"  {nm[:64]:64s} {med:9.1f} us  (x{len(v)})")
            out_rows.append({"prep_grid": grid, "kernel": nm, "median_us": round(med, 1), "launches": len(v)})
        out_rows.append({"prep_grid": grid, "kernel": "(launch span)", "median_us": round(span, 1),
                         "launches": len(Ls)})
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=["prep_grid", "kernel", "median_us", "launches"])
            w.writeheader()
            w.writerows(out_rows)


if __name__ == "__main__":
    main()
