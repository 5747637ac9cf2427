#!/usr/bin/env python3
"""Average duration of a kernel's primary dispatches in a rocprofv3
--kernel-trace csv, to compare with bench.py's live HIP-event timing
(roofline.dominant_kernel).  Batch-equation launches dispatch the bucket
kernels twice (the throughput pass, then the located fallback's pass over
the failing groups); per stream, in dispatch order, the first of each pair
is the primary one.

  python tools/trace_kernel_avg.py <kernel_trace.csv> [k_msm_accum] [pairs=2]
"""
import collections
import csv
import json
import sys


def main():
    path = sys.argv[1]
    name = sys.argv[2] if len(sys.argv) > 2 else "k_msm_accum"
    per = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    by_stream = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if name in r["Kernel_Name"]:
            by_stream[r["Stream_Id"]].append((int(r["Dispatch_Id"]),
                                              (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6))
    prim, other = [], []
    for v in by_stream.values():
        v.sort()
        for i, (_, ms) in enumerate(v):
            (prim if i % per == 0 else other).append(ms)
    out = {"kernel": name, "trace": path, "primary_dispatches": len(prim),
           "primary_avg_ms": round(sum(prim) / max(1, len(prim)), 4),
           "other_dispatches": len(other), "other_avg_ms": round(sum(other) / max(1, len(other)), 4)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
