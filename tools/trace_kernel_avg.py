#!/usr/bin/env python3
"""Average duration of a kernel's primary dispatches in a rocprofv3
--kernel-trace csv, to compare with bench.py's live HIP-event timing
(roofline.dominant_kernel).  Batch-equation launches dispatch the bucket
kernels twice (the throughput pass, then the located fallback's pass over
the failing groups); only dispatches of the largest grid (the bench's
launches, not the extras' smaller calls) count, and per stream, in dispatch
order, the first of each pair is the primary one.

  python tools/trace_kernel_avg.py <kernel_trace.csv> [k_msm_accum] [pairs=2] [skip] [take]

skip / take: of the primary dispatches in start-time order, drop the first
`skip` (bench warmup) and keep the next `take` (the timed steps), so the
average covers the same launches as bench.py's live HIP-event timing.
"""
import collections
import csv
import gzip
import json
import sys


def main():
    path = sys.argv[1]
    name = sys.argv[2] if len(sys.argv) > 2 else "k_msm_accum"
    per = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    skip = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    take = int(sys.argv[5]) if len(sys.argv) > 5 else 0
    f = gzip.open(path, "rt") if path.endswith(".gz") else open(path)
    rows = [r for r in csv.DictReader(f) if name in r["Kernel_Name"]]
    grid = max(int(r["Grid_Size_X"]) for r in rows)
    by_stream = collections.defaultdict(list)
    for r in rows:
        if int(r["Grid_Size_X"]) == grid:
            by_stream[r["Stream_Id"]].append((int(r["Dispatch_Id"]), int(r["Start_Timestamp"]),
                                              (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6))
    prim, other = [], []
    for v in by_stream.values():
        v.sort()
        for i, (_, t0, ms) in enumerate(v):
            (prim if i % per == 0 else other).append((t0, ms))
    prim = [ms for _, ms in sorted(prim)]
    other = [ms for _, ms in other]
    if skip or take:
        prim = prim[skip:skip + take if take else None]
    out = {"kernel": name, "trace": path, "grid": grid, "primary_dispatches": len(prim),
           "primary_avg_ms": round(sum(prim) / max(1, len(prim)), 4),
           "other_dispatches": len(other), "other_avg_ms": round(sum(other) / max(1, len(other)), 4)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
