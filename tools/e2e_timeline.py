#!/usr/bin/env python3
"""Timeline of one host-buffer call from a `rocprofv3 --kernel-trace
--memory-copy-trace` run of tools/e2e_probe.py or tools/mixed_e2e.py (their
JSON line carries each call's CLOCK_MONOTONIC bounds, the clock rocprofv3
stamps records with).  Prints, relative to the call's start: the first copy,
the first and last kernel, the device's busy time (union of kernel
intervals), the idle gaps longer than --gap µs with the kernels on either
side, and per-kernel totals inside the call.

  python tools/e2e_timeline.py gpurun_out/X/tracecp_1 gpurun_out/X/tracecp_1.log [--call -1]
"""
import argparse
import collections
import csv
import glob
import json
import os


def _rows(d, suffix):
    out = []
    for p in glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True):
        with open(p) as f:
            out += list(csv.DictReader(f))
    return out


def _short(name):
    name = name.replace("void ", "").replace("tmv::", "")
    return name.split("(")[0][:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("log")
    ap.add_argument("--call", type=int, default=-1)
    ap.add_argument("--gap", type=float, default=30.0)
    a = ap.parse_args()
    line = None
    for ln in open(a.log):
        if ln.startswith("{") and "calls_monotonic_ns" in ln:
            line = json.loads(ln)
    calls = line["calls_monotonic_ns"]
    t0, t1 = calls[a.call]
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Queue_Id", ""))
          for r in _rows(a.trace_dir, "kernel_trace.csv")]
    cs = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Direction", r.get("Kind", "")))
          for r in _rows(a.trace_dir, "memory_copy_trace.csv")]
    ks = sorted(k for k in ks if k[1] > t0 and k[0] < t1)
    cs = sorted(c for c in cs if c[1] > t0 and c[0] < t1)
    us = lambda t: (t - t0) / 1e3  # noqa: E731
    res = {"call_ms": (t1 - t0) / 1e6, "kernels": len(ks), "copies": len(cs)}
    if cs:
        res["first_copy_start_us"] = us(cs[0][0])
        res["last_copy_end_us"] = us(max(c[1] for c in cs))
        by_dir = collections.defaultdict(float)
        for c in cs:
            by_dir[c[2]] += (c[1] - c[0]) / 1e3
        res["copy_busy_us_by_direction"] = {k: round(v, 1) for k, v in by_dir.items()}
    if ks:
        res["first_kernel_start_us"] = us(ks[0][0])
        res["last_kernel_end_us"] = us(max(k[1] for k in ks))
        busy, cur_s, cur_e, gaps = 0, ks[0][0], ks[0][1], []
        prev = ks[0]
        for k in ks[1:]:
            if k[0] > cur_e:
                busy += cur_e - cur_s
                if (k[0] - cur_e) / 1e3 >= a.gap:
                    gaps.append({"at_us": round(us(cur_e), 1), "gap_us": round((k[0] - cur_e) / 1e3, 1),
                                 "after": _short(prev[2]), "before": _short(k[2])})
                cur_s, cur_e = k[0], k[1]
            else:
                cur_e = max(cur_e, k[1])
            if k[1] >= prev[1]:
                prev = k
        busy += cur_e - cur_s
        res["kernel_busy_us"] = round(busy / 1e3, 1)
        res["gaps"] = gaps
        tot = collections.defaultdict(lambda: [0.0, 0])
        for k in ks:
            tot[_short(k[2])][0] += (k[1] - k[0]) / 1e3
            tot[_short(k[2])][1] += 1
        res["kernel_sum_us"] = {n: [round(v[0], 1), v[1]] for n, v in sorted(tot.items(), key=lambda x: -x[1][0])}
        res["queues"] = dict(collections.Counter(k[3] for k in ks))
        tail = [k for k in ks if k[0] >= max(kk[1] for kk in ks) - 6e6]
        res["last_6ms"] = [[round(us(k[0]), 1), round(us(k[1]), 1), _short(k[2]), k[3]] for k in tail]
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
