#!/usr/bin/env python3
"""Per-kernel roofline fractions of single batch-equation launches (one
launch at a time, tools/launch_alone.py --stats), from committed profiles:

  * time: rocprofv3 --kernel-trace of the launches (median per launch of
    each kernel's dispatches, tools/launch_trace.py's grouping);
  * algorithmic work: bench.kernel_products (SURVEY 8(d)'s products: the
    decodes, bucket entries, running sums, Horner chains and fallback
    entries of that launch shape, with the launch's own failing-group and
    fallback counts from launch_alone --stats);
  * executed multiplies (optional): rocprofv3 --pmc SQ_INSTS_VALU_INT64 per
    dispatch x 64 lanes x the kernel's static v_mad_i64_i32 share
    (tools/isa_mix.py), summed per launch.

frac = products / kernel time / peak (<= 1 by construction: the products are
work the kernel must do); executed_mad_frac = executed v_mad_i64_i32 lane-ops
/ kernel time / peak (<= 1: each is one multiply-add issued).  The launch's
pipeline fractions divide the sums by the launch span.

  python tools/kernel_fracs.py --trace T.csv --alone A.jsonl [--pmc P.csv] [--isa profiles/r05/isa_mix.json] > out.json
"""
import gzip
import argparse
import csv
import json
import os
import re
import statistics
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402  (the product model and peak)

PRODUCT_KEY = {  # trace name prefix -> bench.kernel_products key (first match; the located Horner first)
    "k_prep_fused": "k_prep_fused", "k_msm_accum": "k_msm_accum", "k_msm_wpart": "k_msm_wpart",
    "k_msm_horner<false, false, 1>": "k_msm_horner_loc", "k_msm_horner<false, false, true>": "k_msm_horner_loc",
    "k_msm_horner": "k_msm_horner",  # k_msm_horner_helped too: its helper blocks' reductions are not priced
    "k_verify_quad": "fallback", "k_verify_quad_list": "fallback",
}



def _open(path):  # a committed .csv.gz reads like the .csv
    return gzip.open(path, "rt") if path.endswith(".gz") else open(path)


def short(name):
    return re.sub(r"\(.*", "", name).replace("void ", "").replace("tmv::", "")


def launches(rows, key_fn):
    """Split dispatches (sorted by start) into launches at each k_prep;
    returns {prep grid: [ {kernel: summed value} ... ]}."""
    out = defaultdict(list)
    cur = None
    for r in rows:
        nm = short(r["Kernel_Name"])
        if nm.startswith("__amd") or nm.startswith("at::"):
            continue
        if nm.startswith("k_prep"):
            cur = {"_grid": int(r.get("Grid_Size_X") or r.get("Grid_Size")), "_span": [None, None]}
            out[cur["_grid"]].append(cur)
        if cur is None:
            continue
        cur[nm] = cur.get(nm, 0.0) + key_fn(r)
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        cur["_span"][0] = s if cur["_span"][0] is None else min(cur["_span"][0], s)
        cur["_span"][1] = e if cur["_span"][1] is None else max(cur["_span"][1], e)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", required=True)
    ap.add_argument("--alone", required=True, help="launch_alone --stats JSON lines (n, groups_failed, ...)")
    ap.add_argument("--pmc", default="")
    ap.add_argument("--isa", default=os.path.join(REPO, "profiles", "r05", "isa_mix.json"))
    ap.add_argument("--skip", type=int, default=3)
    ap.add_argument("--src-digest", default="",
                    help="the profiled library's compiled source digest (tmv_version src=...); bench.py labels "
                         "executed fractions from a profile of another build as estimates")
    ap.add_argument("--locate-min", type=int, default=400_000,
                    help="the profiled build's TMV_LOCATE_MIN (groups of 128 and the located pass from it)")
    a = ap.parse_args()
    peak = bench._load_peak()
    rows = sorted((r for r in csv.DictReader(_open(a.trace)) if r["Kind"] == "KERNEL_DISPATCH"),
                  key=lambda r: int(r["Start_Timestamp"]))
    tl = launches(rows, lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    pl = {}
    if a.pmc:
        prow = [r for r in csv.DictReader(_open(a.pmc)) if r["Counter_Name"] == "SQ_INSTS_VALU_INT64"]
        prow.sort(key=lambda r: int(r["Start_Timestamp"]))
        pl = launches(prow, lambda r: float(r["Counter_Value"]))
    isa = json.load(open(a.isa))["kernels"] if os.path.exists(a.isa) else {}
    shapes = [json.loads(x) for x in open(a.alone) if x.startswith("{")]
    # prep grid = ceil(2n / 256) + ceil(n / 256) blocks x 256 threads
    grid_of = lambda n: (-(-2 * n // 256) + -(-n // 256)) * 256  # noqa: E731
    res = {"peak_mul_per_s": peak, "source": {"trace": a.trace, "pmc": a.pmc or None, "isa": a.isa,
                                               "src_digest": a.src_digest or None}, "launches": []}
    for sh in shapes:
        n = sh["n"]
        Ls = tl.get(grid_of(n), [])[a.skip:]
        if not Ls:
            continue
        m, c = bench.msm_shape(n, locate_min=a.locate_min)
        located = n >= a.locate_min
        prods = bench.kernel_products(n, m, c, sh.get("fallback_signatures", 0), sh.get("groups_failed", 0), located)
        names = sorted({k for L in Ls for k in L if not k.startswith("_")})
        span = statistics.median((L["_span"][1] - L["_span"][0]) / 1e3 for L in Ls)
        kern = {}
        tot_prod = tot_mad = 0.0
        for nm in names:
            us = statistics.median(L.get(nm, 0.0) for L in Ls)
            d = {"us": round(us, 1)}
            key = next((v for k, v in PRODUCT_KEY.items() if nm.startswith(k)), None)
            if key:  # (one fallback kernel per launch: whole groups, or the located entries' list)
                p = prods.get(key, 0)
                if p:
                    d["algorithmic_products"] = int(p)
                    d["frac"] = round(p / (us * 1e-6) / peak, 4)
                    tot_prod += p
            pls = pl.get(grid_of(n), [])[a.skip:]
            if pls and nm in isa:
                ops = statistics.median(L.get(nm, 0.0) for L in pls) * 64
                share = isa[nm]["mad_share_of_int64"] or 0
                d["int64_lane_ops"] = int(ops)
                d["mad_share_static"] = share
                d["executed_mad_frac"] = round(ops * share / (us * 1e-6) / peak, 4)
                tot_mad += ops * share
            kern[nm] = d
        entry = {"n": n, "group": m, "window_bits": c, "located": located,
                 "groups": sh.get("groups"), "groups_failed": sh.get("groups_failed"),
                 "fallback_signatures": sh.get("fallback_signatures"),
                 "launch_span_us": round(span, 1), "launch_alone_ms_events": sh.get("ms_median"),
                 "verifies_per_s": round(n / (span * 1e-6), 1), "kernels": kern,
                 "pipeline_algorithmic_frac": round(tot_prod / (span * 1e-6) / peak, 4)}
        if tot_mad:
            entry["pipeline_executed_mad_frac"] = round(tot_mad / (span * 1e-6) / peak, 4)
        res["launches"].append(entry)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
