#!/usr/bin/env python3
"""Add the executed-work block to a tools/pmc_summary.py json (in place):
SQ_INSTS_VALU / _INT64 / _INT32 per signature over the profiled launches
(tools/pmc_driver.py: batches_per_launch C2 batches of 10k per launch).

  python tools/pmc_executed.py profiles/r02/pmc_batch.json [batches_per_launch]
"""
import json
import sys


def main():
    path = sys.argv[1]
    bpl = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    d = json.load(open(path))
    sigs = bpl * 10_000
    k = d["kernels"].values()
    valu = sum(v.get("SQ_INSTS_VALU", 0) for v in k)
    i64 = sum(v.get("SQ_INSTS_VALU_INT64", 0) for v in k)
    i32 = sum(v.get("SQ_INSTS_VALU_INT32", 0) for v in k)
    d["batches_per_launch"] = bpl
    d["executed"] = {
        "valu_wave_instr_per_sig": round(valu / sigs, 1),
        "int64_lane_ops_per_sig": int(i64 * 64 / sigs),
        "int32_lane_ops_per_sig": int(i32 * 64 / sigs),
        "note": ("PMC over tools/pmc_driver.py (launches of %d C2 batches, batch equation incl. the fallback): "
                 "SQ_INSTS_VALU_INT64 counts 64-bit integer VALU wave-instructions (v_mad_i64_i32 = the "
                 "field-multiply products, plus 64-bit adds / shifts of the carry chains), x 64 lanes / "
                 "signatures. executed_frac in bench.py = verifies/s x int64_lane_ops_per_sig / peak "
                 "v_mad_i64_i32 rate: an upper bound on the share of the multiply peak the pipeline executes" % bpl),
    }
    json.dump(d, open(path, "w"), indent=1)
    print(path, d["executed"]["valu_wave_instr_per_sig"], d["executed"]["int64_lane_ops_per_sig"])


if __name__ == "__main__":
    main()
