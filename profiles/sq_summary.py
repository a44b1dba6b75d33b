#!/usr/bin/env python3
"""Summarise an SQ counter pass (profiles/run_r03k.sh) per fast kernel: per-launch counter
means and the derived LDS picture.  SQ_* counters are summed over the chip's CUs and
GRBM_GUI_ACTIVE over its 8 XCDs, so per-CU LDS occupancy = SQ_LDS_IDX_ACTIVE / 256 over the
kernel's cycles (GRBM_GUI_ACTIVE / 8).
usage: sq_summary.py <out.json> <run_counter_collection.csv>..."""
import collections
import csv
import json
import os
import sys

KERNELS = ("tiles_group_kernel", "tiles_rowcrc", "rows_group_kernel", "rows_xpose_kernel",
           "decode_rows_kernel")


def summarise(path, cus=256, xcds=8):
    sums = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.Counter()
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        if not any(x in k for x in KERNELS):
            continue
        sums[k][r["Counter_Name"]] += float(r["Counter_Value"])
        n[(k, r["Counter_Name"])] += 1
    out = {}
    for k, d in sums.items():
        m = {c: v / n[(k, c)] for c, v in d.items()}
        cyc = m.get("GRBM_GUI_ACTIVE", 0) / xcds
        e = {"per_launch": m, "launches": n[(k, "SQ_INSTS_LDS")]}
        if cyc and m.get("SQ_LDS_IDX_ACTIVE"):
            e["kernel_cycles_per_xcd"] = cyc
            e["lds_busy_frac_per_cu"] = m["SQ_LDS_IDX_ACTIVE"] / cus / cyc
            e["bank_conflict_frac_of_lds_cycles"] = m["SQ_LDS_BANK_CONFLICT"] / m["SQ_LDS_IDX_ACTIVE"]
            e["valu_insts_per_lds_inst"] = m["SQ_INSTS_VALU"] / m["SQ_INSTS_LDS"]
        out[k] = e
    return out


if __name__ == "__main__":
    res = {os.path.basename(os.path.dirname(p)): summarise(p) for p in sys.argv[2:]}
    json.dump(res, open(sys.argv[1], "w"), indent=1)
    for run, ks in res.items():
        for k, e in ks.items():
            print(run, k[:70], {x: round(e[x], 3) for x in e if x.endswith("frac") or
                                x.endswith("frac_per_cu") or x.endswith("lds_inst")})
