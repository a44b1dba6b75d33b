#!/usr/bin/env python3
"""Where a kernel's waves spend their cycles, from one SQ pass (profiles/run_r03s.sh):
SQ_WAIT_ANY (parked on s_waitcnt / barrier) + SQ_WAIT_INST_ANY (issue stalls) +
SQ_ACTIVE_INST_ANY (issuing) = SQ_WAVE_CYCLES (MI355X_MICROARCH.md, SQ table; all in
quad-cycles), and the VMEM / LDS / VALU issue shares.  Per launch, per fast kernel.
usage: wait_summary.py <out.json> <run_counter_collection.csv>..."""
import collections
import csv
import json
import os
import sys

KERNELS = ("tiles_group_kernel", "tiles_rowcrc", "rows_group_kernel", "rows_xpose_kernel",
           "decode_rows_kernel")

res = {}
for path in sys.argv[2:]:
    sums = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.Counter()
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        if any(x in k for x in KERNELS):
            sums[k][r["Counter_Name"]] += float(r["Counter_Value"])
            n[(k, r["Counter_Name"])] += 1
    run = os.path.basename(os.path.dirname(path))
    for k, d in sums.items():
        m = {c: v / n[(k, c)] for c, v in d.items()}
        w = m.get("SQ_WAVE_CYCLES", 0)
        if not w:
            continue
        e = {c: round(m[c] / w, 4) for c in m if c.startswith("SQ_") and c != "SQ_WAVE_CYCLES"}
        e["kernel_ms_at_2.4GHz"] = round(m.get("GRBM_GUI_ACTIVE", 0) / 8 / 2.4e6, 2)
        res[f"{run}: {k}"] = e
        print(run, k[:60], e)
json.dump(res, open(sys.argv[1], "w"), indent=1)
