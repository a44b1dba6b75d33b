#!/usr/bin/env python3
"""Per-dispatch table of a rocprofv3 --pmc run of placement_pmc.py: each decode dispatch's
duration (counter-collection timestamps) beside its counters.  usage: pmc_dispatch_table.py DIR..."""
import collections
import csv
import os
import sys

for d in sys.argv[1:]:
    rows = [r for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv")))
            if any(k in r["Kernel_Name"] for k in ("decode_tiles_kernel", "decode_rows_kernel",
                                                  "tiles_group_kernel"))]
    rows = [r for r in rows if not r["Kernel_Name"].split(">")[0].rstrip().endswith("true")]
    by = collections.OrderedDict()
    for r in rows:
        e = by.setdefault(r["Dispatch_Id"], collections.defaultdict(float))
        e[r["Counter_Name"]] += float(r["Counter_Value"])
        e["ms"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    print(os.path.basename(d.rstrip("/")))
    for i, c in enumerate(by.values()):
        print(f"  {i} {c['ms']:7.3f} ms  " + "  ".join(f"{k}={v:.4g}" for k, v in c.items() if k != "ms"))
