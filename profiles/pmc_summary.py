#!/usr/bin/env python3
"""Summarise rocprofv3 output for one config into profiles/<round>/<config>_summary.json.

HBM bytes per launch of the dominant kernel (the decode scatter kernel), corrected as
/opt/skills/guides/MI355X_MICROARCH.md §HBM prescribes for gfx950:
  FETCH_SIZE (KiB) reads exactly half of a wide coalesced streaming read → x2;
  WRITE_SIZE (KiB) is exact for 16-byte-per-lane streaming stores.
FETCH_SIZE and WRITE_SIZE come from separate --pmc passes (they do not fit one pass).
usage: pmc_summary.py <gpurun_out/rXX> <config> <out.json>
"""
import csv
import json
import os
import sys


def kernel_rows(path, match):
    rows = []
    for r in csv.DictReader(open(path)):
        if match(r["Kernel_Name"]):
            rows.append(r)
    return rows


def main(src, config, out):
    decode = lambda n: "scatter_kernel" in n and "false," in n.split("<")[1].split(",")[1] + ","
    fetch = kernel_rows(os.path.join(src, f"pmc_fetch_{config}", "run_counter_collection.csv"),
                        decode)
    write = kernel_rows(os.path.join(src, f"pmc_write_{config}", "run_counter_collection.csv"),
                        decode)
    stats = list(csv.DictReader(open(os.path.join(src, f"trace_{config}",
                                                  "run_kernel_stats.csv"))))
    f_kib = [float(r["Counter_Value"]) for r in fetch]
    w_kib = [float(r["Counter_Value"]) for r in write]
    fetch_b = 2 * 1024 * sum(f_kib) / len(f_kib)
    write_b = 1024 * sum(w_kib) / len(w_kib)
    dec = [s for s in stats if "scatter_kernel<4, false" in s["Name"]][0]
    res = {
        "config": config,
        "kernel": dec["Name"],
        "kernel_trace": {"calls": int(dec["Calls"]), "avg_ns": float(dec["AverageNs"]),
                         "min_ns": float(dec["MinNs"]), "max_ns": float(dec["MaxNs"])},
        "pmc": {"FETCH_SIZE_KiB_raw": sum(f_kib) / len(f_kib),
                "WRITE_SIZE_KiB_raw": sum(w_kib) / len(w_kib),
                "fetch_bytes_corrected_x2": fetch_b, "write_bytes": write_b,
                "traffic_bytes_per_launch": fetch_b + write_b, "launches": len(f_kib)},
        "all_kernels": [{"name": s["Name"], "calls": int(s["Calls"]),
                         "avg_ns": float(s["AverageNs"])} for s in stats],
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res["pmc"]))


if __name__ == "__main__":
    main(*sys.argv[1:4])
