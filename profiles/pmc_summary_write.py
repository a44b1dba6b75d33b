#!/usr/bin/env python3
"""Summarise rocprofv3 output of `bench.py --op write` for one config into
profiles/<round>/write_<config>_summary.json: the encode kernel's (the fast kernels on the
encode view, FLAGS = true) average duration, and its HBM bytes per launch from separate
FETCH_SIZE and WRITE_SIZE passes, corrected as /opt/skills/guides/MI355X_MICROARCH.md §HBM
prescribes for gfx950 (FETCH_SIZE x2, WRITE_SIZE exact).  Algorithmic bytes per launch: the
region read (O) + the payloads written (+ 4 B per chunk with the inner crc32c).
usage: pmc_summary_write.py <gpurun_out/rXX> <config> <out.json> <alg_bytes>
"""
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import FAST, DECODE_ONLY, flags_arg, is_encode_flags, kernel_rows  # noqa: E402


def encode_view(n):
    if "tiles_rowcrc_enc_aln_kernel" in n:
        return True
    return any(k in n for k in FAST) and not any(k in n for k in DECODE_ONLY) and \
        is_encode_flags(flags_arg(n))


def main(src, config, out, alg):
    alg = int(alg)
    fetch = kernel_rows(os.path.join(src, f"wfetch_{config}", "run_counter_collection.csv"),
                        encode_view)
    write = kernel_rows(os.path.join(src, f"wwrite_{config}", "run_counter_collection.csv"),
                        encode_view)
    stats = list(csv.DictReader(open(os.path.join(src, f"wtrace_{config}",
                                                  "run_kernel_stats.csv"))))
    enc = [s for s in stats if encode_view(s["Name"])]
    nf, nw = len(fetch), len(write)
    f_kib = sum(float(r["Counter_Value"]) for r in fetch) / max(1, nf)
    w_kib = sum(float(r["Counter_Value"]) for r in write) / max(1, nw)
    fetch_b, write_b = 2 * 1024 * f_kib, 1024 * w_kib
    calls = sum(int(s["Calls"]) for s in enc)
    avg_ns = sum(float(s["TotalDurationNs"]) for s in enc) / max(1, calls)
    res = {
        "config": config, "op": "write",
        "kernel": " + ".join(s["Name"] for s in enc),
        "kernel_trace": {"calls": calls, "avg_ns": avg_ns},
        "alg_bytes_per_launch": alg,
        "pmc": {"FETCH_SIZE_KiB_raw": f_kib, "WRITE_SIZE_KiB_raw": w_kib,
                "fetch_bytes_corrected_x2": fetch_b, "write_bytes": write_b,
                "traffic_bytes_per_launch": fetch_b + write_b,
                "traffic_over_alg": (fetch_b + write_b) / alg if alg else None,
                "launches": [nf, nw]},
        "achieved_GBps": alg / avg_ns if avg_ns else None,
        "all_kernels": [{"name": s["Name"], "calls": int(s["Calls"]),
                         "avg_ns": float(s["AverageNs"])} for s in stats],
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({"kernel_ms": avg_ns / 1e6, **res["pmc"]}))


if __name__ == "__main__":
    main(*sys.argv[1:5])
