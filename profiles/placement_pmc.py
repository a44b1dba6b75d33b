#!/usr/bin/env python3
"""Allocation-placement bimodality: decode the same quarter-size c4 slab
(1x1024x4096x1536 uint32, 24 GiB out) into NB separately allocated output buffers, REPS
times each in buffer order, and print each dispatch's HIP-event kernel time, so that a
rocprofv3 --pmc run of this script can put per-dispatch TCC/EA counters (memory-side
request and stall counts, per L2 channel) beside the fast and the slow buffers.
usage: placement_pmc.py [config] [NB] [REPS] [mix]
mode: plain (hipMalloc), scatter (ZH_MALLOC_SCATTER: VMM physical chunks of ZH_SCATTER_MB,
mapped in a coprime-stride order) or mix (alternating)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from zarrhip import _abi as A  # noqa: E402
from zarrhip._lib import DeviceContext, lib  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c4"
NB = int(sys.argv[2]) if len(sys.argv) > 2 else 6
REPS = int(sys.argv[3]) if len(sys.argv) > 3 else 2
dev = DeviceContext(0)
meta = bench.build_meta(A, cfg, 4)
n = meta.ndim
shape = [meta.shape[d] for d in range(n)]
L = lib()
coords = bench.all_coords(L, meta)
caps = bench.chunk_capacities(meta, coords)
offs, tot = bench.slab_layout(caps)
nel = 1
for s in shape:
    nel *= s
nb = nel * 4
src = dev.malloc(nb)
slab = dev.malloc(tot)
dev.synth_fill(src, nel, 4, 0, bench.SEED)
sizes = dev.array_write(meta, src, [0] * n, shape, [(slab + o, c) for o, c in zip(offs, caps)])
dev.free(src)
MODE = sys.argv[4] if len(sys.argv) > 4 else "plain"
kinds = [("scatter" if (MODE == "mix" and k % 2) or MODE == "scatter" else "hipMalloc")
         for k in range(NB)]
bufs = [dev.malloc(nb, A.ZH_MALLOC_SCATTER | A.ZH_MALLOC_REQUIRE if kd == "scatter" else 0)
        for kd in kinds]
plan = dev.plan(meta, [(slab + o, s) for o, s in zip(offs, sizes)], [0] * n, shape,
                A.ZH_SRC_DEVICE | A.ZH_OUT_DEVICE)
plan.set_timing(True)
order, ms = [], []
for r in range(REPS):
    for k, b in enumerate(bufs):
        plan.kernel_time()
        plan.execute(b)
        plan.wait()
        t = plan.kernel_time()
        order.append(k)
        ms.append(round(t["scatter_ms"], 3))
bad = sum(dev.synth_verify(b, shape, [0] * n, shape, 4, bench.SEED) for b in bufs)
alg = plan.stats()
print(json.dumps({"config": cfg, "buffers": NB, "reps": REPS, "kinds": kinds,
                  "scatter_mb": os.environ.get("ZH_SCATTER_MB"), "dispatch_buffer": order,
                  "kernel_ms": ms, "GiBps": [round(nb / (m / 1e3) / (1 << 30), 1) for m in ms],
                  "addresses": [hex(b) for b in bufs], "verify_mismatches": int(bad),
                  "alg_bytes": alg["in_bytes"] + alg["out_bytes"]}))
