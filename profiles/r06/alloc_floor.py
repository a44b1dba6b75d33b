#!/usr/bin/env python3
"""Round 6 lab: which output allocation kind has the highest FLOOR on the
full c4 array, and does the box's own copy ceiling move with the allocation?

One process, the full 1x4096x4096x1536 c4 array: the shard slab in one hipMalloc buffer; the
96 GiB output allocated 3 rounds x {hipMalloc, 1 GiB VMM chunks, 16 MiB VMM chunks}, each
freed before the next (the full output fits only once beside the slab).  Round r first takes a
spacer of r x 20 GiB (hipMalloc) so the allocator hands out other physical memory.  Per
candidate: decode kernel ms (HIP events, median of 3 x 2 launches, first output verified),
the copy ceiling slab -> output (zh_device_copy_rate), the contiguous store probe over the
whole output and over each 1 GiB slice.  Writes argv[1] (JSON lines)."""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
from zarrhip import _abi as A  # noqa: E402
from zarrhip._lib import DeviceContext, lib  # noqa: E402

GiB = 1 << 30
out_path = sys.argv[1]
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
dev = DeviceContext(0)
meta = bench.build_meta(A, "c4", 1)
n = meta.ndim
shape = [meta.shape[d] for d in range(n)]
nel = 1
for s in shape:
    nel *= s
nb = nel * 4
L = lib()
coords = bench.all_coords(L, meta)
caps = bench.chunk_capacities(meta, coords)
offs, tot = bench.slab_layout(caps)
PLAIN = getattr(A, "ZH_MALLOC_PLAIN", 0)  # hipMalloc (flags 0 before round 6's default change)
slab = dev.malloc(tot, PLAIN)
gen = dev.malloc(nb, PLAIN)
dev.synth_fill(gen, nel, 4, 0, bench.SEED)
sizes = dev.array_write(meta, gen, [0] * n, shape, [(slab + o, c) for o, c in zip(offs, caps)])
plan = dev.plan(meta, [(slab + o, s) for o, s in zip(offs, sizes)], [0] * n, shape,
                A.ZH_SRC_DEVICE | A.ZH_OUT_DEVICE)
st = plan.stats()
alg = st["in_bytes"] + st["out_bytes"]
plan.set_timing(True)
fo = open(out_path, "w")


def measure(kind, out, rnd):
    t0 = time.perf_counter()
    plan.execute(out)
    plan.wait()
    bad = dev.synth_verify(out, shape, [0] * n, shape, 4, bench.SEED)
    plan.kernel_time()
    ks = []
    for _ in range(3):
        for _ in range(2):
            plan.execute(out)
        plan.wait()
        kt = plan.kernel_time()
        ks.append(kt["scatter_ms"] / kt["launches"])
    kms = statistics.median(ks)
    copy = dev.copy_rate(out, slab, nb, 3)
    probe = dev.write_rate(out, nb, 0, 3)
    sl = [dev.write_rate(out + i * GiB, GiB, 0, 3) for i in range(nb // GiB)]
    rec = {"kind": kind, "round": rnd, "verify_bad": bad, "kernel_ms": round(kms, 3),
           "kernel_ms_samples": [round(x, 3) for x in ks],
           "frac": round(alg / (kms / 1e3) / 8e12, 4),
           "GiBps": round(nb / (kms / 1e3) / GiB, 1),
           "copy_ceiling_GBps": round(copy, 1), "frac_of_copy": round(alg / (kms / 1e3) / 1e9 / copy, 4),
           "probe_GBps": round(probe, 1),
           "slice_probe": {"min": round(min(sl), 1), "median": round(statistics.median(sl), 1),
                           "max": round(max(sl), 1), "n_below_90pct_median":
                           sum(1 for x in sl if x < 0.9 * statistics.median(sl))},
           "slices": [round(x) for x in sl], "s": round(time.perf_counter() - t0, 2)}
    fo.write(json.dumps(rec) + "\n")
    fo.flush()
    print(json.dumps({k: v for k, v in rec.items() if k != "slices"}), flush=True)


measure("hipMalloc(first, gen buffer)", gen, -1)
dev.free(gen)
kinds = [("hipMalloc", getattr(A, "ZH_MALLOC_PLAIN", 0), None),
         ("vmm1g", A.ZH_MALLOC_SCATTER, "1024"),
         ("vmm16m", A.ZH_MALLOC_SCATTER, "16")]
for r in range(rounds):
    spacer = dev.malloc(r * 20 * GiB, PLAIN) if r else None
    for name, flags, mb in kinds:
        if mb:
            os.environ["ZH_SCATTER_MB"] = mb
        t0 = time.perf_counter()
        out = dev.malloc(nb, flags)
        ta = time.perf_counter() - t0
        print(f"alloc {name} {ta:.2f}s", flush=True)
        measure(name, out, r)
        dev.free(out)
    if spacer:
        dev.free(spacer)
plan.close()
dev.free(slab)
print("done", flush=True)
