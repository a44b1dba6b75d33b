#!/usr/bin/env python3
"""What sets the write mode of a ZH_MALLOC_SCATTER arena: its physical chunks, their order, or
the virtual range they sit at?  (DESIGN §4 "Placement".)  Decodes the quarter-size c4 slab
(1x1024x4096x1536 uint32, 24 GiB out) into NB arenas of 1 GiB chunks and into VIEWS extra
views of each (the same physical chunks mapped again at a fresh virtual range, view k in chunk
order k: zh_device_scatter_view).  Per (arena, view): the contiguous write probe (GB/s), the
decode kernel time (HIP events, min of 2) and a verification of that decode through the same
pointer.  Then every view is freed, a plain 24 GiB buffer is filled and checked, and every
arena is decoded and checked once more (no cross-talk from freed mappings).
usage: placement_calib.py [NB] [VIEWS]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from zarrhip import _abi as A  # noqa: E402
from zarrhip._lib import DeviceContext, lib  # noqa: E402

NB = int(sys.argv[1]) if len(sys.argv) > 1 else 6
VIEWS = int(sys.argv[2]) if len(sys.argv) > 2 else 3
dev = DeviceContext(0)
meta = bench.build_meta(A, "c4", 4)
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
plan = dev.plan(meta, [(slab + o, s) for o, s in zip(offs, sizes)], [0] * n, shape,
                A.ZH_SRC_DEVICE | A.ZH_OUT_DEVICE)
plan.set_timing(True)


def decode_ms(b):
    best = 1e9
    for _ in range(2):
        plan.kernel_time()
        plan.execute(b)
        plan.wait()
        best = min(best, plan.kernel_time()["scatter_ms"])
    return best


def measure(arena, view, ptr):
    p0 = dev.write_rate(ptr, nb, 0, 3)
    ms = decode_ms(ptr)
    bad = dev.synth_verify(ptr, shape, [0] * n, shape, 4, bench.SEED)
    row = {"arena": arena, "view": view, "va": hex(ptr), "probe0_GBps": round(p0, 1),
           "decode_ms": round(ms, 3), "decode_GiBps": round(nb / (ms / 1e3) / 2**30, 1),
           "verify_mismatches": int(bad)}
    print(json.dumps(row), flush=True)
    return row


arenas = [dev.malloc(nb, A.ZH_MALLOC_SCATTER | A.ZH_MALLOC_REQUIRE) for _ in range(NB)]
views = {k: [dev.scatter_view(b, v) for v in range(VIEWS)] for k, b in enumerate(arenas)}
rows = []
for rep in range(2):
    for k, b in enumerate(arenas):
        rows.append(measure(k, -1, b))
        for v, p in enumerate(views[k]):
            rows.append(measure(k, v, p))
for vs in views.values():
    for p in vs:
        dev.free(p)
other = dev.malloc(nb, 0)
dev.synth_fill(other, nel, 4, 0, 9)
bad_other = dev.synth_verify(other, [nel], [0], [nel], 4, 9)
after = [measure(k, -2, b) for k, b in enumerate(arenas)]
bad_other += dev.synth_verify(other, [nel], [0], [nel], 4, 9)
print(json.dumps({"summary": True, "rows": len(rows),
                  "verify_mismatches": sum(r["verify_mismatches"] for r in rows + after),
                  "other_buffer_mismatches": int(bad_other)}))
