#!/usr/bin/env python3
"""Does visiting items in a coprime-stride order (ZH_ITEM_PERM=1) remove the allocation
sensitivity seen in placement_exp3?  c4 (or
argv[1]) at quarter size, one slab, six output allocations, interleaved rounds of plans
built with ZH_ITEM_PERM=0 (keys "nt0") and 1 ("nt1"); non-temporal streams in both."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from zarrhip import _abi as A  # noqa: E402
from zarrhip._lib import DeviceContext, lib, i64arr, i32arr  # noqa: E402
import ctypes as C  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c4"
dev = DeviceContext(0)
GB = 26 << 30
NB = 8
bufs = [dev.malloc(GB) for _ in range(NB)]
meta = bench.build_meta(A, cfg, 4)
n = meta.ndim
shape = [meta.shape[d] for d in range(n)]
cs = [meta.chunk_shape[d] for d in range(n)]
L = lib()
num = L.zh_compute_chunk_coords(n, i64arr(shape), i32arr(cs), i64arr([0] * n), i64arr(shape), None, 0)
cb = (C.c_int64 * (num * n))()
L.zh_compute_chunk_coords(n, i64arr(shape), i32arr(cs), i64arr([0] * n), i64arr(shape), cb, num)
coords = [tuple(cb[i * n + d] for d in range(n)) for i in range(num)]
caps = bench.chunk_capacities(meta, coords)
offs, tot = [], 0
for c in caps:
    offs.append(tot)
    tot += (c + 255) // 256 * 256
nel = 1
for s in shape:
    nel *= s
dev.synth_fill(bufs[0], nel, 4, 0, bench.SEED)
slab = bufs[1]
sizes = dev.array_write(meta, bufs[0], [0] * n, shape, [(slab + o, c) for o, c in zip(offs, caps)])
plans = {}
for nt in (0, 1):
    os.environ["ZH_ITEM_PERM"] = str(nt)
    p = dev.plan(meta, [(slab + o, s) for o, s in zip(offs, sizes)], [0] * n, shape,
                 A.ZH_SRC_DEVICE | A.ZH_OUT_DEVICE)
    p.set_timing(True)
    plans[nt] = p


def dec(p, out):
    p.execute(out)
    p.wait()
    p.kernel_time()
    p.execute(out)
    p.wait()
    return p.kernel_time()["scatter_ms"]


res = {f"b{k}_nt{nt}": [] for k in range(2, NB) for nt in plans}
for r in range(3):
    for k in range(2, NB):
        for nt, p in plans.items():
            res[f"b{k}_nt{nt}"].append(dec(p, bufs[k]))
gib = lambda v: round(nel * 4 / statistics.median(v) * 1e3 / 2**30, 1)  # noqa: E731
print(json.dumps({"config": cfg, "GiBps": {k: gib(v) for k, v in res.items()},
                  "verify": [dev.synth_verify(bufs[k], shape, [0] * n, shape, 4, bench.SEED)
                             for k in range(2, NB)]}))
