#!/usr/bin/env python3
"""Can the allocation itself remove the slow placement mode?  Decode c4 (or argv[1]) at
quarter size from one slab into output buffers allocated as: plain hipMalloc (x2), and
ZH_MALLOC_SCATTER (physical chunks mapped in a coprime-stride order) at 2 MiB, 64 MiB and
1 GiB chunks (x2 / x2 / x1).  Interleaved rounds, kernel time by HIP events, all verified."""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from zarrhip import _abi as A  # noqa: E402
from zarrhip._lib import DeviceContext, lib, i64arr, i32arr  # noqa: E402
import ctypes as C  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c4"
dev = DeviceContext(0)
meta = bench.build_meta(A, cfg, 4)
n = meta.ndim
shape = [meta.shape[d] for d in range(n)]
cs = [meta.chunk_shape[d] for d in range(n)]
nel = 1
for s in shape:
    nel *= s
nb = nel * 4
src = dev.malloc(nb, 0)
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
slab = dev.malloc(tot, 0)
outs, alloc_s = {}, {}
for name, flags, mb in [("plain_a", 0, 0), ("plain_b", 0, 0), ("scat2_a", 4 | 2, 2),
                        ("scat2_b", 4 | 2, 2), ("scat64_a", 4 | 2, 64), ("scat64_b", 4 | 2, 64),
                        ("scat1024", 4 | 2, 1024)]:
    os.environ["ZH_SCATTER_MB"] = str(mb or 2)
    t0 = time.perf_counter()
    outs[name] = dev.malloc(nb, flags)
    alloc_s[name] = round(time.perf_counter() - t0, 3)
dev.synth_fill(src, nel, 4, 0, bench.SEED)
sizes = dev.array_write(meta, src, [0] * n, shape, [(slab + o, c) for o, c in zip(offs, caps)])
plan = dev.plan(meta, [(slab + o, s) for o, s in zip(offs, sizes)], [0] * n, shape,
                A.ZH_SRC_DEVICE | A.ZH_OUT_DEVICE)
plan.set_timing(True)


def dec(out):
    plan.execute(out)
    plan.wait()
    plan.kernel_time()
    plan.execute(out)
    plan.wait()
    return plan.kernel_time()["scatter_ms"]


res = {k: [] for k in outs}
for r in range(3):
    for k, o in outs.items():
        res[k].append(dec(o))
print(json.dumps({"config": cfg,
                  "GiBps": {k: round(nb / statistics.median(v) * 1e3 / 2**30, 1) for k, v in res.items()},
                  "alloc_s": alloc_s,
                  "verify": {k: dev.synth_verify(o, shape, [0] * n, shape, 4, bench.SEED)
                             for k, o in outs.items()}}))
for o in outs.values():
    dev.free(o)
