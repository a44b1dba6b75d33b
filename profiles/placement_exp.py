#!/usr/bin/env python3
"""Does the relative placement of the encoded shards and the decoded region in HBM change
the c3 decode rate?  Two region buffers, one allocated BEFORE the shard slab (as bench.py's
weak mode does) and one AFTER it; interleaved timing in one process."""
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

dev = DeviceContext(0)
meta = bench.build_meta(A, sys.argv[1] if len(sys.argv) > 1 else "c3", 2)  # 48 GiB regions: two fit beside the slab
n = meta.ndim
shape = [meta.shape[d] for d in range(n)]
cs = [meta.chunk_shape[d] for d in range(n)]
L = lib()
num = L.zh_compute_chunk_coords(n, i64arr(shape), i32arr(cs), i64arr([0] * n), i64arr(shape), None, 0)
buf = (C.c_int64 * (num * n))()
L.zh_compute_chunk_coords(n, i64arr(shape), i32arr(cs), i64arr([0] * n), i64arr(shape), buf, num)
coords = [tuple(buf[i * n + d] for d in range(n)) for i in range(num)]
caps = bench.chunk_capacities(meta, coords)
nel = 1
for s in shape:
    nel *= s
before = dev.malloc(nel * 4)
offs, tot = [], 0
for c in caps:
    offs.append(tot)
    tot += (c + 255) // 256 * 256
slab = dev.malloc(tot)
after = dev.malloc(nel * 4)
dev.synth_fill(before, nel, 4, 0, bench.SEED)
sizes = dev.array_write(meta, before, [0] * n, shape, [(slab + o, c) for o, c in zip(offs, caps)])
plan = dev.plan(meta, [(slab + o, s) for o, s in zip(offs, sizes)], [0] * n, shape,
                A.ZH_SRC_DEVICE | A.ZH_OUT_DEVICE)
res = {"before": [], "after": []}
for name, out in (("before", before), ("after", after)):
    plan.execute(out)
    plan.wait()
for r in range(6):
    for name, out in (("before", before), ("after", after)):
        dev.sync()
        t0 = time.perf_counter()
        for _ in range(3):
            plan.execute(out)
        plan.wait()
        res[name].append((time.perf_counter() - t0) / 3 * 1e3)
out = {k: {"median_ms": round(statistics.median(v), 3),
           "GiB/s": round(nel * 4 / statistics.median(v) * 1e3 / 2**30, 1)} for k, v in res.items()}
out["addresses"] = {"before": hex(before), "slab": hex(slab), "after": hex(after)}
out["verify"] = [dev.synth_verify(x, shape, [0] * n, shape, 4, bench.SEED) for x in (before, after)]
print(json.dumps(out))
