#!/usr/bin/env python3
"""Placement follow-up: is the per-buffer decode rate (bimodal in placement_exp2) tied to
the ALLOCATION (physical fragments / TLB reach) or to ADDRESS BITS (channel mapping)?
Decode c4/c3 (quarter-size, 24 GiB) into each of 6 buffers at sub-buffer offsets
0 / 2 MiB / 64 MiB / 1 GiB; also hipMemset and slab->buffer D2D per buffer."""
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
NB = 7
FLAGS = int(sys.argv[2], 0) if len(sys.argv) > 2 else 0  # A.ZH_MALLOC_* (3 = contiguous, required)
bufs = [dev.malloc(GB, FLAGS) for _ in range(NB)]
e0, e1 = dev.event(), dev.event()


def timed(fn, reps=2):
    fn()
    dev.sync()
    dev.record(e0)
    for _ in range(reps):
        fn()
    dev.record(e1)
    dev.sync()
    return dev.elapsed_ms(e0, e1) / reps


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
nb = nel * 4
assert tot <= GB and nb + (1 << 30) <= GB
dev.synth_fill(bufs[0], nel, 4, 0, bench.SEED)
slab = bufs[1]
sizes = dev.array_write(meta, bufs[0], [0] * n, shape, [(slab + o, c) for o, c in zip(offs, caps)])
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


OFFS = [0, 2 << 20, 64 << 20, 1 << 30]
res = {f"b{k}+{o >> 20}M": [] for k in range(2, NB) for o in OFFS}
ms = {f"b{k}": [] for k in range(2, NB)}
cp = {f"b{k}": [] for k in range(2, NB)}
for r in range(3):
    for k in range(2, NB):
        for o in OFFS:
            res[f"b{k}+{o >> 20}M"].append(dec(bufs[k] + o))
        ms[f"b{k}"].append(timed(lambda: dev.memset(bufs[k], 0, nb)))
        cp[f"b{k}"].append(timed(lambda: dev.memcpy(bufs[k], slab, nb, 2, sync=False)))
gib = lambda v: round(nb / statistics.median(v) * 1e3 / 2**30, 1)  # noqa: E731
print(json.dumps({
    "decode_GiBps": {k: gib(v) for k, v in res.items()},
    "memset_GBps": {k: round(nb / statistics.median(v) / 1e6, 1) for k, v in ms.items()},
    "copy_GBps": {k: round(2 * nb / statistics.median(v) / 1e6, 1) for k, v in cp.items()},
    "addresses": [hex(b) for b in bufs], "malloc_flags": FLAGS,
}))
