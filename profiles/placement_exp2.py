#!/usr/bin/env python3
"""Is the decode rate a function of WHERE the buffers sit in HBM?  Eight 26 GiB buffers;
(1) hipMemcpy D2D of 24 GiB between several buffer pairs, (2) the c4 decode (quarter-size
region, 24 GiB) from a slab in buffer 1 into each of buffers 2..7.  Kernel-side HIP-event
timing, interleaved rounds, one process."""
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
bufs = [dev.malloc(GB) for _ in range(8)]
e0, e1 = dev.event(), dev.event()


def timed(fn, reps=3):
    fn()
    dev.sync()
    dev.record(e0)
    for _ in range(reps):
        fn()
    dev.record(e1)
    dev.sync()
    return dev.elapsed_ms(e0, e1) / reps


nb = 24 << 30
pairs = [(0, 1), (1, 0), (2, 3), (3, 2), (4, 5), (6, 7), (0, 7), (7, 0), (3, 4)]
cp = {p: [] for p in pairs}
for r in range(3):
    for p in pairs:
        cp[p].append(timed(lambda: dev.memcpy(bufs[p[1]], bufs[p[0]], nb, 2, sync=False)))

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
assert tot <= GB
nel = 1
for s in shape:
    nel *= s
dev.synth_fill(bufs[0], nel, 4, 0, bench.SEED)
slab = bufs[1]
sizes = dev.array_write(meta, bufs[0], [0] * n, shape, [(slab + o, c) for o, c in zip(offs, caps)])
plan = dev.plan(meta, [(slab + o, s) for o, s in zip(offs, sizes)], [0] * n, shape,
                A.ZH_SRC_DEVICE | A.ZH_OUT_DEVICE)
plan.set_timing(True)
dec = {k: [] for k in range(2, 8)}


def run(out):
    plan.execute(out)
    plan.wait()
    return plan.kernel_time()["scatter_ms"]


for r in range(4):
    for k in dec:
        run(bufs[k])
        dec[k].append(run(bufs[k]))
res = {
    "copy_GBps": {f"{a}->{b}": round(2 * nb / statistics.median(v) / 1e6, 1) for (a, b), v in cp.items()},
    "decode_GiBps": {f"1->{k}": round(nel * 4 / statistics.median(v) * 1e3 / 2**30, 1)
                     for k, v in dec.items()},
    "decode_spread": {f"1->{k}": [round(x, 3) for x in v] for k, v in dec.items()},
    "addresses": [hex(b) for b in bufs],
    "verify": [dev.synth_verify(bufs[k], shape, [0] * n, shape, 4, bench.SEED) for k in dec],
}
print(json.dumps(res))
