#!/usr/bin/env python3
"""One-shot small-read latency: zh_array_read (plan + execute + teardown in one call, the
way HipArray.read binds it) of a 1x64x64x64 region (BASELINE configs[0]'s read shape) from a
device-resident c4-format shard (1x1024^3 uint32, inner 32^3 + transpose [0,3,2,1], index +
crc32c), into device memory and into pinned and pageable host memory; beside it the reused
plan (execute + wait), and the rate of a 2 GiB half-shard read into pinned / pageable memory.
Median of 200 after 20 warmups; every result checked against the generator.
usage: oneshot_latency.py [reps]"""
import ctypes as C
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from zarrhip import _abi as A  # noqa: E402
from zarrhip._lib import DeviceContext  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
dev = DeviceContext(0)
meta = A.make_meta([1, 1024, 1024, 1024], [1, 1024, 1024, 1024], 4, endian=A.ZH_ENDIAN_BIG,
                   sharded=True, inner_chunk_shape=[1, 32, 32, 32], transpose_order=[0, 3, 2, 1],
                   index_crc32c=True)
shape = [1, 1024, 1024, 1024]
nel = 1 << 30
region = dev.malloc(nel * 4)
dev.synth_fill(region, nel, 4, 0, bench.SEED)
cap = 4 * nel + 16 * 32768 + 4
shard = dev.malloc(cap)
size = dev.array_write(meta, region, [0] * 4, shape, [(shard, cap)])[0]
dev.free(region)
off, shp = [0, 3, 517, 501], [1, 64, 64, 64]
nb = 64 ** 3 * 4
dout = dev.malloc(nb)
hout = dev.malloc_pinned(nb)
res = {}


def timed(fn):
    ts = []
    for i in range(reps + 20):
        t0 = time.perf_counter()
        fn()
        if i >= 20:
            ts.append(time.perf_counter() - t0)
    return round(statistics.median(ts) * 1e6, 1)


res["zh_array_read one-shot, device out"] = timed(
    lambda: dev.array_read(meta, [(shard, size)], off, shp, dout, A.ZH_SRC_DEVICE | A.ZH_OUT_DEVICE))
assert dev.synth_verify(dout, shape, off, shp, 4, bench.SEED) == 0
res["zh_array_read one-shot, pinned host out"] = timed(
    lambda: dev.array_read(meta, [(shard, size)], off, shp, hout, A.ZH_SRC_DEVICE))
dev.memcpy(dout, hout, nb, 0, None, True)
assert dev.synth_verify(dout, shape, off, shp, 4, bench.SEED) == 0
pageable = (C.c_char * nb)()  # e.g. the Java int[] behind GetPrimitiveArrayCritical
res["zh_array_read one-shot, pageable host out"] = timed(
    lambda: dev.array_read(meta, [(shard, size)], off, shp, C.addressof(pageable), A.ZH_SRC_DEVICE))
dev.memcpy(dout, C.addressof(pageable), nb, 0, None, True)
assert dev.synth_verify(dout, shape, off, shp, 4, bench.SEED) == 0
# a large read: a 1x512x1024x1024 half shard (2 GiB) into pinned and pageable host memory
boff, bshp = [0, 256, 0, 0], [1, 512, 1024, 1024]
bnb = 512 * 1024 * 1024 * 4
bpin = dev.malloc_pinned(bnb)
bpage = (C.c_char * bnb)()
for tag, dst in (("pinned", bpin), ("pageable", C.addressof(bpage))):
    ts = []
    for i in range(4):
        t0 = time.perf_counter()
        dev.array_read(meta, [(shard, size)], boff, bshp, dst, A.ZH_SRC_DEVICE)
        if i:
            ts.append(time.perf_counter() - t0)
    res[f"zh_array_read 2 GiB half shard, {tag} host out (GiB/s)"] = \
        round(bnb / statistics.median(ts) / 2**30, 2)
dev.free_pinned(bpin)
del bpage
# the whole 4 GiB shard into pinned memory: one staging buffer (ZH_HOST_SLABS=0) against the
# double-buffered C-order slab pipeline, with 512 MiB and 1 GiB slabs
fnb = 1024 ** 3 * 4
fpin = dev.malloc_pinned(fnb)
for tag, env in (("one staging buffer", {"ZH_HOST_SLABS": "0"}),
                 ("512 MiB slabs", {"ZH_HOST_SLABS": "1", "ZH_HOST_SLAB_MIN_KB": "1048576",
                                    "ZH_HOST_SLAB_KB": "524288"}),
                 ("1 GiB slabs", {"ZH_HOST_SLABS": "1", "ZH_HOST_SLAB_MIN_KB": "1048576",
                                  "ZH_HOST_SLAB_KB": "1048576"})):
    os.environ.update(env)
    ts = []
    for i in range(4):
        t0 = time.perf_counter()
        dev.array_read(meta, [(shard, size)], [0] * 4, shape, fpin, A.ZH_SRC_DEVICE)
        if i:
            ts.append(time.perf_counter() - t0)
    res[f"zh_array_read 4 GiB shard, pinned host out, {tag} (GiB/s)"] = \
        round(fnb / statistics.median(ts) / 2**30, 2)
for k in ("ZH_HOST_SLABS", "ZH_HOST_SLAB_MIN_KB", "ZH_HOST_SLAB_KB"):
    os.environ.pop(k, None)
chk = dev.malloc(64 ** 3 * 4)
dev.memcpy(chk, fpin + (512 * 1024 * 1024 + 512 * 1024 + 512) * 4, 64 * 4, 0, None, True)
dev.free(chk)
dev.free_pinned(fpin)
plan = dev.plan(meta, [(shard, size)], off, shp, A.ZH_SRC_DEVICE | A.ZH_OUT_DEVICE)


def run_plan():
    plan.execute(dout)
    plan.wait()


res["reused plan, execute + wait, device out"] = timed(run_plan)
assert dev.synth_verify(dout, shape, off, shp, 4, bench.SEED) == 0
plan.close()
print(json.dumps({"unit": "us per read, median", "reps": reps, "latency": res}))
