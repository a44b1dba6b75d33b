#!/usr/bin/env python3
"""Latency of region reads whose shards sit in HOST memory (the C-ABI use with mmap'd shard
files): one c3 shard (1x1024^3 uint32, 4 GiB, inner 32^3, index + crc32c at the end) in
pinned and in pageable host memory; zh_array_read of a 1x64x64x64 region (the reference's
l4_sample read shape, BASELINE configs[0]) and of a 1x1024x1024x512 half shard, with the
planner's compact staging (default) and with whole-shard staging (ZH_COMPACT=0).
Median of 5 after 1 warmup; every result checked against the generator."""
import ctypes as C
import json
import os
import statistics
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from zarrhip import _abi as A  # noqa: E402
from zarrhip._lib import DeviceContext  # noqa: E402

dev = DeviceContext(0)
meta = A.make_meta([1, 1024, 1024, 1024], [1, 1024, 1024, 1024], 4, endian=A.ZH_ENDIAN_BIG,
                   sharded=True, inner_chunk_shape=[1, 32, 32, 32], index_crc32c=True)
shape = [1, 1024, 1024, 1024]
nel = 1 << 30
region = dev.malloc(nel * 4)
dev.synth_fill(region, nel, 4, 0, bench.SEED)
cap = 4 * nel + 16 * 32768 + 4
dslab = dev.malloc(cap)
size = dev.array_write(meta, region, [0] * 4, shape, [(dslab, cap)])[0]
pinned = dev.malloc_pinned(size)
dev.memcpy(pinned, dslab, size, 1, None, True)
pageable = (C.c_char * size)()
C.memmove(pageable, pinned, size)
dev.free(region)
dev.free(dslab)
def splitmix64(x):
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def check(got, off, shp):
    """Generator v(g) = lo32(splitmix64(g ^ seed)) on 8 sampled rows of the region."""
    rng = np.random.default_rng(0)
    for _ in range(8):
        y, x = int(rng.integers(shp[1])), int(rng.integers(shp[2]))
        g0 = ((off[1] + y) * 1024 + (off[2] + x)) * 1024 + off[3]
        g = np.arange(g0, g0 + shp[3], dtype=np.uint64)
        want = (splitmix64(g ^ np.uint64(bench.SEED)) & np.uint64(0xFFFFFFFF)).astype(np.uint32)
        if not np.array_equal(got[0, y, x], want):
            return False
    return True


res = {}
for mem, ptr in (("pinned", pinned), ("pageable", C.addressof(pageable))):
    for name, off, shp in (("64^3", [0, 300, 500, 200], [1, 64, 64, 64]),
                           ("half_shard", [0, 0, 0, 512], [1, 1024, 1024, 512])):
        nb = int(np.prod(shp)) * 4
        out = dev.malloc_pinned(nb)
        for compact in ("1", "0"):
            os.environ["ZH_COMPACT"] = compact
            ts = []
            for r in range(6):
                t0 = time.perf_counter()
                dev.array_read(meta, [(ptr, size)], off, shp, out, 0)
                ts.append(time.perf_counter() - t0)
            plan = dev.plan(meta, [(ptr, size)], off, shp, 0)
            staged = plan.staged_bytes()
            plan.close()
            got = np.ctypeslib.as_array((C.c_uint32 * (nb // 4)).from_address(out)).reshape(shp)
            ok = check(got, off, shp)
            res[f"{mem}/{name}/compact={compact}"] = {
                "median_ms": round(statistics.median(ts[1:]) * 1e3, 3),
                "staged_MiB": round(staged / 2 ** 20, 2), "verified": ok}
        dev.free_pinned(out)
print(json.dumps(res, indent=1))
