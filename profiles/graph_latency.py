#!/usr/bin/env python3
"""Small-read latency with and without hipGraph replay (zh_plan_set_graph): a 1x64x64x64
region (the reference's l4_sample read shape, BASELINE configs[0]) read repeatedly from a
device-resident c4-format shard (1x1024^3 uint32, inner 32^3 + transpose [0,3,2,1], index +
crc32c).  Per-read wall time of execute + wait, median of 200 after 20 warmups; the result
is checked against the generator."""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from zarrhip import _abi as A  # noqa: E402
from zarrhip._lib import DeviceContext  # noqa: E402

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
res = {}
for off, shp, tag in [([0, 0, 512, 512], [1, 64, 64, 64], "64^3 aligned"),
                      ([0, 3, 517, 501], [1, 64, 64, 64], "64^3 unaligned")]:
    out = dev.malloc(64 ** 3 * 4)
    plan = dev.plan(meta, [(shard, size)], off, shp, A.ZH_SRC_DEVICE | A.ZH_OUT_DEVICE)
    for graph in (False, True):
        plan.set_graph(graph)
        ts = []
        for i in range(220):
            t0 = time.perf_counter()
            plan.execute(out)
            plan.wait()
            if i >= 20:
                ts.append(time.perf_counter() - t0)
        bad = dev.synth_verify(out, shape, off, shp, 4, bench.SEED)
        assert bad == 0, bad
        res[f"{tag}, {'hipGraph' if graph else 'stream enqueue'}"] = \
            round(statistics.median(ts) * 1e6, 1)
    plan.close()
    dev.free(out)
print(json.dumps({"unit": "us per read (execute + wait), median of 200", "latency": res}))
