#!/usr/bin/env python3
"""Interleaved A/B of the small one-shot read (profiles/small_read_trace.py's shard and
region) under environment switches read per call: median of `reps` per variant, rounds
interleaved; every read verified.  usage: small_read_ab.py REPS VAR=VAL[,VAR=VAL] ..."""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from zarrhip import _abi as A  # noqa: E402
from zarrhip._lib import DeviceContext  # noqa: E402

reps = int(sys.argv[1])
variants = sys.argv[2:]
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
out = dev.malloc(64 ** 3 * 4)
res = {v: [] for v in variants}
for rnd in range(4):
    for v in variants:
        saved = {}
        for kv in ([] if v == "-" else v.split(",")):
            k, val = kv.split("=")
            saved[k] = os.environ.get(k)
            os.environ[k] = val
        for i in range(reps + 10):
            t0 = time.perf_counter()
            dev.array_read(meta, [(shard, size)], off, shp, out, A.ZH_SRC_DEVICE | A.ZH_OUT_DEVICE)
            if i >= 10:
                res[v].append(time.perf_counter() - t0)
        assert dev.synth_verify(out, shape, off, shp, 4, bench.SEED) == 0
        for k, old in saved.items():
            if old is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = old
print(json.dumps({v: round(statistics.median(t) * 1e6, 1) for v, t in res.items()}))
