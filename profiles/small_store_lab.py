#!/usr/bin/env python3
"""BASELINE configs[0]'s call shape from the store: zarrhip.Array.read of the unaligned 64^3
region {0,3,517,501} from a c4 shard file on /dev/shm (zh_array_read_files: the index + 27
ranges read, one plan), through the page-locked staging (default) and into heap buffers
(ZH_FILE_PIN=0), interleaved; plus the mirror's own store
reads (ZH_FILES=0) and the device-resident one-shot read for reference.  Median of R reads per
setting and round.  Prints one JSON object.  usage: small_store_lab.py out.json [reps]"""
import json
import os
import shutil
import sys
import time
import ctypes as C

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import zarrhip as z  # noqa: E402
from zarrhip import _abi as A  # noqa: E402
from zarrhip.array import device  # noqa: E402

out_path = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
trace = len(sys.argv) > 3 and sys.argv[3] == "trace"  # one setting, one round (rocprofv3)
dev = device()
shape = [1, 1024, 1024, 1024]
meta = A.make_meta(shape, [1, 1024, 1024, 1024], 4, endian=A.ZH_ENDIAN_BIG, sharded=True,
                   inner_chunk_shape=[1, 32, 32, 32], transpose_order=[0, 3, 2, 1],
                   index_crc32c=True)
nel = 1 << 30
region = dev.malloc(nel * 4)
dev.synth_fill(region, nel, 4, 0, bench.SEED)
cap = 4 * nel + 16 * 32768 + 4
shard = dev.malloc(cap)
size = dev.array_write(meta, region, [0] * 4, shape, [(shard, cap)])[0]
base = f"/dev/shm/zh_small_{os.getpid()}"
m = (z.ArrayMetadataBuilder().withShape(*shape).withDataType(z.DataType.UINT32)
     .withChunkShape(*shape).withFillValue(0)
     .withCodecs(lambda c: c.withSharding([1, 32, 32, 32],
                                          lambda c1: c1.withTranspose([0, 3, 2, 1]).withBytes("BIG")))
     .build())
z.Array.create(z.FilesystemStore(base).resolve("a"), m)
p = os.path.join(base, "a", "c", "0", "0", "0", "0")
os.makedirs(os.path.dirname(p), exist_ok=True)
pin = dev.malloc_pinned(size)
dev.memcpy(pin, shard, size, 1, None, True)
with open(p, "wb") as f:
    f.write((C.c_char * size).from_address(pin))
dev.free_pinned(pin)
arr = z.Array.open(z.FilesystemStore(base).resolve("a"))
off, shp = [0, 3, 517, 501], [1, 64, 64, 64]
settings = [("files", {}), ("files_heap", {"ZH_FILE_PIN": "0"}),
            ("store_reads", {"ZH_FILES": "0"})]
if trace:
    settings = settings[:1]
res = {"reps": reps, "region_offset": off, "region_shape": shp, "rounds": []}
try:
    for rnd in range(1 if trace else 3):
        row = {}
        for name, env in settings:
            os.environ.update(env)
            ts = []
            for k in range(reps + 20):
                t0 = time.perf_counter()
                got = arr.read(off, shp)
                if k >= 20:
                    ts.append(time.perf_counter() - t0)
            for key in env:
                os.environ.pop(key, None)
            ts.sort()
            row[name] = round(ts[len(ts) // 2] * 1e6, 1)
            dev.memcpy(region, got.ctypes.data, got.nbytes, 0, None, True)
            row[name + "_mismatches"] = int(dev.synth_verify(region, shape, off, shp, 4,
                                                             bench.SEED))
        print(json.dumps(row), file=sys.stderr, flush=True)
        res["rounds"].append(row)
    out = dev.malloc(64 ** 3 * 4)
    ts = []
    for k in range(reps + 20):
        t0 = time.perf_counter()
        dev.array_read(meta, [(shard, size)], off, shp, out, A.ZH_SRC_DEVICE | A.ZH_OUT_DEVICE)
        if k >= 20:
            ts.append(time.perf_counter() - t0)
    ts.sort()
    res["device_resident_us"] = round(ts[len(ts) // 2] * 1e6, 1)
finally:
    shutil.rmtree(base, ignore_errors=True)
print(json.dumps(res))
json.dump(res, open(out_path, "w"), indent=1)
