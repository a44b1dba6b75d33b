#!/usr/bin/env python3
"""zh_array_read_files knobs (DESIGN §1 "Reads straight from a FilesystemStore"): BASELINE.md
§3's sub-shard read [1,1024,1024,512] and the two-shard read [1,1024,1024,1536] of c4 shards
(encoded on the device, written to /dev/shm) into a fresh pageable numpy array, per setting of
the pipeline's in/out lanes (ZH_PIPE_THREADS), ring window (ZH_PIPE_CHUNK_KB) and slab size
(ZH_PIPE_SLAB_KB); min of R reads, every output verified.  Prints one JSON object.
usage: files_lab.py out.json [reps]"""
import json
import os
import shutil
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from zarrhip import _abi as A  # noqa: E402
from zarrhip._lib import DeviceContext  # noqa: E402

out_path = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
dev = DeviceContext(0)
shape = [1, 1024, 1024, 2048]  # two c4 shards along z (the second one full)
meta = A.make_meta(shape, [1, 1024, 1024, 1024], 4, endian=A.ZH_ENDIAN_BIG, sharded=True,
                   inner_chunk_shape=[1, 32, 32, 32], transpose_order=[0, 3, 2, 1],
                   index_crc32c=True)
nel = 1 << 31
region = dev.malloc(nel * 4)
dev.synth_fill(region, nel, 4, 0, bench.SEED)
cap = 4 * (1 << 30) + 16 * 32768 + 4
shards = [dev.malloc(cap) for _ in range(2)]
sizes = dev.array_write(meta, region, [0] * 4, shape, [(s, cap) for s in shards])
d = f"/dev/shm/zh_files_lab_{os.getpid()}"
os.makedirs(d, exist_ok=True)
paths = []
pin = dev.malloc_pinned(max(sizes))
import ctypes as C  # noqa: E402
for i, (s, n) in enumerate(zip(shards, sizes)):
    dev.memcpy(pin, s, n, 1, None, True)
    p = os.path.join(d, f"c{i}")
    with open(p, "wb") as f:
        f.write((C.c_char * n).from_address(pin))
    paths.append(p)
dev.free_pinned(pin)
for s in shards:
    dev.free(s)
res = {"reps": reps, "runs": []}
cases = {"sub_shard": ([0, 0, 0, 512], [1, 1024, 1024, 512], paths[:1]),
         "two_shards": ([0, 0, 0, 0], [1, 1024, 1024, 2048], paths),
         "two_shards_pageable": ([0, 0, 0, 0], [1, 1024, 1024, 2048], None)}
settings = [dict(), dict(ZH_PIPE_THREADS="8"), dict(ZH_PIPE_THREADS="10"),
            dict(ZH_PIPE_CHUNK_KB="32768"), dict(ZH_PIPE_THREADS="8", ZH_PIPE_CHUNK_KB="32768")]
# the generic pipelined read from pageable host memory (the shards read into numpy first)
host = [np.fromfile(p, np.uint8) for p in paths]
try:
    for name, (off, shp, ps) in cases.items():
        ts = {i: [] for i in range(len(settings))}
        bad = 0
        for rnd in range(reps + 1):  # settings interleaved round-robin (drift hits all alike)
            for i, st in enumerate(settings):
                for k, v in st.items():
                    os.environ[k] = v
                for warm in (True, False):  # an untimed read after each switch: a new ring
                    got = np.empty(shp, np.uint32)  # window size re-allocates the rings
                    t0 = time.perf_counter()
                    if ps is None:
                        dev.array_read(meta, [(h.ctypes.data, h.size) for h in host], off, shp,
                                       got.ctypes.data, 0)
                    else:
                        dev.array_read_files(meta, ps, off, shp, got.ctypes.data, 0)
                    if rnd and not warm:
                        ts[i].append(time.perf_counter() - t0)
                    if warm:
                        del got
                for k in st:
                    os.environ.pop(k, None)
                if rnd == reps:
                    dev.memcpy(region, got.ctypes.data, got.nbytes, 0, None, True)
                    bad += int(dev.synth_verify(region, shape, off, shp, 4, bench.SEED))
                nb = got.nbytes
                del got
        for i, st in enumerate(settings):
            t = sorted(ts[i])
            r = {"case": name, "env": st, "ms_min": round(t[0] * 1e3, 1),
                 "ms_median": round(t[len(t) // 2] * 1e3, 1),
                 "GiBps": round(nb / t[0] / 2 ** 30, 2), "verify_mismatches": bad}
            print(json.dumps(r), file=sys.stderr, flush=True)
            res["runs"].append(r)
finally:
    shutil.rmtree(d, ignore_errors=True)
json.dump(res, open(out_path, "w"), indent=1)
print(json.dumps(res))
