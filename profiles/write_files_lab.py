#!/usr/bin/env python3
"""zh_array_write_files stages (DESIGN §1 "Reads straight from a FilesystemStore", write side):
one c4 shard region [1,1024,1024,1024] (4 GiB of uint32) written into a FilesystemStore on
/dev/shm, from a pageable host array, a page-locked one, and device memory (no H2D), with the
copy lanes at 6 and 12; the encode alone (zh_array_write device to device) and the region's H2D
alone for the split.  Min of R runs, every file compared with the first.  One JSON object.
usage: write_files_lab.py out.json [reps]"""
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
shape = [1, 1024, 1024, 1024]
meta = A.make_meta(shape, [1, 1024, 1024, 1024], 4, endian=A.ZH_ENDIAN_BIG, sharded=True,
                   inner_chunk_shape=[1, 32, 32, 32], transpose_order=[0, 3, 2, 1],
                   index_crc32c=True)
nel = 1 << 30
d_region = dev.malloc(nel * 4)
dev.synth_fill(d_region, nel, 4, 0, bench.SEED)
host = np.empty(nel, np.uint32)
dev.memcpy(host.ctypes.data, d_region, nel * 4, 1, None, True)
d = f"/dev/shm/zh_wlab_{os.getpid()}"
os.makedirs(d, exist_ok=True)
res = {"reps": reps, "runs": []}
ref = None


def one(name, src, flags, env=None):
    global ref
    for k, v in (env or {}).items():
        os.environ[k] = v
    ts = []
    for r in range(reps):
        p = os.path.join(d, f"{name}_{r}", "c", "0", "0", "0", "0")
        t0 = time.perf_counter()
        sizes = dev.array_write_files(meta, src, [0, 0, 0, 0], shape, [p], flags)
        ts.append(time.perf_counter() - t0)
        b = np.fromfile(p, np.uint8)
        if ref is None:
            ref = b
        same = bool(b.size == ref.size and np.array_equal(b, ref))
        shutil.rmtree(os.path.join(d, f"{name}_{r}"), ignore_errors=True)
    for k in (env or {}):
        os.environ.pop(k, None)
    t = min(ts)
    rec = {"case": name, "env": env or {}, "ms_min": round(t * 1e3, 1),
           "GiBps_in": round(nel * 4 / t / 2 ** 30, 2), "file_bytes": int(sizes[0]),
           "file_same": same}
    print(json.dumps(rec), file=sys.stderr, flush=True)
    res["runs"].append(rec)


try:
    # the split: H2D of the region alone (pageable), the encode alone (device to device)
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        dev.memcpy(d_region, host.ctypes.data, nel * 4, 0, None, True)
        t.append(time.perf_counter() - t0)
    res["h2d_pageable_ms"] = round(min(t) * 1e3, 1)
    cap = 4 * nel + 16 * 32768 + 4
    d_out = dev.malloc(cap)
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        dev.array_write(meta, d_region, [0] * 4, shape, [(d_out, cap)])
        t.append(time.perf_counter() - t0)
    res["encode_device_ms"] = round(min(t) * 1e3, 1)
    nb = dev.array_write(meta, d_region, [0] * 4, shape, [(d_out, cap)])[0]
    pin = dev.malloc_pinned(nb)
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        dev.memcpy(pin, d_out, nb, 1, None, True)
        t.append(time.perf_counter() - t0)
    res["d2h_pinned_ms"] = round(min(t) * 1e3, 1)
    # the file write alone from page-locked memory (one thread, then 6 in parallel)
    f = os.path.join(d, "raw")
    buf = (np.ctypeslib.as_array((__import__("ctypes").c_uint8 * nb).from_address(pin)))
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        with open(f, "wb") as fh:
            fh.write(memoryview(buf))
        t.append(time.perf_counter() - t0)
        os.remove(f)
    res["file_write_1thread_ms"] = round(min(t) * 1e3, 1)
    dev.free_pinned(pin)
    dev.free(d_out)
    one("host_pageable", host.ctypes.data, 0)
    one("host_pageable_12", host.ctypes.data, 0, {"ZH_PIPE_THREADS": "12"})
    one("device_src", d_region, A.ZH_SRC_DEVICE)
    dev.host_register(host.ctypes.data, host.nbytes)
    one("host_pinned", host.ctypes.data, 0)
    dev.host_unregister(host.ctypes.data)
    # two shards (8 GiB in, two files written by the lanes together)
    meta2 = A.make_meta([1, 1024, 1024, 2048], [1, 1024, 1024, 1024], 4,
                        endian=A.ZH_ENDIAN_BIG, sharded=True, inner_chunk_shape=[1, 32, 32, 32],
                        transpose_order=[0, 3, 2, 1], index_crc32c=True)
    host2 = np.empty((1024, 1024, 2048), np.uint32)
    host2[:, :, :1024] = host.reshape(1024, 1024, 1024)
    host2[:, :, 1024:] = host.reshape(1024, 1024, 1024)
    ts = []
    for r in range(reps):
        ps = [os.path.join(d, f"two_{r}", "c", "0", "0", "0", str(z_)) for z_ in (0, 1)]
        t0 = time.perf_counter()
        sz = dev.array_write_files(meta2, host2.ctypes.data, [0] * 4, [1, 1024, 1024, 2048], ps)
        ts.append(time.perf_counter() - t0)
        shutil.rmtree(os.path.join(d, f"two_{r}"), ignore_errors=True)
    rec = {"case": "two_shards_pageable", "ms_min": round(min(ts) * 1e3, 1),
           "GiBps_in": round(host2.nbytes / min(ts) / 2 ** 30, 2), "file_bytes": sz}
    print(json.dumps(rec), file=sys.stderr, flush=True)
    res["runs"].append(rec)
    del host2
finally:
    shutil.rmtree(d, ignore_errors=True)
print(json.dumps(res))
json.dump(res, open(out_path, "w"), indent=1)
