#!/usr/bin/env python3
"""The JNI shim's critical-section policy measured (round 4): BASELINE.md §3's sub-shard read
([1,1024,1024,512] of one c4-format 1x1024^3 uint32 shard: the index + 2 GiB of referenced
payload in 64 MiB ranges) through arrayReadPieces under the fake JVM (tests/jni, no copy mode:
the arrays are handed out in place, as HotSpot does), at several ZH_JNI_SLAB_MB caps.  Per cap:
wall time of the call, the number of critical windows and the longest one (the time a GC
locker would defer collections).  The library's one-call read of the same pieces (the ctypes
form, tests/helpers.py jni_read) is the reference output; every shim output must equal it; the
65536 MiB cap is the unbounded (one window) call.  usage: jni_window_lab.py <out.json>"""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "zarr-java_amd"), os.path.join(ROOT, "oracle"),
          os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402

from helpers import jni_fetch, jni_read  # noqa: E402
from jni_harness import FakeJVM  # noqa: E402
from zarrhip import _abi as A  # noqa: E402
from zarrhip._lib import DeviceContext, lib  # noqa: E402


def main(out_path):
    dev = DeviceContext(0)
    shape = [1, 1024, 1024, 1024]
    meta = A.make_meta(shape, shape, 4, endian=A.ZH_ENDIAN_BIG, sharded=True,
                       inner_chunk_shape=[1, 32, 32, 32], transpose_order=[0, 3, 2, 1])
    nel = 1 << 30
    src = dev.malloc(nel * 4)
    bound = lib().zh_array_encoded_bound(C.byref(meta))
    dst = dev.malloc(bound)
    dev.synth_fill(src, nel, 4, 0, 0x5A5A2026)
    dev.sync()
    (nb,) = dev.array_write(meta, src, [0] * 4, shape, [(dst, bound)])
    dev.free(src)
    path = f"/dev/shm/zh_jnilab_{os.getpid()}"
    host = np.empty(nb, np.uint8)
    dev.memcpy(host.ctypes.data, dst, nb, 1)
    dev.free(dst)
    host.tofile(path)
    del host
    res = {"workload": "arrayReadPieces of [1,1024,1024,512] from one c4 shard (2 GiB of "
                       "payload in 64 MiB ranges + the 512 KiB index), host arrays in place",
           "runs": []}
    try:
        off, shp = [0, 0, 0, 0], [1, 1024, 1024, 512]
        fetched = jni_fetch(meta, [path], off, shp, max_run=64 << 20)
        want = jni_read(dev, meta, fetched, off, shp)  # the reference output (ctypes form)
        jvm = FakeJVM(copy_mode=False)
        pa = jvm._pieces_args(fetched)
        out = jvm.output(4, int(np.prod(shp)))
        args = (jvm.longs([dev.h.value]),) + jvm.meta_args(meta) + tuple(pa) + \
            (jvm.longs(off), jvm.longs(shp), out)
        fn = jvm._fn("arrayReadPieces")
        for mb in (64, 128, 256, 512, 1024, 65536):
            os.environ["ZH_JNI_SLAB_MB"] = str(mb)
            jvm.array_of(out, np.uint32, copy=False)[:] = 0  # every cap writes the result anew
            best = None
            for _ in range(3):
                jvm.L.fj_reset_stats()
                t0 = time.perf_counter()
                rc = fn(C.c_void_p(jvm.env), None, *map(C.c_void_p, args))
                dt = time.perf_counter() - t0
                assert rc == 0 and jvm.exception() is None
                s = jvm.stats()
                if best is None or dt < best[0]:
                    best = (dt, s.windows, s.max_window_ns, s.total_window_ns)
            got = jvm.array_of(out, np.uint32, copy=False).reshape(shp)
            ok = bool(np.array_equal(got, want))
            jvm.check_rules()
            r = {"slab_mb": mb, "ms": round(1e3 * best[0], 1), "windows": best[1],
                 "max_window_ms": round(best[2] / 1e6, 1),
                 "gib_per_s": round(2.0 / best[0], 2), "equal_to_library_read": ok}
            print(json.dumps(r), flush=True)
            res["runs"].append(r)
            assert ok
    finally:
        os.unlink(path)
    json.dump(res, open(out_path, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main(sys.argv[1])
