"""Host-terminated read lab (round 3): where the time of a host-in / host-out zh_array_read
goes, and how the pipelined path (zh_pipeline.cpp) behaves under its switches.

Workload: BASELINE.md §3's sub-shard read, region [1,1024,1024,512] of one c4-format 1×1024³
uint32 shard (encoded on the device from the synthetic generator), 2 GiB of referenced payload
in, 2 GiB out; and the 4-shard host-inclusive region [1,1024,4096,1024] (16 GiB each way).
Sources: the shard in page-locked or pageable host memory (whole objects: the library stages
only the referenced ranges), or the pieces form from pinned staging.  Outputs: page-locked,
pageable touched once (a warm heap), pageable fresh (np.empty per call).  Every variant's
output is verified on the device against the generator.  Prints one JSON object."""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zarr-java_amd"))
from zarrhip import _abi as A  # noqa: E402
from zarrhip._lib import DeviceContext, ShardSource, lib, shard_ranges  # noqa: E402

SEED = 0x5A5A2026
GiB = 1 << 30


def tmed(fn, reps):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return ts[0], ts[len(ts) // 2]


def main():
    reps = int(os.environ.get("LAB_REPS", "5"))
    dev = DeviceContext(0)
    L = lib()
    shape = [1, 1024, 1024, 1024]
    meta = A.make_meta(shape, shape, 4, endian=A.ZH_ENDIAN_BIG, sharded=True,
                       inner_chunk_shape=[1, 32, 32, 32], transpose_order=[0, 3, 2, 1])
    nel = 1 << 30
    src = dev.malloc(nel * 4)
    bound = L.zh_array_encoded_bound(C.byref(meta))
    dshard = dev.malloc(bound)
    dev.synth_fill(src, nel, 4, 0, SEED)
    dev.sync()
    (nb,) = dev.array_write(meta, src, [0] * 4, shape, [(dshard, bound)])
    chk = src  # device scratch for the checks
    pin_shard = dev.malloc_pinned(nb)
    dev.memcpy(pin_shard, dshard, nb, 1)
    page_shard = np.empty(nb, np.uint8)
    C.memmove(page_shard.ctypes.data, pin_shard, nb)
    off, shp = [0, 0, 0, 512], [1, 1024, 1024, 512]
    obytes = 1 << 31
    pin_out = dev.malloc_pinned(obytes)
    warm_out = np.ones(obytes, np.uint8)
    res = {"workload": "sub-shard [1,1024,1024,512] of a c4 1x1024^3 shard: 2 GiB payload in, "
                       "2 GiB out", "reps": reps, "variants": {}}

    def check(ptr):
        dev.memcpy(chk, ptr, obytes, 0)
        return int(dev.synth_verify(chk, shape, off, shp, 4, SEED))

    def run(name, srcs, outp_fn, pieces=None, env=None):
        old = {}
        for k, v in (env or {}).items():
            old[k] = os.environ.get(k)
            os.environ[k] = v
        try:
            holder = {}

            def call():
                outp = outp_fn()
                holder["o"] = outp
                if pieces is not None:
                    dev.array_read_pieces(meta, pieces, off, shp, outp if isinstance(outp, int)
                                          else outp.ctypes.data, 0)
                else:
                    dev.array_read(meta, srcs, off, shp, outp if isinstance(outp, int)
                                   else outp.ctypes.data, 0)
            call()  # first call: rings, cached device blocks
            tmin, tmedian = tmed(call, reps)
            o = holder["o"]
            bad = check(o if isinstance(o, int) else o.ctypes.data)
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        r = {"ms_min": round(tmin * 1e3, 1), "ms_median": round(tmedian * 1e3, 1),
             "GiBps_min": round(obytes / tmin / GiB, 2), "verify_mismatches": bad,
             "env": env or {}}
        res["variants"][name] = r
        print(name, json.dumps(r), file=sys.stderr, flush=True)

    pin_src = [(pin_shard, nb)]
    page_src = [(page_shard.ctypes.data, nb)]
    run("pinned_in_pinned_out", pin_src, lambda: pin_out)
    run("pinned_in_warm_out", pin_src, lambda: warm_out)
    run("pinned_in_fresh_out", pin_src, lambda: np.empty(obytes, np.uint8))
    run("pageable_in_warm_out", page_src, lambda: warm_out)
    run("pageable_in_fresh_out", page_src, lambda: np.empty(obytes, np.uint8))
    run("one_plan_pinned_in_pinned_out", pin_src, lambda: pin_out, env={"ZH_PIPE": "0"})
    run("one_plan_pageable_in_warm_out", page_src, lambda: warm_out, env={"ZH_PIPE": "0"})
    for k in ("4", "8", "12"):
        run(f"pageable_in_warm_out_threads{k}", page_src, lambda: warm_out,
            env={"ZH_PIPE_THREADS": k})
    for kb in ("65536", "262144"):
        run(f"pageable_in_warm_out_slab{int(kb) >> 10}M", page_src, lambda: warm_out,
            env={"ZH_PIPE_SLAB_KB": kb})
    # the pieces form, staged like the JNI does (index + ranges in pinned staging)
    isz = L.zh_shard_index_size(C.byref(meta))
    idx = bytes((C.c_char * isz).from_address(pin_shard + nb - isz))
    rs = shard_ranges(meta, idx, nb, [0, 0, 0, 512], [1, 1024, 1024, 1024], 64 << 20)
    tot = isz + sum(x for _, x in rs)
    base = dev.host_staging(tot)
    C.memmove(base, pin_shard + nb - isz, isz)
    pos, ps = isz, []
    for o, x in rs:
        C.memmove(base + pos, pin_shard + o, x)
        ps.append((o, x, base + pos, x))
        pos += x
    pieces = [ShardSource(base, isz, nb, ps)]
    run("pieces_pinned_in_pinned_out", None, lambda: pin_out, pieces=pieces)
    run("pieces_pinned_in_warm_out", None, lambda: warm_out, pieces=pieces)
    # the pieces form as the JNI passes it: each piece its own pageable (Java heap) array
    heap = [np.frombuffer(bytes((C.c_char * x).from_address(pin_shard + o)), np.uint8).copy()
            for o, x in rs]
    hidx = np.frombuffer(idx, np.uint8).copy()
    hp = [ShardSource(hidx.ctypes.data, isz, nb,
                      [(o, x, h.ctypes.data, x) for (o, x), h in zip(rs, heap)])]
    run("pieces_pageable_in_warm_out", None, lambda: warm_out, pieces=hp)
    run("pieces_pageable_in_fresh_out", None, lambda: np.empty(obytes, np.uint8), pieces=hp)
    dev.free_pinned(pin_out)
    dev.free_pinned(pin_shard)
    dev.free(dshard)
    dev.free(src)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
