"""Round 5 lab: mid-size reads into pageable host memory (a Java array's case between the
small-output landing buffer, <= 4 MiB, and the pipelined host read, >= ZH_PIPE_MIN_KB = 64 MiB
by default): one c4-format shard on the device, regions of 8-48 MiB, settings of
ZH_PIPE_MIN_KB interleaved in one process; median wall time of `reps` one-shot reads each.
MID_BIG=1: regions of 64-512 MiB, the pipelined read (64 MiB) against one plan (1 GiB);
MID_HUGE=1: 1 and 2 GiB against 4 GiB; MID_SMALL=1: 0.5-4 MiB with ZH_HOUT_PIN 1 / 0; MID_VAR: the switch (ZH_PIPE_DOUT_MIN_KB since it
exists: device sources with a host output).
usage: python3 profiles/r05/mid_ab.py OUT.json [rounds] [reps]"""
import ctypes as C
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "zarr-java_amd")]
import bench  # noqa: E402


def main():
    out_path = sys.argv[1]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    from zarrhip import _abi as A
    from zarrhip._lib import DeviceContext, lib
    dev = DeviceContext(0)
    meta = bench.build_meta(A, "c4", 4)  # y/4: the region's shard is one 4 GiB c4 shard
    L = lib()
    shape = [meta.shape[d] for d in range(meta.ndim)]
    coords = bench.all_coords(L, meta)
    caps = bench.chunk_capacities(meta, coords)
    offs, tot = bench.slab_layout(caps)
    nel = 1
    for s in shape:
        nel *= s
    region = dev.malloc(nel * 4)
    slab = dev.malloc(tot)
    dev.synth_fill(region, nel, 4, 0, bench.SEED)
    sizes = dev.array_write(meta, region, [0] * len(shape), shape,
                            [(slab + o, c) for o, c in zip(offs, caps)])
    sources = [(slab + o, s) for o, s in zip(offs, sizes)]
    pos = {c: i for i, c in enumerate(coords)}
    src = [sources[pos[(0, 0, 0, 0)]]]
    big = os.environ.get("MID_BIG") == "1"  # 64-512 MiB: pipelined (64 MiB) vs one plan
    shapes = {"8MiB": [1, 64, 128, 256], "16MiB": [1, 128, 128, 256], "32MiB": [1, 128, 256, 256],
              "48MiB": [1, 192, 256, 256]}
    settings = ["65536", "16384", "4096"]
    var = os.environ.get("MID_VAR", "ZH_PIPE_MIN_KB")
    if big:
        shapes = {"64MiB": [1, 256, 256, 256], "128MiB": [1, 256, 512, 256],
                  "256MiB": [1, 512, 512, 256], "512MiB": [1, 512, 512, 512]}
        settings = ["65536", "1048576"]
    if os.environ.get("MID_SMALL") == "1":  # 0.5-4 MiB: the pinned landing buffer on / off
        shapes = {"512KiB": [1, 32, 64, 64], "1MiB": [1, 64, 64, 64], "2MiB": [1, 64, 64, 128],
                  "4MiB": [1, 64, 128, 128]}
        settings = ["1", "0"]  # (a third form, 2, page-locked the caller's pages; removed)
        var = "ZH_HOUT_PIN"
    huge = os.environ.get("MID_HUGE") == "1"
    if huge:  # 1-2 GiB: pipelined (64 MiB) vs one plan (4 GiB)
        shapes = {"1GiB": [1, 512, 1024, 512], "2GiB": [1, 1024, 1024, 512]}
        settings = ["65536", "4194304"]
    cap = max(4 * s[1] * s[2] * s[3] for s in shapes.values())
    host = (C.c_char * cap)()
    dout = dev.malloc(cap)
    res = {"reps": reps, "settings": settings, "rounds": []}
    for r in range(rounds):
        row = {}
        for name, shp in shapes.items():
            nb = 4 * shp[1] * shp[2] * shp[3]
            off = [0, 0, 0, 0] if huge else [0, 1, 3, 5]  # inside the first shard
            for st in settings:
                os.environ[var] = st
                ts = []
                for i in range(reps + 3):
                    t0 = time.perf_counter()
                    dev.array_read(meta, src, off, shp, C.addressof(host), A.ZH_SRC_DEVICE)
                    if i >= 3:
                        ts.append(time.perf_counter() - t0)
                ms = statistics.median(ts) * 1e3
                row[f"{name}:min_kb={st}"] = [round(ms, 3), round(nb / 2**30 / (ms / 1e3), 2)]
                dev.memcpy(dout, C.addressof(host), nb, 0, None, True)
                bad = int(dev.synth_verify(dout, shape, off, shp, 4, bench.SEED))
                assert bad == 0, (name, st, bad)
        res["rounds"].append(row)
        print(json.dumps(row), flush=True)
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
