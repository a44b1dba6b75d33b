"""Round 5 lab: the small read (BASELINE configs[0]'s call shape, bench.small_read) under two
settings of one switch read at plan creation, interleaved in one process over one c4-format
array (y/4: the region's shard is the same 4 GiB c4 shard).  Median of `reps` one-shot reads
per setting and round.  First use: the index crc32c on a side stream (ZH_CRC_SIDE, since
removed); then the index crc32c inside the slow kernel's launch (ZH_IDX_CRC_FUSE=1; the first run named it ZH_CRC_FUSE) or on its own
ahead of the resolve kernel (0).
usage: python3 profiles/r05/small_ab.py OUT.json [rounds] [reps] [VAR]"""
import json
import os
import statistics
import sys
import time
import ctypes as C

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "zarr-java_amd")]
import bench  # noqa: E402


def main():
    out_path = sys.argv[1]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 200
    var = sys.argv[4] if len(sys.argv) > 4 else "ZH_IDX_CRC_FUSE"
    from zarrhip import _abi as A
    from zarrhip._lib import DeviceContext, lib
    dev = DeviceContext(0)
    meta = bench.build_meta(A, "c4", 4)
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
    off, shp = [0, 3, 517, 501], [1, 64, 64, 64]
    nb = 4 * 64 ** 3
    dout = dev.malloc(nb)
    host = (C.c_char * nb)()
    res = {"region_offset": off, "region_shape": shp, "reps": reps, "switch": var, "rounds": []}
    for r in range(rounds):
        row = {}
        for side in ("1", "0"):
            os.environ[var] = side
            for tag, dst, flags in (("device_out_us", dout, A.ZH_SRC_DEVICE | A.ZH_OUT_DEVICE),
                                    ("host_out_us", C.addressof(host), A.ZH_SRC_DEVICE)):
                ts = []
                for i in range(reps + 20):
                    t0 = time.perf_counter()
                    dev.array_read(meta, src, off, shp, dst, flags)
                    if i >= 20:
                        ts.append(time.perf_counter() - t0)
                row[f"{var}={side}:{tag}"] = round(statistics.median(ts) * 1e6, 1)
                if dst != dout:
                    dev.memcpy(dout, dst, nb, 0, None, True)
                bad = int(dev.synth_verify(dout, shape, off, shp, 4, bench.SEED))
                assert bad == 0, (side, tag, bad)
        res["rounds"].append(row)
        print(json.dumps(row), flush=True)
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
