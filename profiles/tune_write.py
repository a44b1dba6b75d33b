#!/usr/bin/env python3
"""Interleaved A/B tuning of the one-pass write path (zh_array_write) on one GPU, one
process, one source region: cache policy of the encode-view fast kernel (ZH_ENC_NT),
rows in flight per lane (ZH_ENC_DEEP, uint32 rows), golden-ratio visit order (ZH_ITEM_PERM),
workgroups per CU (ZH_ENC_GROUP: a grouped short-row kernel, measured and removed:
profiles/r01/experiments/tune_write_group_c3.json).  The knobs are read per call, so every variant writes the same data
into the same buffers.  Every variant's shards are decoded and checked against the generator.
usage: tune_write.py CONFIG [rounds]"""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

from zarrhip import _abi as A  # noqa: E402
from zarrhip._lib import DeviceContext  # noqa: E402


def variants():
    nts = [int(x) for x in os.environ.get("TUNE_NT", "0,1,2,3").split(",")]
    deeps = [int(x) for x in os.environ.get("TUNE_DEEP", "0,1").split(",")]
    perms = [int(x) for x in os.environ.get("TUNE_PERM", "0,1").split(",")]
    grids = [int(x) for x in os.environ.get("TUNE_GRIDS", "256").split(",")]
    groups = [int(x) for x in os.environ.get("TUNE_GROUP", "0").split(",")]
    return [(nt, d, p, g, gr) for nt in nts for d in deeps for p in perms for g in grids
            for gr in groups]


def set_env(v):
    nt, deep, perm, g, group = v
    os.environ["ZH_ENC_GROUP"] = str(group)
    os.environ["ZH_ENC_NT"] = str(nt)
    os.environ["ZH_ENC_DEEP"] = str(deep)
    os.environ["ZH_ITEM_PERM"] = str(perm)
    os.environ["ZH_BLOCKS_PER_CU"] = str(g)


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    dev = DeviceContext(0)
    meta = bench.build_meta(A, cfg)
    n = meta.ndim
    shape = [meta.shape[d] for d in range(n)]
    import ctypes as C
    from zarrhip._lib import lib, i64arr, i32arr
    L = lib()
    cs = [meta.chunk_shape[d] for d in range(n)]
    num = L.zh_compute_chunk_coords(n, i64arr(shape), i32arr(cs), i64arr([0] * n), i64arr(shape), None, 0)
    buf = (C.c_int64 * (num * n))()
    L.zh_compute_chunk_coords(n, i64arr(shape), i32arr(cs), i64arr([0] * n), i64arr(shape), buf, num)
    coords = [tuple(buf[i * n + d] for d in range(n)) for i in range(num)]
    caps = bench.chunk_capacities(meta, coords)
    nel = 1
    for s in shape:
        nel *= s
    region = dev.malloc(nel * 4)
    offs, tot = [], 0
    for c in caps:
        offs.append(tot)
        tot += (c + 255) // 256 * 256
    slab = dev.malloc(tot)
    dev.synth_fill(region, nel, 4, 0, bench.SEED)
    dsts = [(slab + o, c) for o, c in zip(offs, caps)]
    vs = variants()
    res = {v: [] for v in vs}
    for v in vs:  # warm every variant once
        set_env(v)
        dev.array_write(meta, region, [0] * n, shape, dsts)
    for r in range(rounds):
        for v in vs:
            set_env(v)
            dev.sync()
            t0 = time.perf_counter()
            for _ in range(3):
                sizes = dev.array_write(meta, region, [0] * n, shape, dsts)
            res[v].append((time.perf_counter() - t0) / 3 * 1e3)
        print(f"round {r} done", file=sys.stderr, flush=True)
    bad = {}
    for v in vs:  # every variant must write shards that decode to the generator (decoded
        set_env(v)  # into the source buffer: three 96 GiB buffers do not fit in HBM)
        dev.synth_fill(region, nel, 4, 0, bench.SEED)
        sizes = dev.array_write(meta, region, [0] * n, shape, dsts)
        p = dev.plan(meta, [(slab + o, s) for o, s in zip(offs, sizes)], [0] * n, shape,
                     A.ZH_SRC_DEVICE | A.ZH_OUT_DEVICE)
        dev.memset(region, 0, nel * 4)
        p.execute(region)
        p.wait()
        p.close()
        bad[str(v)] = dev.synth_verify(region, shape, [0] * n, shape, 4, bench.SEED)
    rows = []
    for (nt, deep, perm, g, group), t in sorted(res.items(), key=lambda kv: statistics.median(kv[1])):
        med = statistics.median(t)
        rows.append({"enc_nt": nt, "enc_deep": deep, "item_perm": perm, "blocks_per_cu": g,
                     "enc_group": group,
                     "median_ms": round(med, 3), "min_ms": round(min(t), 3),
                     "GiB/s": round(nel * 4 / med * 1e3 / 2**30, 1)})
    print(json.dumps({"config": cfg, "rounds": rounds, "verify_mismatches": bad, "results": rows}))


if __name__ == "__main__":
    main()
