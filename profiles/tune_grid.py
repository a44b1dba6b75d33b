#!/usr/bin/env python3
"""Interleaved A/B tuning of the decode launch shape on one GPU, one process, one data set
(MI355X_MICROARCH.md / cdna_hip_programming.md §5.4 rule 24: perf deltas come from
interleaved rounds in one process).  usage: tune_grid.py CONFIG [rounds]"""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

from zarrhip import _abi as A  # noqa: E402
from zarrhip._lib import DeviceContext  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    grids = [int(g) for g in os.environ.get("TUNE_GRIDS", "32,64,128,192,256,384,512").split(",")]
    nts = [int(x) for x in os.environ.get("TUNE_NT", "0,3").split(",")]
    variants = [int(x) for x in os.environ.get("TUNE_VARIANTS", "0").split(",")]
    dev = DeviceContext(0)
    meta = bench.build_meta(A, cfg)
    n = meta.ndim
    shape = [meta.shape[d] for d in range(n)]
    from zarrhip._lib import lib, i64arr, i32arr
    L = lib()
    cs = [meta.chunk_shape[d] for d in range(n)]
    num = L.zh_compute_chunk_coords(n, i64arr(shape), i32arr(cs), i64arr([0] * n), i64arr(shape), None, 0)
    import ctypes as C
    buf = (C.c_int64 * (num * n))()
    L.zh_compute_chunk_coords(n, i64arr(shape), i32arr(cs), i64arr([0] * n), i64arr(shape), buf, num)
    coords = [tuple(buf[i * n + d] for d in range(n)) for i in range(num)]
    caps = bench.chunk_capacities(meta, coords)
    nel = 1
    for s in shape:
        nel *= s
    mflags = int(os.environ.get("ZH_MALLOC", str(A.ZH_MALLOC_SCATTER)), 0)  # bench's arena
    out = dev.malloc(nel * 4, mflags)
    offs, tot = [], 0
    for c in caps:
        offs.append(tot)
        tot += (c + 255) // 256 * 256
    slab = dev.malloc(tot, mflags)
    dev.synth_fill(out, nel, 4, 0, bench.SEED)
    sizes = dev.array_write(meta, out, [0] * n, shape, [(slab + o, c) for o, c in zip(offs, caps)])
    plans = {}
    for g in grids:
        for nt in nts:
            for v in variants:
                os.environ["ZH_BLOCKS_PER_CU"] = str(g)
                os.environ["ZH_NT"] = str(nt)
                os.environ["ZH_TILE_VARIANT"] = str(v)
                plans[(g, nt, v)] = dev.plan(meta, [(slab + o, s) for o, s in zip(offs, sizes)],
                                             [0] * n, shape, A.ZH_SRC_DEVICE | A.ZH_OUT_DEVICE)
    res = {k: [] for k in plans}
    for k, p in plans.items():  # warm every variant once
        p.execute(out)
        p.wait()
    for r in range(rounds):
        for k, p in plans.items():
            dev.sync()
            t0 = time.perf_counter()
            for _ in range(3):
                p.execute(out)
            p.wait()
            res[k].append((time.perf_counter() - t0) / 3 * 1e3)
        print(f"round {r} done", file=sys.stderr, flush=True)
    bad = {}
    for k, p in plans.items():  # every variant must decode bit-exactly
        dev.memset(out, 0, nel * 4)
        p.execute(out)
        p.wait()
        bad[str(k)] = dev.synth_verify(out, shape, [0] * n, shape, 4, bench.SEED)
    rows = []
    for (g, nt, var), v in sorted(res.items()):
        med = statistics.median(v)
        rows.append({"blocks_per_cu": g, "nt": nt, "tile_variant": var, "median_ms": round(med, 3),
                     "min_ms": round(min(v), 3), "GiB/s": round(nel * 4 / med * 1e3 / 2**30, 1)})
    print(json.dumps({"config": cfg, "rounds": rounds, "malloc_flags": mflags,
                      "verify_mismatches": bad, "results": rows}))


if __name__ == "__main__":
    main()
