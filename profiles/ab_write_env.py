#!/usr/bin/env python3
"""Interleaved A/B of write-path variants selected by environment switches (read per call),
one process: zh_array_write of the region (quarter or full array) into the shard slab, wall
clock around the call (it synchronises).  The slab is the faster of an arena pair (it takes
the writes).  After every timed write the shards are decoded by one fixed plan and checked
against the generator.  usage: ab_write_env.py CONFIG YDIV ROUNDS VAR=VAL[,VAR=VAL] ..."""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from zarrhip import _abi as A  # noqa: E402
from zarrhip._lib import DeviceContext, lib  # noqa: E402

cfg, ydiv, rounds = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
variants = sys.argv[4:]
dev = DeviceContext(0)
meta = bench.build_meta(A, cfg, ydiv)
n = meta.ndim
shape = [meta.shape[d] for d in range(n)]
L = lib()
coords = bench.all_coords(L, meta)
caps = bench.chunk_capacities(meta, coords)
offs, tot = bench.slab_layout(caps)
nel = 1
for s in shape:
    nel *= s
nb = nel * 4
slab, region, arena = bench.arena_pair(dev, A, max(nb, tot))
out = dev.malloc(nb) if ydiv > 1 else None
dev.synth_fill(region, nel, 4, 0, bench.SEED)
dsts = [(slab + o, c) for o, c in zip(offs, caps)]


def with_env(v, fn):
    saved = {}
    for kv in ([] if v == "-" else v.split(",")):
        k, val = kv.split("=")
        saved[k] = os.environ.get(k)
        os.environ[k] = val
    try:
        return fn()
    finally:
        for k, old in saved.items():
            if old is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = old


def write():
    dev.sync()
    t0 = time.perf_counter()
    sz = dev.array_write(meta, region, [0] * n, shape, dsts)
    return (time.perf_counter() - t0) * 1e3, sz


sizes = None
for v in variants:
    _, sizes = with_env(v, write)
plan = dev.plan(meta, [(slab + o, s) for o, s in zip(offs, sizes)], [0] * n, shape,
                A.ZH_SRC_DEVICE | A.ZH_OUT_DEVICE)
res = {v: [] for v in variants}
bad = {v: 0 for v in variants}
for r in range(rounds):
    for v in variants:
        ms, sz = with_env(v, write)
        res[v].append(round(ms, 3))
        if out is not None:  # quarter arrays: decode into a third buffer and check
            plan.execute(out)
            plan.wait()
            bad[v] += int(dev.synth_verify(out, shape, [0] * n, shape, 4, bench.SEED)) + \
                int(sz != sizes)
        else:
            bad[v] += int(sz != sizes)
    print(f"round {r}: " + ", ".join(f"{v} {res[v][-1]} ms" for v in variants), file=sys.stderr,
          flush=True)
print(json.dumps({"config": cfg, "ydiv": ydiv, "arena": arena,
                  "results": {v: {"ms": ms, "median_ms": statistics.median(ms),
                                  "GiBps": round(nb / (statistics.median(ms) / 1e3) / 2**30, 1)}
                              for v, ms in res.items()},
                  "mismatches": bad}, indent=1), flush=True)
