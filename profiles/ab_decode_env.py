#!/usr/bin/env python3
"""Interleaved A/B of decode plan variants selected by environment switches (read at plan
creation), one process, one arena pair (the faster by the store probe takes the writes), the
full array unless YDIV > 1.  Each variant: its own plan over the same shards, HIP-event kernel
time of the scatter launch, output verified against the generator after every timed launch.
usage: ab_decode_env.py CONFIG YDIV ROUNDS VAR=VAL[,VAR=VAL] [VAR=VAL ...]
(one argument per variant; "-" = no switches)"""
import json
import os
import statistics
import sys

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
out, slab, arena = bench.arena_pair(dev, A, max(nb, tot))
dev.synth_fill(out, nel, 4, 0, bench.SEED)
sizes = dev.array_write(meta, out, [0] * n, shape, [(slab + o, c) for o, c in zip(offs, caps)])
plans = {}
for v in variants:
    saved = {}
    for kv in ([] if v == "-" else v.split(",")):
        k, val = kv.split("=")
        saved[k] = os.environ.get(k)
        os.environ[k] = val
    p = dev.plan(meta, [(slab + o, s) for o, s in zip(offs, sizes)], [0] * n, shape,
                 A.ZH_SRC_DEVICE | A.ZH_OUT_DEVICE)
    p.set_timing(True)
    plans[v] = p
    for k, old in saved.items():
        if old is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = old
res = {v: [] for v in variants}
bad = {v: 0 for v in variants}
for v, p in plans.items():  # warm
    p.execute(out)
    p.wait()
    p.kernel_time()
for r in range(rounds):
    for v, p in plans.items():
        dev.memset(out, 0, nb)
        p.execute(out)
        p.wait()
        res[v].append(round(p.kernel_time()["scatter_ms"], 3))
        bad[v] += int(dev.synth_verify(out, shape, [0] * n, shape, 4, bench.SEED))
alg = plans[variants[0]].stats()
alg = alg["in_bytes"] + alg["out_bytes"]
print(json.dumps({"config": cfg, "ydiv": ydiv, "arena": arena,
                  "results": {v: {"ms": ms, "median_ms": statistics.median(ms),
                                  "GiBps": round(nb / (statistics.median(ms) / 1e3) / 2**30, 1),
                                  "TBps": round(alg / (statistics.median(ms) / 1e3) / 1e12, 3)}
                              for v, ms in res.items()},
                  "mismatches": bad}, indent=1), flush=True)
