#!/usr/bin/env python3
"""Round 5 lab: does the headline's allocation kind move the decode?  (VERDICT r04 item 6:
the N=1 line now decodes into hipMalloc buffers.)  Half the array (ydiv 2: 48 GiB out, far
beyond the 256 MB MALL) of config argv[1]; output and shard slab each allocated twice — plain
hipMalloc (H) and ZH_MALLOC_SCATTER 1 GiB VMM chunks (S) — and the four (output, slab) pairings
decoded in interleaved rounds in one process; kernel time by HIP events, every output verified.
Writes argv[2] (JSON)."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
from zarrhip import _abi as A  # noqa: E402
from zarrhip._lib import DeviceContext, lib  # noqa: E402

cfg = sys.argv[1]
out_json = sys.argv[2]
dev = DeviceContext(0)
meta = bench.build_meta(A, cfg, 2)
n = meta.ndim
shape = [meta.shape[d] for d in range(n)]
nel = 1
for s in shape:
    nel *= s
nb = nel * 4
L = lib()
coords = bench.all_coords(L, meta)
caps = bench.chunk_capacities(meta, coords)
offs, tot = bench.slab_layout(caps)
kinds = {"H": 0, "S": A.ZH_MALLOC_SCATTER}
outs = {k: dev.malloc(nb, f) for k, f in kinds.items()}
slabs = {k: dev.malloc(tot, f) for k, f in kinds.items()}
dev.synth_fill(outs["H"], nel, 4, 0, bench.SEED)
plans = {}
for k, slab in slabs.items():
    sizes = dev.array_write(meta, outs["H"], [0] * n, shape,
                            [(slab + o, c) for o, c in zip(offs, caps)])
    plans[k] = dev.plan(meta, [(slab + o, s) for o, s in zip(offs, sizes)], [0] * n, shape,
                        A.ZH_SRC_DEVICE | A.ZH_OUT_DEVICE)
    plans[k].set_timing(True)
st = plans["H"].stats()
res = {f"out{o}_slab{s}": [] for o in kinds for s in kinds}
for r in range(6):
    for key in res:
        o, s = key[3], key[-1]
        p = plans[s]
        p.execute(outs[o])
        p.wait()
        p.kernel_time()
        for _ in range(2):
            p.execute(outs[o])
        p.wait()
        kt = p.kernel_time()
        res[key].append(kt["scatter_ms"] / kt["launches"])
        if r == 0:
            bad = dev.synth_verify(outs[o], shape, [0] * n, shape, 4, bench.SEED)
            assert bad == 0, (key, bad)
alg = st["in_bytes"] + st["out_bytes"]
summary = {k: {"kernel_ms_median": round(statistics.median(v), 3),
               "kernel_ms_min": round(min(v), 3),
               "frac_median": round(alg / (statistics.median(v) / 1e3) / 8e12, 4),
               "samples": [round(x, 3) for x in v]} for k, v in res.items()}
rates = {k: round(dev.write_rate(outs[k], nb, 0, 2), 1) for k in kinds}
rec = {"config": cfg, "ydiv": 2, "shape": shape, "alg_bytes": alg, "kinds": {
    "H": "hipMalloc", "S": "ZH_MALLOC_SCATTER (1 GiB VMM chunks, coprime order)"},
    "results": summary, "store_probe_GBps": rates}
json.dump(rec, open(out_json, "w"), indent=1)
print(json.dumps(rec))
