#!/usr/bin/env python3
"""Interleaved A/B of the lane-exchange row kernel (rows_xpose_kernel) against the grouped row
kernels, one process, one quarter-size array (1x1024x4096x1536 uint32, 24 GiB):
  write:  ZH_ENC_XPOSE=0 (rows_group_kernel, G = 2) vs 1 (8 chunks, 1 KiB on both sides)
  decode: ZH_DEC_RGROUP=0 (decode_rows_kernel) vs 8 (rows_xpose_kernel, decode direction)
Write time = wall clock around zh_array_write (it synchronises); decode = HIP-event kernel
time of the scatter launch.  Every write variant's shards are decoded and every decode
variant's output is checked against the generator.  usage: ab_xpose.py [config] [rounds]"""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from zarrhip import _abi as A  # noqa: E402
from zarrhip._lib import DeviceContext, lib  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
dev = DeviceContext(0)
meta = bench.build_meta(A, cfg, 4)
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
region = dev.malloc(nb, A.ZH_MALLOC_SCATTER)
slab = dev.malloc(tot, A.ZH_MALLOC_SCATTER)
out = dev.malloc(nb, A.ZH_MALLOC_SCATTER)
dev.synth_fill(region, nel, 4, 0, bench.SEED)
dsts = [(slab + o, c) for o, c in zip(offs, caps)]
res = {}
bad = {}


def write(xp):
    os.environ["ZH_ENC_XPOSE"] = str(xp)
    dev.sync()
    t0 = time.perf_counter()
    sizes = dev.array_write(meta, region, [0] * n, shape, dsts)
    return (time.perf_counter() - t0) * 1e3, sizes


def decode(plan):
    plan.kernel_time()
    plan.execute(out)
    plan.wait()
    return plan.kernel_time()["scatter_ms"]


sizes = None
for xp in (0, 1):  # warm both
    _, sizes = write(xp)
plans = {}
for rg in (0, 8):
    os.environ["ZH_DEC_RGROUP"] = str(rg)
    p = dev.plan(meta, [(slab + o, s) for o, s in zip(offs, sizes)], [0] * n, shape,
                 A.ZH_SRC_DEVICE | A.ZH_OUT_DEVICE)
    p.set_timing(True)
    decode(p)
    plans[rg] = p
for r in range(rounds):
    for xp in (0, 1):
        ms, sz = write(xp)
        res.setdefault(f"write_xpose{xp}", []).append(round(ms, 3))
        dev.memset(out, 0, nb)
        decode(plans[0])
        bad[f"write_xpose{xp}"] = bad.get(f"write_xpose{xp}", 0) + int(
            dev.synth_verify(out, shape, [0] * n, shape, 4, bench.SEED)) + int(sz != sizes)
    for rg in (0, 8):
        dev.memset(out, 0, nb)
        ms = decode(plans[rg])
        res.setdefault(f"decode_rgroup{rg}", []).append(round(ms, 3))
        bad[f"decode_rgroup{rg}"] = bad.get(f"decode_rgroup{rg}", 0) + int(
            dev.synth_verify(out, shape, [0] * n, shape, 4, bench.SEED))
summ = {k: {"ms": v, "median_ms": statistics.median(v),
            "GiBps": round(nb / (statistics.median(v) / 1e3) / 2**30, 1)} for k, v in res.items()}
print(json.dumps({"config": cfg, "quarter": True, "results": summ, "mismatches": bad}, indent=1))
