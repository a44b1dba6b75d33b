"""Round 5 lab: interleaved A/B of decode plan variants selected by environment switches (read
at plan creation), one process, plain hipMalloc buffers (the headline's allocation), the full
array.  Each variant has its own plan over the same shards; per round every variant runs
`steps` launches, HIP-event kernel time of the scatter launch; the output is verified after
each variant's launches; the wall time per launch (execute × steps + wait) beside it.
usage: python3 profiles/r05/env_ab.py OUT.json CONFIG ROUNDS STEPS VAR=VAL[,VAR=VAL] ...
("-" = no switches).  AB_YDIV divides the array's y extent; AB_OUTS > 1 allocates that many
output buffers (each held while the next is allocated, so each gets other memory) and runs
every variant into each: a switch's effect per placement of the output."""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "zarr-java_amd")]
import bench  # noqa: E402


def main():
    out_path, cfg = sys.argv[1], sys.argv[2]
    rounds, steps = int(sys.argv[3]), int(sys.argv[4])
    variants = sys.argv[5:]
    from zarrhip import _abi as A
    from zarrhip._lib import DeviceContext, lib
    dev = DeviceContext(0)
    ydiv = int(os.environ.get("AB_YDIV", "1"))
    nouts = int(os.environ.get("AB_OUTS", "1"))
    meta = bench.build_meta(A, cfg, ydiv)
    L = lib()
    n = meta.ndim
    shape = [meta.shape[d] for d in range(n)]
    coords = bench.all_coords(L, meta)
    caps = bench.chunk_capacities(meta, coords)
    offs, tot = bench.slab_layout(caps)
    nel = 1
    for s in shape:
        nel *= s
    slab = dev.malloc(max(nel * 4, tot))
    outs = [dev.malloc(nel * 4) for _ in range(nouts)]
    out = outs[0]
    dev.synth_fill(out, nel, 4, 0, bench.SEED)
    sizes = dev.array_write(meta, out, [0] * n, shape,
                            [(slab + o, c) for o, c in zip(offs, caps)])
    sources = [(slab + o, s) for o, s in zip(offs, sizes)]
    flags = A.ZH_SRC_DEVICE | A.ZH_OUT_DEVICE
    plans = {}
    for v in variants:
        saved = {}
        for kv in ([] if v == "-" else v.split(",")):
            k, val = kv.split("=")
            saved[k] = os.environ.get(k)
            os.environ[k] = val
        plans[v] = dev.plan(meta, sources, [0] * n, shape, flags)
        plans[v].set_timing(True)
        for k, old in saved.items():
            if old is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = old
    keys = [f"out{k}:{v}" if nouts > 1 else v for k in range(nouts) for v in variants]
    res = {"config": cfg, "ydiv": ydiv, "outputs": nouts, "steps": steps, "variants": variants,
           "kernel_ms": {key: [] for key in keys}, "step_ms": {key: [] for key in keys}}
    for r in range(rounds):
        row = {}
        for k, o in enumerate(outs):
            for v in variants:
                key = f"out{k}:{v}" if nouts > 1 else v
                p = plans[v]
                p.kernel_time()  # drain earlier timings
                t0 = time.perf_counter()
                for _ in range(steps):
                    p.execute(o)
                p.wait()
                t1 = time.perf_counter()
                kt = p.kernel_time()
                res["kernel_ms"][key].append(round(kt["scatter_ms"] / max(1, kt["launches"]), 3))
                res["step_ms"][key].append(round((t1 - t0) * 1e3 / steps, 3))
                row[key] = [res["kernel_ms"][key][-1], res["step_ms"][key][-1]]
                bad = int(dev.synth_verify(o, shape, [0] * n, shape, 4, bench.SEED))
                assert bad == 0, (key, bad)
        print(json.dumps(row), flush=True)
    res["median_ms"] = {v: statistics.median(x) for v, x in res["kernel_ms"].items()}
    res["median_step_ms"] = {v: statistics.median(x) for v, x in res["step_ms"].items()}
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res["median_ms"]), flush=True)
    print(json.dumps(res["median_step_ms"]), flush=True)


if __name__ == "__main__":
    main()
