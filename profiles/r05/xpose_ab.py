"""Round 5 lab: c3's lane-exchange row kernel (rows_xpose_kernel) with the next step's loads
issued before this step's stores (ZH_XPOSE_PF=1) or after them (0), interleaved in one
process over one plan of the full c3 array (bench.py's setup), every output verified.
usage: python3 profiles/r05/xpose_ab.py OUT.json [rounds] [steps]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "zarr-java_amd")]
import bench  # noqa: E402


def main():
    out_path = sys.argv[1]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    from zarrhip import _abi as A
    from zarrhip._lib import DeviceContext, lib
    dev = DeviceContext(0)
    meta = bench.build_meta(A, os.environ.get("AB_CONFIG", "c3"), 1)
    L = lib()
    shape = [meta.shape[d] for d in range(meta.ndim)]
    coords = bench.all_coords(L, meta)
    caps = bench.chunk_capacities(meta, coords)
    offs, tot = bench.slab_layout(caps)
    nel = 1
    for s in shape:
        nel *= s
    out = dev.malloc(nel * 4)
    slab = dev.malloc(tot)
    dev.synth_fill(out, nel, 4, 0, bench.SEED)
    sizes = dev.array_write(meta, out, [0] * len(shape), shape,
                            [(slab + o, c) for o, c in zip(offs, caps)])
    sources = [(slab + o, s) for o, s in zip(offs, sizes)]
    flags = A.ZH_SRC_DEVICE | A.ZH_OUT_DEVICE
    res = {"config": os.environ.get("AB_CONFIG", "c3"), "steps": steps, "rounds": []}
    for r in range(rounds):
        row = {}
        for pf in ("1", "0"):
            os.environ["ZH_XPOSE_PF"] = pf
            plan = dev.plan(meta, sources, [0] * len(shape), shape, flags)
            plan.execute(out)
            plan.wait()
            plan.set_timing(True)
            dev.sync()
            t0 = time.perf_counter()
            for _ in range(steps):
                plan.execute(out)
            plan.wait()
            dev.sync()
            dt = (time.perf_counter() - t0) / steps
            kt = plan.kernel_time()
            bad = int(dev.synth_verify(out, shape, [0] * len(shape), shape, 4, bench.SEED))
            assert bad == 0, (pf, bad)
            dev.memset(out, 0, nel * 4)
            plan.close()
            row[f"pf{pf}_ms"] = round(dt * 1e3, 3)
            row[f"pf{pf}_kernel_ms"] = round(kt["scatter_ms"], 3)
        res["rounds"].append(row)
        print(json.dumps(row), flush=True)
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
