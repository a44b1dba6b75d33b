#!/usr/bin/env python3
"""PCIe ceiling for the host-terminated read (DESIGN §4 "Host-inclusive rate"): page-locked
host ↔ device copies of N × 128 MiB slabs (the pipeline's slab size), one direction alone and
both directions at once on two streams, min of R runs.  Prints one JSON object (GB/s, 1e9)."""
import json
import sys
import time

import torch

n_slabs = int(sys.argv[1]) if len(sys.argv) > 1 else 32
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
slab = 128 << 20
dev = torch.device("cuda:0")
h_in = [torch.empty(slab, dtype=torch.uint8).pin_memory() for _ in range(4)]
h_out = [torch.empty(slab, dtype=torch.uint8).pin_memory() for _ in range(4)]
d_in = [torch.empty(slab, dtype=torch.uint8, device=dev) for _ in range(4)]
d_out = [torch.empty(slab, dtype=torch.uint8, device=dev) for _ in range(4)]
s_h2d = torch.cuda.Stream(dev)
s_d2h = torch.cuda.Stream(dev)


def run(h2d, d2h):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(n_slabs):
        if h2d:
            with torch.cuda.stream(s_h2d):
                d_in[i % 4].copy_(h_in[i % 4], non_blocking=True)
        if d2h:
            with torch.cuda.stream(s_d2h):
                h_out[i % 4].copy_(d_out[i % 4], non_blocking=True)
    torch.cuda.synchronize()
    return time.perf_counter() - t0


res = {}
for name, h2d, d2h in (("h2d", True, False), ("d2h", False, True), ("both", True, True)):
    run(h2d, d2h)
    best = min(run(h2d, d2h) for _ in range(rounds))
    gb = n_slabs * slab / 1e9
    res[name] = {"s": round(best, 4), "GBps_per_direction": round(gb / best, 2)}
    print(name, res[name], file=sys.stderr, flush=True)
print(json.dumps({"slab_bytes": slab, "slabs": n_slabs, "rounds": rounds, "results": res}),
      flush=True)
