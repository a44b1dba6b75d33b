#!/usr/bin/env python3
"""Is a freed ZH_MALLOC_SCATTER range safe to reuse?  One scenario per process:
  plain  : allocate n0 chunks, fill, free; allocate n1 chunks, fill (kernel), then check with
           a kernel (synth_verify), a D2H copy and a D2D copy checked by a kernel
  view   : the same, with a view of the first allocation created and freed before its free
  inplace: re-map nothing; allocate, create a view, free the view, allocate a second arena
usage: va_reuse_lab.py SCENARIO CHUNK_MB n0 n1"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "zarr-java_amd"))
import numpy as np  # noqa: E402
from zarrhip import _abi as A  # noqa: E402
from zarrhip._lib import DeviceContext  # noqa: E402

sc, mb, n0, n1 = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
os.environ["ZH_SCATTER_MB"] = str(mb)
dev = DeviceContext(0)
cb = mb << 20
F = A.ZH_MALLOC_SCATTER | A.ZH_MALLOC_REQUIRE
p0 = dev.malloc(n0 * cb, F)
dev.synth_fill(p0, n0 * cb // 4, 4, 0, 1)
if sc == "view":
    v = dev.scatter_view(p0, 1)
    dev.synth_verify(v, [n0 * cb // 4], [0], [n0 * cb // 4], 4, 1)
    dev.free(v)
dev.sync()
dev.free(p0)
p1 = dev.malloc(n1 * cb, F)
nel = n1 * cb // 4
dev.synth_fill(p1, nel, 4, 0, 2)
dev.sync()
k = int(dev.synth_verify(p1, [nel], [0], [nel], 4, 2))
host = np.frombuffer(dev.d2h(p1, min(n1 * cb, 1 << 30)), dtype=np.uint32)
zeros = int(np.count_nonzero(host == 0))
q = dev.malloc(n1 * cb, 0)
dev.memcpy(q, p1, n1 * cb, 2)
d2d = int(dev.synth_verify(q, [nel], [0], [nel], 4, 2))
print(json.dumps({"scenario": sc, "chunk_mb": mb, "n0": n0, "n1": n1, "same_va": p0 == p1,
                  "p0": hex(p0), "p1": hex(p1), "kernel_mismatches": k,
                  "d2h_zero_words": zeros, "d2d_mismatches": d2d,
                  "retire": os.environ.get("ZH_SCATTER_RETIRE", "0")}), flush=True)
