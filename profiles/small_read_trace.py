#!/usr/bin/env python3
"""The bench's small_read (BASELINE configs[0]'s call shape: one-shot zh_array_read of the
unaligned 1x64x64x64 region {0,3,517,501} from a device-resident c4-format shard) repeated,
for a HIP API + kernel trace of where the ~85 us go.  One 1x1024^3 shard (4 GiB) only.
usage: small_read_trace.py [reps]"""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from zarrhip import _abi as A  # noqa: E402
from zarrhip._lib import DeviceContext  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 100
dev = DeviceContext(0)
meta = A.make_meta([1, 1024, 1024, 1024], [1, 1024, 1024, 1024], 4, endian=A.ZH_ENDIAN_BIG,
                   sharded=True, inner_chunk_shape=[1, 32, 32, 32], transpose_order=[0, 3, 2, 1],
                   index_crc32c=True)
shape = [1, 1024, 1024, 1024]
nel = 1 << 30
region = dev.malloc(nel * 4)
dev.synth_fill(region, nel, 4, 0, bench.SEED)
cap = 4 * nel + 16 * 32768 + 4
shard = dev.malloc(cap)
size = dev.array_write(meta, region, [0] * 4, shape, [(shard, cap)])[0]
dev.free(region)
off, shp = [0, 3, 517, 501], [1, 64, 64, 64]
out = dev.malloc(64 ** 3 * 4)
ts = []
for i in range(reps + 10):
    t0 = time.perf_counter()
    dev.array_read(meta, [(shard, size)], off, shp, out, A.ZH_SRC_DEVICE | A.ZH_OUT_DEVICE)
    if i >= 10:
        ts.append(time.perf_counter() - t0)
assert dev.synth_verify(out, shape, off, shp, 4, bench.SEED) == 0
print(f"one-shot 64^3 read, device out: median {statistics.median(ts) * 1e6:.1f} us over {reps}")
