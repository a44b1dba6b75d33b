"""zh_plan_set_graph: a device-resident plan replayed as one hipGraph gives the same bytes
as plain execution, re-reads its sources on every replay, recaptures for a new output
buffer, and still reports deferred device errors (the status reset is inside the graph)."""
import numpy as np
import pytest

import oracle as O
from helpers import chunk_coords, encode_oracle, rand_array, shape_of
from zarrhip import _abi as A
from zarrhip._lib import ZhError

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("order", [None, [0, 3, 2, 1]])
def test_graph_replay(dev, order):
    meta = A.make_meta([1, 64, 64, 96], [1, 64, 64, 64], 4, endian=A.ZH_ENDIAN_BIG, sharded=True,
                       inner_chunk_shape=[1, 32, 32, 32], transpose_order=order)
    arr = rand_array(shape_of(meta), 4, seed=81)
    shards = encode_oracle(meta, arr)
    off, shp = [0, 3, 5, 7], [1, 60, 50, 80]
    sel = chunk_coords(meta, off, shp)
    pos = {c: i for i, c in enumerate(chunk_coords(meta, [0] * 4, shape_of(meta)))}
    srcs = [shards[pos[c]] for c in sel]
    want = np.frombuffer(O.array_read(meta, srcs, off, shp), np.uint32).reshape(shp)
    bufs = []
    for s in srcs:
        b = dev.malloc(len(s))
        dev.h2d(b, s)
        bufs.append((b, len(s)))
    nbytes = int(np.prod(shp)) * 4
    outs = [dev.malloc(nbytes) for _ in range(2)]
    plan = dev.plan(meta, bufs, off, shp, A.ZH_SRC_DEVICE | A.ZH_OUT_DEVICE)
    try:
        plan.set_graph(True)
        for k in (0, 0, 1, 0):                   # capture, replay, recapture, recapture
            dev.memset(outs[k], 0, nbytes)
            dev.sync()
            plan.execute(outs[k])
            plan.wait()
            got = np.frombuffer(dev.d2h(outs[k], nbytes), np.uint32).reshape(shp)
            np.testing.assert_array_equal(got, want)
        # corrupt the first shard's index under its crc32c: the replay must report it
        bad = bytearray(srcs[0])
        bad[-10] ^= 0x01
        dev.h2d(bufs[0][0], bytes(bad))
        with pytest.raises(O.OracleError) as eo:
            O.array_read(meta, [bytes(bad)] + srcs[1:], off, shp)
        plan.execute(outs[0])
        with pytest.raises(ZhError) as ed:
            plan.wait()
        assert str(ed.value) == str(eo.value)
        dev.h2d(bufs[0][0], srcs[0])             # restored: clean again
        plan.execute(outs[0])
        plan.wait()
        plan.set_graph(False)
        plan.execute(outs[1])
        plan.wait()
        got = np.frombuffer(dev.d2h(outs[1], nbytes), np.uint32).reshape(shp)
        np.testing.assert_array_equal(got, want)
    finally:
        plan.close()
        for b, _ in bufs:
            dev.free(b)
        for o in outs:
            dev.free(o)
