"""The oracle's FilesystemStore read (zo_array_read_store): the partial path's per-inner-chunk
range reads (ShardingIndexedCodec.java:253,333-357) and whole-chunk reads
(FilesystemStore.java:49-59) must give the in-memory read's bytes.  This is the CPU
baseline's workload shape (bench.py cpu_baseline)."""
import numpy as np
import pytest

import oracle as O
from helpers import chunk_coords, encode_oracle, rand_array
from zarrhip import _abi as A


def _store(tmp_path, meta, shards, drop=()):
    coords = chunk_coords(meta, [0] * meta.ndim, [meta.shape[d] for d in range(meta.ndim)])
    paths = {}
    for i, (c, b) in enumerate(zip(coords, shards)):
        if b is None or i in drop:
            continue
        p = tmp_path / ("c/" + "/".join(map(str, c)))
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_bytes(b)
        paths[c] = str(p)
    return coords, paths


@pytest.mark.parametrize("sharded,order,loc", [(True, None, A.ZH_INDEX_END),
                                               (True, [0, 3, 2, 1], A.ZH_INDEX_END),
                                               (True, None, A.ZH_INDEX_START),
                                               (False, None, A.ZH_INDEX_END)])
def test_store_read_equals_memory_read(tmp_path, sharded, order, loc):
    shape = [1, 40, 32, 48]
    meta = A.make_meta(shape, [1, 16, 16, 32], 4, endian=A.ZH_ENDIAN_BIG, sharded=sharded,
                       inner_chunk_shape=[1, 8, 8, 8] if sharded else None,
                       transpose_order=order, index_location=loc)
    arr = rand_array(shape, 4, seed=11)
    shards = encode_oracle(meta, arr)
    coords, paths = _store(tmp_path, meta, shards, drop=(3,))
    allc = chunk_coords(meta, [0] * 4, shape)
    pos = {c: i for i, c in enumerate(allc)}
    for off, shp in [([0, 0, 0, 0], shape), ([0, 3, 5, 7], [1, 30, 20, 33]),
                     ([0, 16, 16, 0], [1, 16, 16, 32]), ([0, 17, 1, 2], [1, 5, 6, 7])]:
        sel = chunk_coords(meta, off, shp)
        want = O.array_read(meta, [shards[pos[c]] if pos[c] != 3 else None for c in sel], off,
                            shp)
        got = O.array_read_store(meta, [paths.get(c) for c in sel], off, shp, nthreads=2)
        assert got == want
    full = np.frombuffer(O.array_read_store(meta, [paths.get(c) for c in allc], [0] * 4, shape),
                         np.uint32).reshape(shape)
    c3 = allc[3]
    keep = np.ones(shape, bool)
    keep[tuple(slice(c3[d] * meta.chunk_shape[d], (c3[d] + 1) * meta.chunk_shape[d])
               for d in range(4))] = False
    np.testing.assert_array_equal(full[keep], arr[keep])


def test_store_read_truncated_shard_raises(tmp_path):
    shape = [1, 16, 16, 16]
    meta = A.make_meta(shape, [1, 16, 16, 16], 4, endian=A.ZH_ENDIAN_LITTLE, sharded=True,
                       inner_chunk_shape=[1, 8, 8, 8], index_location=A.ZH_INDEX_START)
    shards = encode_oracle(meta, rand_array(shape, 4, seed=3))
    _, paths = _store(tmp_path, meta, shards)
    p = paths[(0, 0, 0, 0)]
    b = open(p, "rb").read()
    # cut 10 bytes off the last inner chunk's payload (index at the start stays intact), so
    # that chunk's range ends past the file → "Could not load byte data" (an
    # out-of-range entry raises the reference's chunk message)
    open(p, "wb").write(b[:-10])
    with pytest.raises(O.OracleError, match=r"Could not load byte data for chunk \[0, 1, 1, 1\]"):
        O.array_read_store(meta, [p], [0, 0, 0, 0], [1, 16, 16, 15])
