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


def _one_shard(tmp_path, loc, crc=True, seed=3):
    shape = [1, 16, 16, 16]
    meta = A.make_meta(shape, [1, 16, 16, 16], 4, endian=A.ZH_ENDIAN_LITTLE, sharded=True,
                       inner_chunk_shape=[1, 8, 8, 8], index_location=loc, index_crc32c=crc)
    shard = encode_oracle(meta, rand_array(shape, 4, seed=seed))[0]
    _, paths = _store(tmp_path, meta, [shard])
    return meta, shard, paths[(0, 0, 0, 0)]


@pytest.mark.parametrize("loc", [A.ZH_INDEX_START, A.ZH_INDEX_END])
def test_store_part_of_truncated_shard_reads_zeros(tmp_path, loc):
    """FilesystemStore.get(keys, start, end) (FilesystemStore.java:84-102) allocates end - start
    bytes and reads what the file holds: a part whose inner chunk lost its tail decodes what
    the file has at the entry's offsets and zeros past its end — the in-memory read of a shard
    whose payload region holds exactly that — and a range entirely past the end reads all
    zeros."""
    meta, shard, p = _one_shard(tmp_path, loc)
    isz = 16 * 8 + 4
    payload_end = len(shard) if loc == A.ZH_INDEX_START else len(shard) - isz
    for cut in (10, 2048 + 100):  # into the last chunk; the last chunk gone and more
        keep = payload_end - cut
        stored = shard[:keep] + (shard[payload_end:] if loc == A.ZH_INDEX_END else b"")
        open(p, "wb").write(stored)
        # what each range read returns: the file's bytes at the entry's offsets (with the
        # index at the end, the moved index where the payload was), zeros past the end
        padded = (stored + bytes(payload_end))[:payload_end] + \
            (shard[payload_end:] if loc == A.ZH_INDEX_END else b"")
        for off, shp in (([0, 0, 0, 0], [1, 16, 16, 15]), ([0, 8, 8, 8], [1, 8, 8, 8]),
                         ([0, 3, 9, 9], [1, 13, 7, 6])):
            want = O.array_read(meta, [padded], off, shp)
            assert O.array_read_store(meta, [p], off, shp) == want, (cut, off)


def test_store_whole_truncated_shard_raises(tmp_path):
    """The whole shard is read in one piece (decodePartial → chunkHandle.read(),
    ShardingIndexedCodec.java:246-251) and sliced: an entry beyond the bytes cannot be served
    (the reference's ByteBuffer slice throws IllegalArgumentException; reported as "Could not
    load byte data")."""
    meta, shard, p = _one_shard(tmp_path, A.ZH_INDEX_START)
    open(p, "wb").write(shard[:-10])
    with pytest.raises(O.OracleError, match=r"Could not load byte data for chunk \[0, 1, 1, 1\]"):
        O.array_read_store(meta, [p], [0, 0, 0, 0], [1, 16, 16, 16])


def test_store_short_index_reads(tmp_path):
    """A file shorter than its index: a suffix read (index_location end, get(keys, -n)) resolves
    to a negative position, which the reference's channel rejects — an error; a prefix read
    (start, get(keys, 0, n)) returns the file's bytes zero-padded to the index's length, whose
    crc32c then fails with the reference's message (stored 0)."""
    meta, shard, p = _one_shard(tmp_path, A.ZH_INDEX_END)
    open(p, "wb").write(shard[:50])
    with pytest.raises(O.OracleError, match="is smaller than its index"):
        O.array_read_store(meta, [p], [0, 0, 0, 0], [1, 8, 8, 8])
    meta, shard, p = _one_shard(tmp_path, A.ZH_INDEX_START)
    open(p, "wb").write(shard[:50])
    want_crc = O.crc32c(shard[:50] + bytes(16 * 8 - 50))
    want_crc = want_crc - (1 << 32) if want_crc >= 1 << 31 else want_crc
    with pytest.raises(O.OracleError) as e:
        O.array_read_store(meta, [p], [0, 0, 0, 0], [1, 8, 8, 8])
    assert str(e.value) == ("The checksum of the sharding index is invalid. Stored: 0 "
                            f"Computed: {want_crc}")
