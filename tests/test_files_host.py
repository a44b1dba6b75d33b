"""The store reads zh_array_read_files makes, checked on the host (zh_debug_file_reads; no
device): FilesystemStore semantics (M/store/FilesystemStore.java:43-102) — a missing or
non-regular file is a missing key, a whole chunk is one read, a shard is its index read (a
prefix with index_location start, else the last 16·n + 4 bytes: get(keys, -isz)) followed by the
referenced inner chunks' ranges (StoreHandleDataProvider, ShardingIndexedCodec.java:333-357),
adjacent ones merged, entries beyond the file left out."""
import os
import struct

import numpy as np
import pytest

import oracle as O
from helpers import chunk_coords, encode_oracle, rand_array
from zarrhip import _abi as A
from zarrhip._lib import ZhError, file_reads, shard_ranges

M1 = 2 ** 64 - 1


def _write(tmp_path, shards):
    paths = []
    for i, s in enumerate(shards):
        p = str(tmp_path / f"c{i}")
        if s is not None:
            with open(p, "wb") as f:
                f.write(s)
        paths.append(p)
    return paths


def _entries(meta, index, lo, hi):
    """(offset, nbytes) of the part's referenced, present inner chunks (oracle-independent
    restatement of the index walk, ShardingIndexedCodec.java:206-221)."""
    n = meta.ndim
    inner = [meta.chain.inner_chunk_shape[d] for d in range(n)]
    cps = [meta.chunk_shape[d] // inner[d] for d in range(n)]
    b0 = [lo[d] // inner[d] for d in range(n)]
    b1 = [(hi[d] - 1) // inner[d] for d in range(n)]
    fmt = ">QQ" if meta.chain.index_endian == A.ZH_ENDIAN_BIG else "<QQ"
    out = []
    for idx in np.ndindex(*[b1[d] - b0[d] + 1 for d in range(n)]):
        lin = 0
        for d in range(n):
            lin = lin * cps[d] + b0[d] + idx[d]
        o, nb = struct.unpack(fmt, index[16 * lin:16 * lin + 16])
        if o != M1 and nb != M1 and nb > 0:
            out.append((o, nb))
    return out


@pytest.mark.parametrize("loc", [A.ZH_INDEX_END, A.ZH_INDEX_START])
def test_shard_reads_are_index_then_referenced_ranges(tmp_path, loc):
    shape = [24, 32, 48]
    meta = A.make_meta(shape, [8, 16, 24], 4, sharded=True, inner_chunk_shape=[4, 8, 8],
                       index_location=loc, endian=A.ZH_ENDIAN_BIG)
    arr = rand_array(shape, 4, seed=5)
    arr[:4, :8, :8] = 0  # an all-fill inner chunk: a missing entry
    shards = encode_oracle(meta, arr)
    shards[1] = None
    paths = _write(tmp_path, shards)
    isz = 16 * (2 * 2 * 3) + 4
    allc = chunk_coords(meta, [0, 0, 0], shape)
    for off, shp in [([0, 0, 0], shape), ([3, 5, 7], [17, 20, 33]), ([1, 1, 1], [1, 1, 1])]:
        cs = chunk_coords(meta, off, shp)
        rp = [paths[allc.index(c)] for c in cs]
        got = file_reads(meta, rp, off, shp)
        want = []
        for i, c in enumerate(cs):
            s = shards[allc.index(c)]
            if s is None:
                continue
            size = len(s)
            index = s[:isz] if loc == A.ZH_INDEX_START else s[-isz:]
            want.append((i, 0 if loc == A.ZH_INDEX_START else size - isz, isz))
            lo = [max(off[d], c[d] * meta.chunk_shape[d]) - c[d] * meta.chunk_shape[d]
                  for d in range(3)]
            hi = [min(off[d] + shp[d], (c[d] + 1) * meta.chunk_shape[d]) -
                  c[d] * meta.chunk_shape[d] for d in range(3)]
            rs = shard_ranges(meta, index, size, lo, hi, 1 << 30)
            want += [(i, o, nb) for o, nb in rs]
            # every referenced present entry lies inside exactly one read range
            mine = [(o, nb) for j, o, nb in got if j == i][1:]
            for o, nb in _entries(meta, index, lo, hi):
                assert sum(ro <= o and o + nb <= ro + rn for ro, rn in mine) == 1
        assert got == want


def test_missing_directories_and_short_files(tmp_path):
    shape = [24, 32, 48]
    meta = A.make_meta(shape, [8, 16, 24], 4, sharded=True, inner_chunk_shape=[4, 8, 8])
    shards = encode_oracle(meta, rand_array(shape, 4, seed=7))
    paths = _write(tmp_path, shards)
    os.remove(paths[0])                       # absent file: missing key
    os.remove(paths[2])
    os.mkdir(paths[2])                        # a directory: missing key (isRegularFile)
    with open(paths[3], "wb") as f:
        f.write(b"tiny")                      # shorter than its index: the whole file, no ranges
    paths[4] = None                           # no path at all
    got = file_reads(meta, paths, [0, 0, 0], shape)
    by = {}
    for i, o, n in got:
        by.setdefault(i, []).append((o, n))
    assert 0 not in by and 2 not in by and 4 not in by
    assert by[3] == [(0, 4)]
    assert all(k in by for k in range(5, len(paths)))


def test_truncated_shard_drops_entries_beyond_the_file(tmp_path):
    shape = [8, 16, 24]
    meta = A.make_meta(shape, [8, 16, 24], 4, sharded=True, inner_chunk_shape=[4, 8, 8],
                       index_location=A.ZH_INDEX_START)
    s = encode_oracle(meta, rand_array(shape, 4, seed=9))[0]
    paths = _write(tmp_path, [s])
    full = file_reads(meta, paths, [0, 0, 0], shape)
    os.truncate(paths[0], len(s) - 100)
    cut = file_reads(meta, paths, [0, 0, 0], shape)
    assert cut[0] == full[0]  # the index read
    assert sum(n for _, _, n in cut[1:]) < sum(n for _, _, n in full[1:])
    assert all(o + n <= len(s) - 100 for _, o, n in cut)


def test_unsharded_whole_objects_and_errors(tmp_path):
    shape = [24, 32, 48]
    meta = A.make_meta(shape, [8, 16, 24], 4, endian=A.ZH_ENDIAN_BIG)
    chunks = encode_oracle(meta, rand_array(shape, 4, seed=11))
    paths = _write(tmp_path, chunks)
    got = file_reads(meta, paths, [0, 0, 0], shape)
    assert got == [(i, 0, len(c)) for i, c in enumerate(chunks)]
    with pytest.raises(ZhError) as e:
        file_reads(meta, paths, [1, 0, 0], shape)
    assert str(e.value) == "Requested data is outside of the array's domain."
    with pytest.raises(ZhError) as e:
        file_reads(meta, paths[:-1], [0, 0, 0], shape)
    assert e.value.status == A.ZH_EINVAL
    if os.geteuid() != 0:
        os.chmod(paths[0], 0)
        try:
            with pytest.raises(ZhError) as e:
                file_reads(meta, paths, [0, 0, 0], shape)
            assert e.value.status == A.ZH_EIO
        finally:
            os.chmod(paths[0], 0o600)
