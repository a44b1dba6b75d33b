"""The store reads zh_array_read_files makes, checked on the host (zh_debug_file_reads; no
device): FilesystemStore semantics (M/store/FilesystemStore.java:43-102) — a missing or
non-regular file is a missing key, a whole chunk is one read, a shard is its index read (a
prefix with index_location start, else the last 16·n + 4 bytes: get(keys, -isz)) followed by the
referenced inner chunks' ranges (StoreHandleDataProvider, ShardingIndexedCodec.java:333-357),
adjacent ones merged.  A part's ranges are read like get(keys, start, end) (zero-padded past the
end of the file), so no entry is dropped for its offset; a whole shard is sliced out of the
file as it is (ShardingIndexedCodec.java:246-251), so entries beyond the file are left out."""
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
            whole = all(lo[d] == 0 and hi[d] == meta.chunk_shape[d] for d in range(3))
            rs = shard_ranges(meta, index, size if whole else -1, lo, hi, 1 << 30)
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


def test_truncated_whole_shard_drops_entries_beyond_the_file(tmp_path):
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


@pytest.mark.parametrize("loc", [A.ZH_INDEX_END, A.ZH_INDEX_START])
def test_truncated_part_reads_every_entry(tmp_path, loc):
    """A part of a truncated shard reads the same ranges as of the intact one (the store read
    returns zeros past the end), and a file shorter than a prefix index still reads an index of
    the full length (zero-padded; a suffix index of such a file is reported short)."""
    shape = [8, 16, 24]
    meta = A.make_meta(shape, [8, 16, 24], 4, sharded=True, inner_chunk_shape=[4, 8, 8],
                       index_location=loc, index_crc32c=True)
    s = encode_oracle(meta, rand_array(shape, 4, seed=9, fill_frac=0.0))[0]
    paths = _write(tmp_path, [s])
    off, shp = [0, 0, 0], [8, 16, 23]
    full = file_reads(meta, paths, off, shp)
    isz = 16 * (2 * 2 * 3) + 4
    with open(paths[0], "wb") as f:  # the payload loses its last 3000 bytes, the index stays
        f.write(s[:-3000 - isz] + s[-isz:] if loc == A.ZH_INDEX_END else s[:-3000])
    cut = file_reads(meta, paths, off, shp)
    assert cut[0][2] == full[0][2] == isz and cut[1:] == full[1:]
    os.truncate(paths[0], 20)
    got = file_reads(meta, paths, off, shp)
    if loc == A.ZH_INDEX_START:
        assert got[0] == (0, 0, isz)
    else:
        assert got == [(0, 0, 20)]  # what the file holds: the planner reports it short


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
    if os.geteuid() != 0:  # unreadable: exists (a regular file), the read itself fails
        os.chmod(paths[0], 0)
        try:
            assert file_reads(meta, paths, [0, 0, 0], shape)[0] == (0, 0, len(chunks[0]))
        finally:
            os.chmod(paths[0], 0o600)


def test_shard_unreadable_index_is_store_exception(tmp_path):
    """A shard file that exists but cannot be opened: the index read fails with
    StoreException.readFailed's text (StoreException.java:17-21), naming the store and the key
    below its directory.  (Root reads files regardless of their mode: a directory entry that
    cannot be opened for reading stands in — a FIFO would block, so a dangling permission
    is simulated with a file in a directory without search permission only for non-root.)"""
    shape = [8, 16, 24]
    meta = A.make_meta(shape, [8, 16, 24], 4, sharded=True, inner_chunk_shape=[4, 8, 8])
    s = encode_oracle(meta, rand_array(shape, 4, seed=13))[0]
    d = tmp_path / "store" / "c" / "0"
    d.mkdir(parents=True)
    p = d / "0"
    p.write_bytes(s)
    if os.geteuid() == 0:
        pytest.skip("root reads files regardless of their mode")
    os.chmod(p, 0)
    try:
        with pytest.raises(ZhError) as e:
            file_reads(meta, [str(p)], [0, 0, 0], shape, store=str(tmp_path / "store"))
        assert e.value.status == A.ZH_EIO
        assert str(e.value) == (f"Failed to read from store 'file://{tmp_path}/store' at key "
                                f"'c/0/0/0': {p}")
    finally:
        os.chmod(p, 0o600)


def test_mirror_filesystem_store_exceptions(tmp_path):
    """The Python mirror's FilesystemStore raises StoreException with the reference's texts
    (StoreException.java:17-43 around FilesystemStore's causes, FilesystemStore.java:105-143),
    the same the library's file calls use; and get(keys, start, end) zero-pads past the end."""
    import zarrhip as z
    st = z.FilesystemStore(tmp_path)
    name = f"file://{tmp_path}"
    (tmp_path / "blocker").write_bytes(b"x")
    with pytest.raises(z.StoreException) as e:
        st.set(["blocker", "c", "0"], b"abc")
    assert str(e.value) == (f"Failed to write to store '{name}' at key 'blocker/c/0': "
                            f"Failed to create parent directories for path: {tmp_path}/blocker/c")
    (tmp_path / "d" / "x").mkdir(parents=True)
    with pytest.raises(z.StoreException) as e:
        st.delete(["d"])
    assert str(e.value) == (f"Failed to delete from store '{name}' at key 'd': "
                            f"Failed to delete file: {tmp_path}/d")
    with pytest.raises(z.StoreException) as e:
        st.get(["d"])
    assert str(e.value).startswith(f"Failed to read from store '{name}' at key 'd': {tmp_path}/d: ")
    st.set(["k"], b"0123456789")
    assert st.get(["k"], 2, 6) == b"2345"
    assert st.get(["k"], 8, 14) == b"89" + bytes(4)  # get(keys, start, end): zero-padded
    assert st.get(["k"], 20, 22) == bytes(2)
    assert st.get(["k"], -4) == b"6789"
    with pytest.raises(ValueError):  # a resolved negative position (position(< 0))
        st.get(["k"], -11)
    assert st.get(["nope"], 0, 4) is None


@pytest.mark.parametrize("chain", ["sharded", "start_beindex", "nested", "nested_crc"])
def test_corrupt_index_entries_plan_sane_reads(tmp_path, chain):
    """The host planner over the corrupt indexes of test_gpu_fuzz_index (huge, negative,
    wrapping, straddling, colliding entries; index crc32c off): every planned read lies inside
    [0, 2^63) with a length a Java buffer holds (≤ Integer.MAX_VALUE, the reference's (int)
    allocation), or the plan fails with a message — never a crash (this test also runs under
    the host sanitizer build).  What the device then makes of the ranges is the GPU test."""
    from test_gpu_fuzz_index import corrupt, make_case
    meta, arr = make_case(chain, seed=211)
    shards = encode_oracle(meta, arr)
    shape = [meta.shape[d] for d in range(meta.ndim)]
    rng = np.random.default_rng(223)
    for t in range(40):
        bad = list(shards)
        for i in rng.choice(len(bad), size=2, replace=False):
            if bad[i] is not None:
                bad[i], _ = corrupt(rng, meta, bad[i], int(rng.integers(1, 5)))
        d = tmp_path / f"t{t}"
        d.mkdir()
        paths = _write(d, bad)
        full = rng.random() < 0.5
        off = [0, 0, 0] if full else [int(rng.integers(0, s)) for s in shape]
        shp = shape if full else [int(rng.integers(1, s - o + 1)) for s, o in zip(shape, off)]
        allc = chunk_coords(meta, [0, 0, 0], shape)
        rp = [paths[allc.index(c)] for c in chunk_coords(meta, off, shp)]
        try:
            reads = file_reads(meta, rp, off, shp)
        except ZhError:
            continue
        for k, o, nb in reads:
            assert 0 <= k < len(rp) and o >= 0 and nb >= 0, (t, k, o, nb)
            assert o <= 2 ** 63 - 1 - nb and nb <= 2 ** 31 - 1, (t, k, o, nb)


def test_file_table_queue_stays_bounded(tmp_path):
    """the file table's queue of opens drops its stale entries as files are given
    back, so a long-running process doing many reads of few files keeps it bounded (it grew
    by one entry per descriptor opened until 64 were open at once)."""
    import ctypes as C
    from zarrhip._lib import lib
    shape = [16, 16]
    meta = A.make_meta(shape, [8, 8], 4, sharded=True, inner_chunk_shape=[4, 4])
    arr = rand_array(shape, 4, seed=9)
    paths = _write(tmp_path, encode_oracle(meta, arr))
    st = (C.c_int64 * 3)()
    for _ in range(300):  # each read opens, pins and gives back the 4 shard files
        assert len(file_reads(meta, paths, [0, 0], shape)) > 0
        assert lib().zh_debug_file_table(st) == 0
        assert list(st) == [0, 0, 0]
