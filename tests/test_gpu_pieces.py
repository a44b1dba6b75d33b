"""Sub-shard reads from the stored index + the referenced ranges (zh_array_read_pieces), the
JNI shim's call sequence for HipArray.read, and the pipelined host read (zh_pipeline.cpp).

Reference: StoreHandleDataProvider (ShardingIndexedCodec.java:245-255, 333-357) reads the
index and one range per referenced inner chunk; the index crc32c (Crc32cCodec.java:24-48) and
the entries (:215-230) are checked on the device here.  Every case is compared bit-exactly
with the oracle (oracle/zh_oracle.c) on the same stored bytes."""
import ctypes as C
import os
import struct

import numpy as np
import pytest

import oracle as O
from helpers import (NP_DT, chunk_coords, encode_oracle, jni_fetch, jni_read, rand_array,
                     shard_part)
from zarrhip import _abi as A
from zarrhip._lib import ShardSource, ZhError, lib

pytestmark = pytest.mark.gpu

M1 = 2 ** 64 - 1


def write_store(tmp_path, meta, shards, tag="a"):
    """Shards as files of a FilesystemStore-like directory: one path per chunk key."""
    d = tmp_path / tag
    d.mkdir(exist_ok=True)
    paths = []
    for i, s in enumerate(shards):
        p = str(d / f"c{i}")
        if s is not None:
            with open(p, "wb") as f:
                f.write(s)
        paths.append(p if s is not None else None)
    return paths


def region_paths(meta, paths, offset, shape):
    n = meta.ndim
    allc = chunk_coords(meta, [0] * n, [meta.shape[d] for d in range(n)])
    pos = {c: i for i, c in enumerate(allc)}
    return [paths[pos[c]] for c in chunk_coords(meta, offset, shape)]


def oracle_region(meta, shards, offset, shape):
    n = meta.ndim
    allc = chunk_coords(meta, [0] * n, [meta.shape[d] for d in range(n)])
    pos = {c: i for i, c in enumerate(allc)}
    srcs = [shards[pos[c]] for c in chunk_coords(meta, offset, shape)]
    return np.frombuffer(O.array_read(meta, srcs, offset, shape),
                         NP_DT[meta.dtype_size]).reshape(shape)


CHAINS = {
    "sharded": dict(sharded=True, inner_chunk_shape=[4, 8, 8]),
    "transpose_be": dict(sharded=True, inner_chunk_shape=[4, 8, 8], transpose_order=[2, 0, 1],
                         endian=A.ZH_ENDIAN_BIG),
    "start_beindex": dict(sharded=True, inner_chunk_shape=[4, 8, 8],
                          index_location=A.ZH_INDEX_START, index_endian=A.ZH_ENDIAN_BIG),
    "chunk_crc": dict(sharded=True, inner_chunk_shape=[4, 8, 8], inner_crc32c=True,
                      transpose_order=[1, 2, 0]),
    "nested": dict(sharded=True, inner_chunk_shape=[8, 8, 8], nested_chunk_shape=[4, 4, 8]),
}
REGIONS = [([0, 0, 0], [24, 32, 48]), ([3, 5, 7], [17, 20, 33]), ([8, 16, 0], [4, 8, 48]),
           ([1, 1, 1], [1, 1, 1])]


def make_case(chain, dsize=4, seed=3, fill_frac=0.2):
    shape = [24, 32, 48]
    meta = A.make_meta(shape, [8, 16, 24], dsize, fill=(7).to_bytes(dsize, "little"),
                       **CHAINS[chain])
    arr = rand_array(shape, dsize, seed=seed, fill_frac=fill_frac, fill=0)
    arr[:4, :8, :8] = 0  # an inner chunk of zeros: Q1 reads through a missing entry
    return meta, arr, encode_oracle(meta, arr)


@pytest.mark.parametrize("chain", list(CHAINS))
@pytest.mark.parametrize("max_run", [0, 1 << 26])
def test_pieces_read_matches_oracle(dev, tmp_path, chain, max_run):
    meta, arr, shards = make_case(chain)
    shards[3] = None  # a missing shard reads fill_value
    paths = write_store(tmp_path, meta, shards)
    for off, shp in REGIONS:
        rp = region_paths(meta, paths, off, shp)
        fetched = jni_fetch(meta, rp, off, shp, max_run=max_run, size_known=max_run > 0)
        got = jni_read(dev, meta, fetched, off, shp)
        np.testing.assert_array_equal(got, oracle_region(meta, shards, off, shp))


def test_pieces_pageable_host_memory(dev, tmp_path):
    """The same form from ordinary (pageable) host buffers, one buffer per piece."""
    meta, arr, shards = make_case("transpose_be", seed=11)
    paths = write_store(tmp_path, meta, shards)
    off, shp = [2, 3, 4], [20, 25, 40]
    fetched = jni_fetch(meta, region_paths(meta, paths, off, shp), off, shp, max_run=0)
    keep, srcs = [], []
    for s in fetched:
        if s is None:
            srcs.append(None)
            continue
        idx, size, pieces = s
        ib = (C.c_char * len(idx)).from_buffer_copy(idx) if idx is not None else None
        keep.append(ib)
        ps = []
        for o, b in pieces:
            pb = (C.c_char * len(b)).from_buffer_copy(b)
            keep.append(pb)
            ps.append((o, len(b), C.addressof(pb), len(b)))
        srcs.append(ShardSource(C.addressof(ib) if ib is not None else None,
                                len(idx) if idx is not None else 0, size, ps))
    out = np.empty(shp, np.uint32)
    dev.array_read_pieces(meta, srcs, off, shp, out.ctypes.data, 0)
    np.testing.assert_array_equal(out, oracle_region(meta, shards, off, shp))


def test_pieces_device_sources(dev, tmp_path):
    """ZH_SRC_DEVICE: the index and pieces already in HBM (read where they are)."""
    meta, arr, shards = make_case("chunk_crc", seed=13)
    paths = write_store(tmp_path, meta, shards)
    off, shp = [1, 2, 3], [22, 29, 44]
    fetched = jni_fetch(meta, region_paths(meta, paths, off, shp), off, shp, max_run=1 << 20)
    bufs, srcs = [], []

    def up(b):
        p = dev.malloc(max(1, len(b)))
        dev.h2d(p, b)
        bufs.append(p)
        return p
    for s in fetched:
        if s is None:
            srcs.append(None)
            continue
        idx, size, pieces = s
        srcs.append(ShardSource(up(idx) if idx is not None else None,
                                len(idx) if idx is not None else 0, size,
                                [(o, len(b), up(b), len(b)) for o, b in pieces]))
    nb = int(np.prod(shp)) * 4
    d_out = dev.malloc(nb)
    try:
        dev.array_read_pieces(meta, srcs, off, shp, d_out, A.ZH_SRC_DEVICE | A.ZH_OUT_DEVICE)
        got = np.frombuffer(dev.d2h(d_out, nb), np.uint32).reshape(shp)
    finally:
        dev.free(d_out)
        for p in bufs:
            dev.free(p)
    np.testing.assert_array_equal(got, oracle_region(meta, shards, off, shp))


@pytest.mark.parametrize("where", ["entry", "stored_crc"])
def test_corrupt_stored_index_reports_device_crc(dev, tmp_path, where):
    """The stored index goes to the device unchanged: a corrupt index fails the device's
    crc32c with the reference's message (Crc32cCodec.java:39-44), the oracle's text."""
    meta, arr, shards = make_case("sharded", seed=17, fill_frac=0.0)
    bad = list(shards)
    b = bytearray(bad[1])
    b[-9 if where == "entry" else -2] ^= 0x10  # an index entry byte / the stored crc
    bad[1] = bytes(b)
    paths = write_store(tmp_path, meta, bad)
    off, shp = [0, 0, 24], [8, 16, 24]  # all of shard 1 (coords [0, 0, 1])
    with pytest.raises(O.OracleError) as eo:
        O.array_read(meta, [bad[1]], off, shp)
    fetched = jni_fetch(meta, region_paths(meta, paths, off, shp), off, shp)
    assert fetched[0][0] is None  # the whole object
    # and the sub-shard form: a part of the same shard
    off2, shp2 = [1, 0, 24], [6, 16, 24]
    fetched2 = jni_fetch(meta, region_paths(meta, paths, off2, shp2), off2, shp2)
    assert fetched2[0][0] is not None  # index + pieces
    for f, o, s in [(fetched, off, shp), (fetched2, off2, shp2)]:
        with pytest.raises(ZhError) as ed:
            jni_read(dev, meta, f, o, s)
        assert str(ed.value) == str(eo.value)
        assert str(ed.value).startswith("The checksum of the sharding index is invalid.")


def test_missing_piece_reports_reference_message(dev, tmp_path):
    """A referenced range the store could not deliver (its read returned null) reads as
    "Could not load byte data for chunk [...]" (ShardingIndexedCodec.java:226-230)."""
    meta, arr, shards = make_case("sharded", seed=19, fill_frac=0.0)
    paths = write_store(tmp_path, meta, shards)
    off, shp = [1, 1, 1], [6, 14, 22]  # inside shard 0: inner chunks [0..1, 0..1, 0..2]
    fetched = jni_fetch(meta, region_paths(meta, paths, off, shp), off, shp, max_run=0,
                        drop={(0, 2)})
    # ranges sorted by offset = inner chunks in C order of the shard's grid (oracle layout):
    # the third referenced one is chunk [0, 0, 2]
    with pytest.raises(ZhError) as ed:
        jni_read(dev, meta, fetched, off, shp)
    assert str(ed.value) == "Could not load byte data for chunk [0, 0, 2]"


def test_host_decoded_pieces(dev):
    """Pieces whose host byte-to-byte stages were undone (zstd / gzip / blosc in the inner
    chain, DeviceChain.innerHost): each stored range maps to its raw payload exactly."""
    meta, arr, shards = make_case("transpose_be", seed=23)
    isz = lib().zh_shard_index_size(C.byref(meta))
    raw = shards[0]
    body = raw[-isz:-4]
    # the stored form: every payload behind an 8-byte frame header (a stand-in for a codec
    # frame), the index pointing at the framed ranges
    ents = [struct.unpack("<QQ", body[16 * k:16 * k + 16]) for k in range(len(body) // 16)]
    framed, new, pos = b"", [], 0
    for o, nb in ents:
        if o == M1:
            new.append((M1, M1))
            continue
        fr = b"FRAME!!!" + raw[o:o + nb]
        new.append((pos, len(fr)))
        framed += fr
        pos += len(fr)
    nbody = b"".join(struct.pack("<QQ", *e) for e in new)
    nidx = nbody + struct.pack("<I", O.crc32c(nbody))
    shard_len = len(framed) + len(nidx)
    off, shp = [2, 3, 4], [5, 11, 17]
    lo, hi = [2, 3, 4], [7, 14, 21]
    from zarrhip._lib import shard_ranges
    rs = shard_ranges(meta, nidx, shard_len, lo, hi, 0)
    keep, ps = [], []
    for o, nb in rs:
        payload = framed[o + 8:o + nb]  # "decoded" on the host
        b = (C.c_char * len(payload)).from_buffer_copy(payload)
        keep.append(b)
        ps.append((o, nb, C.addressof(b), len(payload)))
    ib = (C.c_char * len(nidx)).from_buffer_copy(nidx)
    out = np.empty(shp, np.uint32)
    dev.array_read_pieces(meta, [ShardSource(C.addressof(ib), len(nidx), shard_len, ps)],
                          off, shp, out.ctypes.data, 0)
    np.testing.assert_array_equal(out, oracle_region(meta, shards, off, shp))


def test_codec_decode_pieces(dev, tmp_path):
    """zh_sharding_decode_pieces (HipShardingIndexedCodec.decodePartial over a StoreHandle)."""
    meta, arr, shards = make_case("start_beindex", seed=29)
    paths = write_store(tmp_path, meta, shards)
    from zarrhip._lib import shard_ranges
    isz = lib().zh_shard_index_size(C.byref(meta))
    raw = open(paths[0], "rb").read()
    idx = raw[:isz]
    lo, part = [1, 2, 3], [6, 9, 20]
    rs = shard_ranges(meta, idx, len(raw), lo, [a + b for a, b in zip(lo, part)], 1 << 20)
    keep = [(C.c_char * len(idx)).from_buffer_copy(idx)]
    ps = []
    for o, nb in rs:
        b = (C.c_char * nb).from_buffer_copy(raw[o:o + nb])
        keep.append(b)
        ps.append((o, nb, C.addressof(b), nb))
    out = np.empty(part, np.uint32)
    dev.sharding_decode_pieces(meta, ShardSource(C.addressof(keep[0]), isz, len(raw), ps), lo,
                               part, out.ctypes.data)
    err = C.create_string_buffer(1024)
    want = np.empty(part, np.uint32)
    rb = (C.c_char * len(raw)).from_buffer_copy(raw)
    st = O.lib().zo_sharding_decode_partial(C.byref(meta), rb, len(raw),
                                            (C.c_int64 * 3)(*lo), (C.c_int32 * 3)(*part),
                                            C.c_void_p(want.ctypes.data), 1, err, 1024)
    assert st == 0, err.value
    np.testing.assert_array_equal(out, want)


# ---- the pipelined host read (zh_pipeline.cpp), thresholds shrunk ------------------------
@pytest.fixture
def pipe(monkeypatch):
    monkeypatch.setenv("ZH_PIPE_MIN_KB", "1")
    monkeypatch.setenv("ZH_PIPE_SLAB_KB", "4")
    monkeypatch.setenv("ZH_PIPE_CHUNK_KB", "64")
    monkeypatch.setenv("ZH_PIPE_THREADS", "3")


@pytest.mark.parametrize("chain", ["sharded", "transpose_be", "chunk_crc", "nested"])
def test_pipelined_pieces_read(dev, tmp_path, pipe, chain):
    """Slabs along the first axis, each planned over its own chunks and staging only its own
    ranges, through the in/out rings (staging pinned, caller's output pageable)."""
    meta, arr, shards = make_case(chain, seed=31)
    shards[5] = None
    paths = write_store(tmp_path, meta, shards)
    for off, shp in REGIONS[:3]:
        fetched = jni_fetch(meta, region_paths(meta, paths, off, shp), off, shp,
                            max_run=1 << 12)
        np.testing.assert_array_equal(jni_read(dev, meta, fetched, off, shp),
                                      oracle_region(meta, shards, off, shp))
        # pageable sources and output (the Python mirror's form)
        from helpers import device_read
        srcs = [None if p is None else open(p, "rb").read()
                for p in region_paths(meta, paths, off, shp)]
        np.testing.assert_array_equal(device_read(dev, meta, srcs, off, shp),
                                      oracle_region(meta, shards, off, shp))


def test_pipelined_device_sources_host_output(dev, pipe):
    """Device-resident shards, host output: only the out lanes run."""
    meta, arr, shards = make_case("transpose_be", seed=37)
    bufs = []
    srcs = []
    for s in shards:
        if s is None:
            srcs.append((None, 0))
            continue
        p = dev.malloc(len(s))
        dev.h2d(p, s)
        bufs.append(p)
        srcs.append((p, len(s)))
    n = 3
    allc = chunk_coords(meta, [0] * n, [24, 32, 48])
    pos = {c: i for i, c in enumerate(allc)}
    try:
        for off, shp in REGIONS[:3]:
            sub = [srcs[pos[c]] for c in chunk_coords(meta, off, shp)]
            out = np.empty(shp, np.uint32)
            dev.array_read(meta, sub, off, shp, out.ctypes.data, A.ZH_SRC_DEVICE)
            np.testing.assert_array_equal(out, oracle_region(meta, shards, off, shp))
    finally:
        for p in bufs:
            dev.free(p)


def test_pipelined_error_is_first_slab(dev, pipe):
    """Two corrupt shards in different slabs: the first in C order is reported, the oracle's
    message."""
    meta, arr, shards = make_case("sharded", seed=41, fill_frac=0.0)
    bad = list(shards)
    for i in (4, 9):
        b = bytearray(bad[i])
        b[-7] ^= 0x01
        bad[i] = bytes(b)
    with pytest.raises(O.OracleError) as eo:
        O.array_read(meta, bad, [0, 0, 0], [24, 32, 48])
    from helpers import device_read
    with pytest.raises(ZhError) as ed:
        device_read(dev, meta, bad, [0, 0, 0], [24, 32, 48])
    assert str(ed.value) == str(eo.value)


def test_jni_sequence_sub_shard_2gib(dev, tmp_path):
    """BASELINE.md §3's read through the JNI shim's exact call sequence: the region
    [1,1024,1024,512] of one c4-format 1×1024³ uint32 shard (inner 1×32³, transpose
    [0,3,2,1], bytes big, index crc32c at the end) references 16 384 inner chunks = 2^31
    bytes of payload — more than one Java array holds, which is why the JNI passes pieces and
    never a compacted shard.  The shard is encoded on the device, stored as a file, fetched as
    index + ranges, passed as they are (the JNI's critical-section form) and decoded through the
    pipelined read; the result equals the oracle's
    FilesystemStore read (zo_array_read_store: suffix index read, one range read per inner
    chunk, ShardingIndexedCodec.java:253, 333-357)."""
    shape = [1, 1024, 1024, 1024]
    meta = A.make_meta(shape, shape, 4, endian=A.ZH_ENDIAN_BIG, sharded=True,
                       inner_chunk_shape=[1, 32, 32, 32], transpose_order=[0, 3, 2, 1])
    nel = 1 << 30
    src = dev.malloc(nel * 4)
    bound = lib().zh_array_encoded_bound(C.byref(meta))
    dst = dev.malloc(bound)
    try:
        dev.synth_fill(src, nel, 4, 0, 0x5A5A2026)
        dev.sync()
        (nb,) = dev.array_write(meta, src, [0] * 4, shape, [(dst, bound)])
        dev.free(src)
        src = None
        assert nb == nel * 4 + 16 * 32768 + 4
        base = "/dev/shm" if os.path.isdir("/dev/shm") else str(tmp_path)
        path = os.path.join(base, f"zh_jni2g_{os.getpid()}")
        host = np.empty(nb, np.uint8)
        dev.memcpy(host.ctypes.data, dst, nb, 1)
        host.tofile(path)
        del host
    finally:
        if src:
            dev.free(src)
        dev.free(dst)
    try:
        off, shp = [0, 0, 0, 0], [1, 1024, 1024, 512]
        fetched = jni_fetch(meta, [path], off, shp, max_run=64 << 20)
        idx, size, pieces = fetched[0]
        assert idx is not None and size == nb
        assert sum(len(b) for _, b in pieces) == 2 ** 31  # the referenced payload
        got = jni_read(dev, meta, fetched, off, shp)
        del fetched, pieces
        want = np.empty(shp, np.uint32)
        O.array_read_store(meta, [path], off, shp, want.ctypes.data, nthreads=16)
        assert np.array_equal(got, want)
        # and a corrupt stored index is reported by the device with the reference's message
        with open(path, "r+b") as f:
            f.seek(nb - 100)
            b = f.read(1)
            f.seek(nb - 100)
            f.write(bytes([b[0] ^ 0x20]))
        with pytest.raises(O.OracleError) as eo:
            O.array_read_store(meta, [path], [0, 0, 0, 0], [1, 32, 32, 32])
        small = jni_fetch(meta, [path], [0, 0, 0, 0], [1, 32, 32, 32])
        with pytest.raises(ZhError) as ed:
            jni_read(dev, meta, small, [0, 0, 0, 0], [1, 32, 32, 32])
        assert str(ed.value) == str(eo.value)
    finally:
        os.unlink(path)


def test_pieces_form_errors(dev, tmp_path):
    """Malformed sub-shard forms fail before any device work: unsorted or overlapping pieces
    and a host-decoded piece under nested sharding → ZH_EINVAL; an index shorter than the
    index size → the 'smaller than its index' message; a shard without index must be one
    whole piece at offset 0."""
    meta, arr, shards = make_case("sharded", seed=43)
    paths = write_store(tmp_path, meta, shards)
    off, shp = [1, 1, 1], [6, 14, 22]
    fetched = jni_fetch(meta, region_paths(meta, paths, off, shp), off, shp, max_run=0)
    idx, size, pieces = fetched[0]
    keep = [(C.c_char * len(idx)).from_buffer_copy(idx)]
    ps = []
    for o, b in pieces:
        keep.append((C.c_char * len(b)).from_buffer_copy(b))
        ps.append((o, len(b), C.addressof(keep[-1]), len(b)))
    out = np.empty(shp, np.uint32)
    ip = C.addressof(keep[0])
    with pytest.raises(ZhError) as e:  # unsorted
        dev.array_read_pieces(meta, [ShardSource(ip, len(idx), size, ps[::-1])], off, shp,
                              out.ctypes.data, 0)
    assert e.value.status == A.ZH_EINVAL
    o0, n0, p0, h0 = ps[0]
    with pytest.raises(ZhError) as e:  # overlapping
        dev.array_read_pieces(meta, [ShardSource(ip, len(idx), size, [ps[0], (o0 + 4, n0, p0,
                                                                         n0)] + ps[1:])],
                              off, shp, out.ctypes.data, 0)
    assert e.value.status == A.ZH_EINVAL
    with pytest.raises(ZhError) as e:  # short index
        dev.array_read_pieces(meta, [ShardSource(ip, len(idx) - 1, size, ps)], off, shp,
                              out.ctypes.data, 0)
    assert e.value.status == A.ZH_EDATA and "smaller than its index" in str(e.value)
    with pytest.raises(ZhError) as e:  # no index, not a whole piece
        dev.array_read_pieces(meta, [ShardSource(None, 0, size, ps[:2])], off, shp,
                              out.ctypes.data, 0)
    assert e.value.status == A.ZH_EINVAL
    # the well-formed call still reads correctly
    dev.array_read_pieces(meta, [ShardSource(ip, len(idx), size, ps)], off, shp,
                          out.ctypes.data, 0)
    np.testing.assert_array_equal(out, oracle_region(meta, shards, off, shp))


def test_pieces_unknown_size_out_of_range_entry(dev):
    """shard_nbytes = -1 (StoreHandle.getSize() unknown): an entry pointing beyond the bytes
    the store could deliver has no piece, so the device reports the reference's "Could not
    load byte data for chunk [...]" — after a correct index crc32c."""
    meta, arr, shards = make_case("sharded", seed=47, fill_frac=0.0)
    isz = lib().zh_shard_index_size(C.byref(meta))
    raw = shards[0]
    body = bytearray(raw[-isz:-4])
    o, nb = struct.unpack("<QQ", body[16:32])  # inner chunk [0, 0, 1]
    body[16:24] = struct.pack("<Q", o + (1 << 40))
    nidx = bytes(body) + struct.pack("<I", O.crc32c(bytes(body)))
    from zarrhip._lib import shard_ranges
    off, shp = [0, 0, 0], [8, 16, 24]
    lo, hi = [0, 0, 0], [8, 16, 24]
    rs = shard_ranges(meta, nidx, -1, lo, hi, 0)
    keep = [(C.c_char * isz).from_buffer_copy(nidx)]
    ps = []
    for ro, rn in rs:
        if ro >= len(raw):  # the store read fails: no piece
            continue
        keep.append((C.c_char * rn).from_buffer_copy(raw[ro:ro + rn]))
        ps.append((ro, rn, C.addressof(keep[-1]), rn))
    out = np.empty(shp, np.uint32)
    with pytest.raises(ZhError) as e:
        dev.array_read_pieces(meta, [ShardSource(C.addressof(keep[0]), isz, -1, ps)], off,
                              [7, 16, 24], out.ctypes.data, 0)
    assert str(e.value) == "Could not load byte data for chunk [0, 0, 1]"


def test_pieces_nested_and_multi_context(dev, tmp_path):
    """Nested sharding through the pieces form on three contexts of the card
    (zh_array_read_pieces_multi: one slab per context, same-device routes)."""
    from zarrhip._lib import DeviceContext, array_read_pieces_multi
    meta, arr, shards = make_case("nested", seed=53)
    paths = write_store(tmp_path, meta, shards)
    off, shp = [2, 3, 5], [21, 27, 40]
    fetched = jni_fetch(meta, region_paths(meta, paths, off, shp), off, shp, max_run=1 << 16)
    keep, srcs = [], []
    for s in fetched:
        if s is None:
            srcs.append(None)
            continue
        idx, size, pieces = s
        ib = (C.c_char * len(idx)).from_buffer_copy(idx) if idx is not None else None
        keep.append(ib)
        ps = []
        for o, b in pieces:
            keep.append((C.c_char * len(b)).from_buffer_copy(b))
            ps.append((o, len(b), C.addressof(keep[-1]), len(b)))
        srcs.append(ShardSource(C.addressof(ib) if ib is not None else None,
                                len(idx) if idx is not None else 0, size, ps))
    ctxs = [dev, DeviceContext(0), DeviceContext(0)]
    try:
        out = np.empty(shp, np.uint32)
        array_read_pieces_multi(ctxs, meta, srcs, off, shp, out.ctypes.data, 0)
        np.testing.assert_array_equal(out, oracle_region(meta, shards, off, shp))
    finally:
        for c in ctxs[1:]:
            c.close()


def test_pieces_from_pinned_staging(dev, tmp_path):
    """zh_host_staging: a binding that copies its sources into the context's page-locked
    staging (and takes the region back through it) gets direct DMA both ways."""
    meta, arr, shards = make_case("transpose_be", seed=59)
    paths = write_store(tmp_path, meta, shards)
    off, shp = [1, 2, 3], [22, 28, 40]
    fetched = jni_fetch(meta, region_paths(meta, paths, off, shp), off, shp, max_run=1 << 20)
    tot = sum((len(s[0]) if s[0] is not None else 0) + sum(len(b) for _, b in s[2])
              for s in fetched if s is not None)
    obytes = int(np.prod(shp)) * 4
    in_cap = (tot + 255) // 256 * 256
    base = dev.host_staging(in_cap + obytes)
    pos, srcs = 0, []
    for s in fetched:
        if s is None:
            srcs.append(None)
            continue
        idx, size, pieces = s
        ip = None
        if idx is not None:
            C.memmove(base + pos, idx, len(idx))
            ip = base + pos
            pos += len(idx)
        ps = []
        for o, b in pieces:
            C.memmove(base + pos, b, len(b))
            ps.append((o, len(b), base + pos, len(b)))
            pos += len(b)
        srcs.append(ShardSource(ip, len(idx) if idx is not None else 0, size, ps))
    dev.array_read_pieces(meta, srcs, off, shp, base + in_cap, 0)
    got = np.frombuffer(C.string_at(base + in_cap, obytes), np.uint32).reshape(shp)
    np.testing.assert_array_equal(got, oracle_region(meta, shards, off, shp))
