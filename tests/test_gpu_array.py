"""End-to-end v3.Array reads/writes through stores, on the HIP path.  Mirrors zarr-java's
ZarrV3Test (testShardingReadWrite, testParallel, testUnalignedArrayAccess,
testLargerChunkSizeThanArraySize, testEndianness, testDefaultChunkShape) and the
ZarrPythonTests codec configurations (parse_codecs.py:104-116) on 16^3 arange data."""
import os

import numpy as np
import pytest

import oracle as O
import zarrhip as z
from helpers import GOLDEN

pytestmark = pytest.mark.gpu


def make_testdata(dt):
    """ZarrTest.testdata: value i at flat index i, 16^3 (ZarrTest.java:157-194)."""
    a = np.arange(16 * 16 * 16)
    if dt == z.DataType.BOOL:
        return (a % 2).astype(np.bool_).reshape(16, 16, 16)
    return a.astype(dt.numpy).reshape(16, 16, 16)


@pytest.mark.parametrize("loc", ["start", "end"])
def test_open_reference_fixture(loc):
    arr = z.Array.open(z.FilesystemStore(GOLDEN).resolve("sharding_index_location", loc))
    np.testing.assert_array_equal(arr.read().ravel(), np.arange(4096, dtype=np.int32))
    np.testing.assert_array_equal(arr.read([1, 2, 3], [5, 6, 7]),
                                  np.arange(4096).reshape(16, 16, 16)[1:6, 2:8, 3:10])
    np.testing.assert_array_equal(arr.readChunk([0, 1, 0]),
                                  np.arange(4096).reshape(16, 16, 16)[:, 8:, :8])


@pytest.mark.parametrize("loc", ["start", "end"])
def test_sharding_read_write(tmp_path, loc):
    """testShardingReadWrite (ZarrV3Test.java:309-323)."""
    src = z.Array.open(z.FilesystemStore(GOLDEN).resolve("sharding_index_location", loc))
    content = src.read()
    dst = z.Array.create(z.FilesystemStore(tmp_path).resolve(loc), src.metadata)
    dst.write(None, content)
    np.testing.assert_array_equal(z.Array.open(z.FilesystemStore(tmp_path).resolve(loc)).read(),
                                  content)


CODECS = {
    "bytes_le": lambda c: c.withBytes("LITTLE"),
    "bytes_be": lambda c: c.withBytes("BIG"),
    "transpose": lambda c: c.withTranspose([1, 0, 2]).withBytes("BIG"),
    "sharding_start": lambda c: c.withSharding([2, 2, 4], lambda c1: c1.withBytes("LITTLE"), "start"),
    "sharding_end": lambda c: c.withSharding([2, 2, 4], lambda c1: c1.withBytes("BIG"), "end"),
    "sharding_transpose": lambda c: c.withSharding(
        [2, 2, 4], lambda c1: c1.withTranspose([2, 0, 1]).withBytes("BIG")),
    "crc32c": lambda c: c.withBytes("LITTLE").withCrc32c(),
    "gzip": lambda c: c.withBytes("LITTLE").withGzip(5),
    "sharding_gzip": lambda c: c.withSharding([2, 2, 4], lambda c1: c1.withBytes("LITTLE").withGzip()),
    "blosc_memcpy": lambda c: c.withBytes("LITTLE").withBlosc(),
    "zstd": lambda c: c.withBytes("BIG").withZstd(3, True),
    "sharding_zstd": lambda c: c.withSharding([2, 2, 4], lambda c1: c1.withBytes("LITTLE")
                                              .withZstd(5, False)),
}


@pytest.mark.parametrize("name", ["v0.5/0", "v0.5/1", "v0.5/labels/nuclei/0",
                                  "v0.5_hcs/A/1/0/0"])
def test_ome_zstd_fixture_read(name):
    """The reference's zstd-compressed OME-Zarr arrays (codecs [bytes little, zstd]): host
    zstd (zh_zstd_decompress) then the device bytes + scatter stages; checked against the
    chunks decoded by libzstd (pyarrow) and assembled with numpy."""
    import json
    pa = pytest.importorskip("pyarrow")
    root = os.path.join(GOLDEN, "ome_zstd", *name.split("/"))
    meta = json.load(open(os.path.join(root, "zarr.json")))
    shape = meta["shape"]
    cs = meta["chunk_grid"]["configuration"]["chunk_shape"]
    dt = np.dtype({"float32": "<f4", "uint8": "u1", "uint16": "<u2", "int32": "<i4",
                   "uint32": "<u4", "int64": "<i8"}[meta["data_type"]])
    want = np.zeros(shape, dt)
    for idx in np.ndindex(*[-(-s // c) for s, c in zip(shape, cs)]):
        path = os.path.join(root, "c", *map(str, idx))
        if not os.path.exists(path):
            continue
        raw = pa.Codec("zstd").decompress(open(path, "rb").read(),
                                          decompressed_size=int(np.prod(cs)) * dt.itemsize,
                                          asbytes=True)
        blk = np.frombuffer(raw, dt).reshape(cs)
        sl = tuple(slice(i * c, min((i + 1) * c, s)) for i, c, s in zip(idx, cs, shape))
        want[sl] = blk[tuple(slice(0, x.stop - x.start) for x in sl)]
    arr = z.Array.open(z.FilesystemStore(os.path.join(GOLDEN, "ome_zstd")).resolve(
        *name.split("/")))
    got = arr.read()
    np.testing.assert_array_equal(got, want)
    off = [s // 3 for s in shape]
    shp = [max(1, s - o - 1) for s, o in zip(shape, off)]
    np.testing.assert_array_equal(arr.read(off, shp),
                                  want[tuple(slice(o, o + n) for o, n in zip(off, shp))])


@pytest.mark.parametrize("name", sorted(CODECS))
def test_codec_configs_roundtrip(tmp_path, name):
    data = make_testdata(z.DataType.INT32)
    m = (z.ArrayMetadataBuilder().withShape(16, 16, 16).withDataType(z.DataType.INT32)
         .withChunkShape(2, 4, 8).withFillValue(0).withCodecs(CODECS[name]).build())
    a = z.Array.create(z.FilesystemStore(tmp_path).resolve(name), m)
    a.write(None, data)
    b = z.Array.open(z.FilesystemStore(tmp_path).resolve(name))
    np.testing.assert_array_equal(b.read(), data)
    np.testing.assert_array_equal(b.read([3, 1, 5], [9, 13, 10]), data[3:12, 1:14, 5:15])


@pytest.mark.parametrize("dt,endian", [(d, e) for d in (z.DataType.INT16, z.DataType.UINT16,
                                                          z.DataType.INT32, z.DataType.UINT32,
                                                          z.DataType.FLOAT32, z.DataType.FLOAT64,
                                                          z.DataType.INT64, z.DataType.UINT8,
                                                          z.DataType.BOOL)
                                       for e in ("LITTLE", "BIG")])
def test_endianness(tmp_path, dt, endian):
    """testEndianness (ZarrV3Test.java:1038-1054), plus 1-byte and 8-byte types."""
    data = make_testdata(dt)
    m = (z.ArrayMetadataBuilder().withShape(16, 16, 16).withDataType(dt)
         .withCodecs(lambda c: c.withBytes(endian)).build())
    a = z.Array.create(z.FilesystemStore(tmp_path).resolve("e"), m)
    a.write(None, data)
    got = z.Array.open(z.FilesystemStore(tmp_path).resolve("e")).read()
    np.testing.assert_array_equal(got, data)
    raw = open(os.path.join(tmp_path, "e", "c", "0", "0", "0"), "rb").read()
    order = ">" if endian == "BIG" and dt.getByteCount() > 1 else "<"
    np.testing.assert_array_equal(np.frombuffer(raw, data.dtype.newbyteorder(order)),
                                  data.ravel())


def test_parallel_large(tmp_path):
    """testParallel (ZarrV3Test.java:463-483) at 256^3 with 100^3 chunks."""
    n = 256
    data = np.arange(n ** 3, dtype=np.uint32).reshape(n, n, n)
    m = (z.ArrayMetadataBuilder().withShape(n, n, n).withDataType(z.DataType.UINT32)
         .withChunkShape(100, 100, 100).withFillValue(0).build())
    a = z.Array.create(z.FilesystemStore(tmp_path).resolve("p"), m)
    a.write(None, data)
    np.testing.assert_array_equal(z.Array.open(z.FilesystemStore(tmp_path).resolve("p")).read(), data)


@pytest.mark.parametrize("ashape,cshape,acc", [(52, 17, 32), (71, 11, 12), (52, 17, 17),
                                               (50, 3, 7), (50, 3, 22), (13, 31, 21)])
def test_unaligned_array_access(ashape, cshape, acc):
    """testUnalignedArrayAccess (ZarrV3Test.java:921-945)."""
    a = z.Array.create(z.MemoryStore().resolve(),
                       z.ArrayMetadataBuilder().withShape(ashape).withDataType(z.DataType.UINT32)
                       .withChunkShape(cshape).withFillValue(0).build())
    data = (np.arange(ashape).astype(np.int8).astype(np.int64) & 0xFFFFFFFF).astype(np.uint32)
    a.write(None, data)
    i = 0
    while i < ashape:
        acc = min(acc, ashape - i)
        np.testing.assert_array_equal(a.read([i], [acc]), data[i:i + acc])
        i += acc


def test_larger_chunk_than_array(tmp_path):
    data = np.arange(4096, dtype=np.uint32).reshape(16, 16, 16)
    m = (z.ArrayMetadataBuilder().withShape(16, 16, 16).withDataType(z.DataType.UINT32)
         .withChunkShape(32, 32, 32).withFillValue(0).build())
    a = z.Array.create(z.FilesystemStore(tmp_path).resolve("l"), m)
    a.write(None, data)
    np.testing.assert_array_equal(z.Array.open(z.FilesystemStore(tmp_path).resolve("l")).read(),
                                  data)


def test_partial_write_read_modify_write():
    m = (z.ArrayMetadataBuilder().withShape(20, 30).withDataType(z.DataType.UINT16)
         .withChunkShape(8, 8).withFillValue(9)
         .withCodecs(lambda c: c.withSharding([4, 4], lambda c1: c1.withBytes("BIG"))).build())
    a = z.Array.create(z.MemoryStore().resolve(), m)
    np.testing.assert_array_equal(a.read(), np.full((20, 30), 9, np.uint16))
    patch = np.arange(7 * 11, dtype=np.uint16).reshape(7, 11)
    a.access().withOffset(3, 5).write(patch)
    got = a.read()
    np.testing.assert_array_equal(got[3:10, 5:16], patch)
    # all-fill inner chunks of a written shard are elided and read back as 0, not 9 (Q1,
    # exactly as the reference: ShardingIndexedCodec.java:129-133 + :189,219-221)
    coords = O.compute_chunk_coords([20, 30], [8, 8], [0, 0], [20, 30])
    srcs = [a.storeHandle.resolve(*a.metadata.chunk_key_encoding.encode_chunk_key(c)).read()
            for c in coords]
    want = np.frombuffer(O.array_read(a.zmeta, srcs, [0, 0], [20, 30]), np.uint16).reshape(20, 30)
    np.testing.assert_array_equal(got, want)
    assert got[0, 0] == 0 and got[19, 29] == 9
    # chunks that stayed all-fill were never written (writeChunk deletes all-fill chunks)
    assert not a.storeHandle.resolve("c", "2", "3").exists()


def test_default_chunk_shape():
    m = z.ArrayMetadataBuilder().withShape(100, 50).withDataType(z.DataType.UINT8).build()
    assert m.chunk_shape == [100, 50]
    m = z.ArrayMetadataBuilder().withShape(2000, 1500).withDataType(z.DataType.UINT8).build()
    assert 0 < m.chunk_shape[0] < 2000 and 0 < m.chunk_shape[1] < 1500


def test_array_read_matches_oracle_with_missing_shards(tmp_path):
    """Missing shard → fill; missing inner chunk → 0 (Q1), via stores."""
    m = (z.ArrayMetadataBuilder().withShape(12, 12).withDataType(z.DataType.UINT32)
         .withChunkShape(6, 6).withFillValue(5)
         .withCodecs(lambda c: c.withSharding([3, 3])).build())
    a = z.Array.create(z.FilesystemStore(tmp_path).resolve("q"), m)
    data = np.full((12, 12), 5, np.uint32)
    data[0, 4] = 1  # shard (0,0): one non-fill inner chunk
    a.write(None, data)
    got = a.read()
    assert got[0, 4] == 1
    assert (got[0:3, 0:3] == 0).all()      # missing inner chunk in a present shard → 0
    assert (got[6:, :] == 5).all()          # missing shards → fill
    srcs = [a.storeHandle.resolve(*a.metadata.chunk_key_encoding.encode_chunk_key(c)).read()
            for c in O.compute_chunk_coords([12, 12], [6, 6], [0, 0], [12, 12])]
    want = np.frombuffer(O.array_read(a.zmeta, srcs, [0, 0], [12, 12]), np.uint32).reshape(12, 12)
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("loc", ["start", "end"])
@pytest.mark.parametrize("inner_bb", [False, True])
def test_partial_shard_staging_reads_only_referenced_chunks(tmp_path, monkeypatch, loc,
                                                           inner_bb):
    """Sub-shard reads fetch the index + referenced inner chunks only (the reference's
    StoreHandleDataProvider path, ShardingIndexedCodec.java:333-357), with identical
    results.  The mirror's own store reads (ZH_FILES=0; with the default a FilesystemStore's
    files go to zh_array_read_files: tests/test_gpu_files.py)."""
    monkeypatch.setenv("ZH_FILES", "0")
    shape = [64, 64, 32]
    fn = (lambda c1: c1.withBytes("BIG").withGzip()) if inner_bb else (lambda c1: c1.withBytes("BIG"))
    m = (z.ArrayMetadataBuilder().withShape(*shape).withDataType(z.DataType.UINT32)
         .withChunkShape(64, 64, 32).withFillValue(0)
         .withCodecs(lambda c: c.withSharding([8, 8, 8], fn, loc)).build())
    a = z.Array.create(z.FilesystemStore(tmp_path).resolve("s"), m)
    data = np.arange(np.prod(shape), dtype=np.uint32).reshape(shape)
    a.write(None, data)
    b = z.Array.open(z.FilesystemStore(tmp_path).resolve("s"))
    got = b.read([5, 9, 3], [10, 12, 6])
    np.testing.assert_array_equal(got, data[5:15, 9:21, 3:9])
    shard_bytes = os.path.getsize(os.path.join(tmp_path, "s", "c", "0", "0", "0"))
    assert b.staged_bytes < shard_bytes / 4
    b.staged_bytes = 0
    np.testing.assert_array_equal(b.read(), data)
    assert b.staged_bytes == shard_bytes


def test_partial_staging_crc_error_message(tmp_path):
    m = (z.ArrayMetadataBuilder().withShape(16, 16).withDataType(z.DataType.UINT32)
         .withChunkShape(16, 16).withCodecs(lambda c: c.withSharding([4, 4])).build())
    a = z.Array.create(z.FilesystemStore(tmp_path).resolve("k"), m)
    a.write(None, np.arange(256, dtype=np.uint32).reshape(16, 16))
    p = os.path.join(tmp_path, "k", "c", "0", "0")
    raw = bytearray(open(p, "rb").read())
    raw[-8] ^= 0x10
    open(p, "wb").write(bytes(raw))
    with pytest.raises(z.ZarrException, match="The checksum of the sharding index is invalid"):
        a.read([1, 1], [3, 3])       # partial path: host CRC check
    with pytest.raises(z.ZarrException, match="The checksum of the sharding index is invalid"):
        a.read()                     # full-shard path: device CRC check


@pytest.mark.parametrize("dt", [z.DataType.INT32, z.DataType.UINT8, z.DataType.FLOAT64])
def test_sharding_nested_python_config(tmp_path, dt):
    """ZarrPythonTests "sharding_nested" (ZarrPythonTests.java:146-151,177-179): 16^3,
    chunk [2,4,8], sharding [2,2,4] → sharding [2,1,2] → bytes(little); write + read back,
    plus sub-shard reads (partial staging of a nested shard)."""
    m = (z.ArrayMetadataBuilder().withShape(16, 16, 16).withDataType(dt).withChunkShape(2, 4, 8)
         .withFillValue(0).withCodecs(lambda c: c.withSharding(
             [2, 2, 4], lambda c1: c1.withSharding([2, 1, 2], lambda c2: c2.withBytes("LITTLE"))))
         .build())
    a = z.Array.create(z.FilesystemStore(tmp_path).resolve("n"), m)
    data = make_testdata(dt)
    a.write(None, data)
    b = z.Array.open(z.FilesystemStore(tmp_path).resolve("n"))
    np.testing.assert_array_equal(b.read(), data)
    np.testing.assert_array_equal(b.read([1, 3, 5], [9, 7, 6]), data[1:10, 3:10, 5:11])
    # the stored shard bytes equal the oracle's encoding of the same chunk
    coords = (0, 1, 1)
    raw = open(os.path.join(tmp_path, "n", "c", *map(str, coords)), "rb").read()
    want = O.array_write(b.zmeta, data.tobytes(), [0, 0, 0], [16, 16, 16])
    idx = O.compute_chunk_coords([16, 16, 16], [2, 4, 8], [0, 0, 0], [16, 16, 16]).index(coords)
    assert raw == want[idx]


@pytest.mark.parametrize("shape,chunk,fn", [
    # ReshapeCodecTest.testReshapeCodecReadWriteSingleChunk (zstd → gzip: no zstd here)
    ([4, 5, 6, 3], [4, 5, 6, 3], lambda c: c.withReshape([[0, 1], [2], 3]).withGzip()),
    # testReshapeCodecReadWriteMultipleChunks
    ([8, 6, 4], [4, 3, 4], lambda c: c.withReshape([[0, 1], [2]]).withBytes("LITTLE")),
    # testReshapeCombinedWithTranspose
    ([4, 4, 4], [4, 4, 4], lambda c: c.withTranspose([2, 1, 0]).withReshape([[0, 1], [2]])
     .withBytes("LITTLE")),
    # merge then transpose (folded into a chunk-dim permutation), big-endian, inside shards
    ([8, 12, 10], [8, 12, 10], lambda c: c.withSharding([4, 6, 5], lambda c1: c1.withReshape(
        [[0, 1], [2]]).withTranspose([1, 0]).withBytes("BIG"))),
])
def test_reshape_read_write(tmp_path, shape, chunk, fn):
    m = (z.ArrayMetadataBuilder().withShape(*shape).withDataType(z.DataType.UINT32)
         .withChunkShape(*chunk).withFillValue(0).withCodecs(fn).build())
    a = z.Array.create(z.FilesystemStore(tmp_path).resolve("r"), m)
    data = np.arange(int(np.prod(shape)), dtype=np.uint32).reshape(shape)
    a.write(None, data)
    b = z.Array.open(z.FilesystemStore(tmp_path).resolve("r"))
    np.testing.assert_array_equal(b.read(), data)
    off = [1] * len(shape)
    shp = [s - 2 for s in shape]
    np.testing.assert_array_equal(b.read(off, shp), data[tuple(slice(1, s - 1) for s in shape)])


@pytest.mark.parametrize("spec", ["0,0", "0,0,0"])
def test_read_spread_over_devices(tmp_path, monkeypatch, spec):
    """ZH_DEVICES: Array.read runs zh_array_read_multi (one slab per listed device, here
    repeated device 0) and returns what the single-device read returns."""
    ref = z.Array.open(z.FilesystemStore(GOLDEN).resolve("sharding_index_location", "end"))
    content = ref.read()
    dst = z.Array.create(z.FilesystemStore(tmp_path).resolve("multi"), ref.metadata)
    dst.write(None, content)
    arr = z.Array.open(z.FilesystemStore(tmp_path).resolve("multi"))
    one = arr.read([1, 2, 3], [14, 13, 12])
    monkeypatch.setenv("ZH_DEVICES", spec)
    np.testing.assert_array_equal(arr.read(), content)
    np.testing.assert_array_equal(arr.read([1, 2, 3], [14, 13, 12]), one)


def test_large_array_with_offset_beyond_max_int(tmp_path):
    """testLargeArrayWithOffsetBeyondMaxInt (ZarrV3Test.java:994-1036): a 3e9 x 3e9 int32
    array of 1000² chunks, fill 42; a [1, 1000] row written at [0, 0] and at
    [1, Integer.MAX_VALUE + 1] (each a read-modify-write of one chunk) reads back, and a
    chunk nobody wrote reads the fill value."""
    big = 3_000_000_000
    m = (z.ArrayMetadataBuilder().withShape(big, big).withDataType(z.DataType.INT32)
         .withChunkShape(1000, 1000).withFillValue(42).build())
    a = z.Array.create(z.FilesystemStore(tmp_path).resolve("large_array_beyond_int"), m)
    a.write([0, 0], np.full((1, 1000), 100, np.int32))
    far = [1, 2 ** 31]
    a.write(far, np.full((1, 1000), 200, np.int32))
    b = z.Array.open(z.FilesystemStore(tmp_path).resolve("large_array_beyond_int"))
    assert b.read([0, 0], [1, 100])[0, 0] == 100
    got = b.read(far, [1, 100])
    assert (got == 200).all()
    assert (b.read([0, 2 ** 31], [1, 100]) == 42).all()  # the same chunk's row 0: fill
    assert (b.read([5000, 5000], [3, 3]) == 42).all()    # a chunk never written
    assert b.metadata.shape == [big, big]
