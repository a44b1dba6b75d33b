"""Zarr v2 arrays (M/v2/) on the device chunk path: ZarrV2Test's cases (create with
zlib / blosc / no compressor, no fill value, endianness for every v2 dtype, default chunk
shapes, .zarray format) and the reference's v2_sample fixtures.  The v2 pipeline is
filters + bytes(dtype endianness) + compressor (M/v2/Array.java:34-43)."""
import json
import os

import numpy as np
import pytest

from helpers import GOLDEN
import zarrhip as z
from zarrhip import v2

ALL = [d for d in v2.DataType]


def test_dtype_strings():
    assert v2.DataType.of("<u4") == v2.DataType.UINT32
    assert v2.DataType.of(">f8") == v2.DataType.FLOAT64_BE
    assert v2.DataType.of("|b1") == v2.DataType.BOOL
    assert v2.DataType.of("<u1") == v2.DataType.UINT8      # numpy spelling of 1-byte types
    assert v2.DataType.INT16_BE.value_name == ">i2" and v2.DataType.INT16_BE.getByteCount() == 2
    with pytest.raises(z.ZarrException):
        v2.DataType.of("<c8")


def test_fixture_metadata():
    for name, dt, cname in (("bool", v2.DataType.BOOL, "blosclz"),
                            ("double", v2.DataType.FLOAT64, "blosclz"),
                            ("subgroup/array", v2.DataType.INT32, "lz4")):
        j = json.load(open(os.path.join(GOLDEN, "v2_sample", name, ".zarray")))
        m = v2.ArrayMetadata.from_json(j)
        assert m.data_type == dt and m.chunk_shape == [2, 4, 8] and m.shape == [16, 16, 16]
        assert m.compressor.cfg["cname"] == cname
        # typesize 0 in the JSON → the dtype's byte count (evolveFromCoreArrayMetadata)
        assert m.compressor.cfg["typesize"] == dt.getByteCount()
        assert [c.name for c in m.codecs] == ["bytes", "blosc"]


def test_zarray_json_roundtrip():
    for comp in (lambda b: b.withBloscCompressor(), lambda b: b.withZlibCompressor(), lambda b: b):
        m = comp(v2.ArrayMetadataBuilder().withShape(10, 10).withDataType(v2.DataType.UINT8)
                 .withChunks(6, 6)).build()
        j = json.loads(m.dumps())
        assert j["zarr_format"] == 2 and j["dtype"] == "|u1" and j["order"] == "C"
        assert json.loads(v2.ArrayMetadata.from_json(j).dumps()) == j
        if j["compressor"]:
            assert list(j["compressor"]).count("id") == 1


def test_default_chunk_shape():
    """testDefaultChunkShape."""
    b = lambda *s: v2.ArrayMetadataBuilder().withShape(*s).withDataType(v2.DataType.UINT8).build()
    assert b(100, 50).chunk_shape == [100, 50]
    c = b(2000, 1500).chunk_shape
    assert 0 < c[0] < 2000 and 0 < c[1] < 1500
    c = b(1024, 100, 2048).chunk_shape
    assert 0 < c[0] <= 1024 and c[1] == 100 and 0 < c[2] <= 2048


def test_invalid_levels():
    with pytest.raises(z.ZarrException, match="'level' needs to be between 0 and 9."):
        v2.ZlibCodec(10)
    with pytest.raises(z.ZarrException, match="'clevel' needs to be between 0 and 9."):
        v2.BloscCodec("lz4", 11)


def test_chunk_keys():
    m = v2.ArrayMetadataBuilder().withShape(4, 4).withDataType(v2.DataType.UINT8).build()
    assert m.chunk_key_encoding.encode_chunk_key([1, 2]) == ["1.2"]
    m = v2.ArrayMetadataBuilder().withShape(4, 4).withDataType(v2.DataType.UINT8) \
        .withDimensionSeparator("/").build()
    assert m.chunk_key_encoding.encode_chunk_key([1, 2]) == ["1", "2"]


# ------------------------------------------------------------------------------- device
@pytest.mark.gpu
@pytest.mark.parametrize("comp", ["none", "zlib0", "zlib5", "blosc"])
def test_create_write_read(tmp_path, comp):
    """testCreate / testCreateZlib / testCreateBlosc (blosc frames are written MEMCPYED: no
    blosc library here; any blosc reader accepts them)."""
    b = (v2.ArrayMetadataBuilder().withShape(15, 10).withDataType(v2.DataType.UINT32)
         .withChunks(4, 5).withFillValue(2))
    if comp.startswith("zlib"):
        b = b.withZlibCompressor(int(comp[4:]))
    elif comp == "blosc":
        b = b.withBloscCompressor("lz4", "shuffle", 6)
    a = v2.Array.create(z.FilesystemStore(tmp_path).resolve("a"), b.build())
    data = np.arange(8 * 7, dtype=np.uint32).reshape(8, 7)
    a.write([2, 2], data)
    want = np.full((15, 10), 2, np.uint32)
    want[2:10, 2:9] = data
    r = v2.Array.open(z.FilesystemStore(tmp_path).resolve("a"))
    np.testing.assert_array_equal(r.read(), want)
    np.testing.assert_array_equal(r.read([2, 2], [8, 7]), data)
    assert os.path.exists(os.path.join(tmp_path, "a", "0.0"))  # v2 "." chunk keys


@pytest.mark.gpu
@pytest.mark.parametrize("dt", ALL, ids=lambda d: d.name)
def test_no_fill_value(tmp_path, dt):
    """testNoFillValue: fill_value null reads as 0 / false and stays null."""
    h = z.FilesystemStore(tmp_path).resolve("n")
    a = v2.Array.create(h, v2.ArrayMetadataBuilder().withShape(15, 10).withDataType(dt)
                        .withChunks(4, 5).build())
    assert a.metadata.fill_value is None
    out = a.read([0, 0], [1, 1])
    assert not out.ravel()[0]
    assert v2.Array.open(h).metadata.fill_value is None
    assert json.load(open(os.path.join(tmp_path, "n", ".zarray")))["fill_value"] is None


@pytest.mark.gpu
@pytest.mark.parametrize("dt", ALL, ids=lambda d: d.name)
def test_endianness(tmp_path, dt):
    """testEndianness: write the ZarrTest testdata, reopen, read; big-endian dtypes store
    byte-swapped elements (checked on the raw chunk bytes)."""
    n = 16 * 16 * 16
    if dt == v2.DataType.BOOL:
        data = (np.arange(n) % 2).astype(np.bool_).reshape(16, 16, 16)
    else:
        data = np.arange(n).astype(dt.numpy).reshape(16, 16, 16)
    h = z.FilesystemStore(tmp_path).resolve("e")
    a = v2.Array.create(h, v2.ArrayMetadataBuilder().withShape(16, 16, 16).withDataType(dt)
                        .withChunks(16, 16, 16).build())
    a.write(None, data)
    np.testing.assert_array_equal(v2.Array.open(h).read(), data)
    raw = open(os.path.join(tmp_path, "e", "0.0.0"), "rb").read()
    order = ">" if dt.value_name[0] == ">" else "<"
    assert raw == data.astype(data.dtype.newbyteorder(order)).tobytes()


@pytest.mark.gpu
def test_fixture_bool_memcpyed_blosc():
    """testReadBloscDetectTypesize(BOOL): the fixture's blosc frame is MEMCPYED, so its raw
    bytes are the chunk; missing chunks read as the fill value (false)."""
    a = v2.Array.open(z.FilesystemStore(GOLDEN).resolve("v2_sample", "bool"))
    assert a.metadata.data_type == v2.DataType.BOOL
    got = a.read([0, 0, 0], [3, 4, 5])
    raw = open(os.path.join(GOLDEN, "v2_sample", "bool", "0.0.0"), "rb").read()[16:]
    chunk = np.frombuffer(raw, np.uint8).reshape(2, 4, 8) != 0
    want = np.zeros((3, 4, 5), np.bool_)
    want[:2] = chunk[:, :4, :5]
    np.testing.assert_array_equal(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("name,dt", [("double", v2.DataType.FLOAT64),
                                     ("subgroup/array", v2.DataType.INT32)])
def test_fixture_compressed_blosc_frames(name, dt):
    """testReadBloscDetectTypesize(FLOAT64) and testOpen's subgroup array: BloscLZ / LZ4
    frames decoded on the host (zh_blosc_decompress), bytes + scatter on the device.  Chunk
    0.0.0 holds the ZarrTest arange values; the other chunks are absent (fill 0)."""
    a = v2.Array.open(z.FilesystemStore(GOLDEN).resolve("v2_sample", *name.split("/")))
    assert a.metadata.data_type == dt
    got = a.read([0, 0, 0], [3, 4, 5])
    want = np.zeros((3, 4, 5), dt.numpy)
    want[:2] = (np.arange(16 ** 3).reshape(16, 16, 16)[:2, :4, :5]).astype(dt.numpy)
    np.testing.assert_array_equal(got, want)
    full = a.read()
    assert full[:2, :4, :8].ravel().tolist() == np.arange(16 ** 3).reshape(16, 16, 16)[:2, :4, :8].ravel().tolist()


@pytest.mark.gpu
def test_null_fill_keeps_zero_chunks(tmp_path):
    """writeChunk deletes an all-fill chunk only when a fill value exists (Array.java:150)."""
    h = z.FilesystemStore(tmp_path).resolve("k")
    a = v2.Array.create(h, v2.ArrayMetadataBuilder().withShape(4, 4).withDataType(v2.DataType.INT16_BE)
                        .withChunks(2, 4).withZlibCompressor(1).build())
    a.write(None, np.zeros((4, 4), np.int16))
    assert sorted(os.listdir(os.path.join(tmp_path, "k"))) == [".zarray", "0.0", "1.0"]
    np.testing.assert_array_equal(v2.Array.open(h).read(), np.zeros((4, 4), np.int16))
    h2 = z.FilesystemStore(tmp_path).resolve("k2")
    a = v2.Array.create(h2, v2.ArrayMetadataBuilder().withShape(4, 4).withDataType(v2.DataType.INT16)
                        .withChunks(2, 4).withFillValue(0).build())
    a.write(None, np.zeros((4, 4), np.int16))
    assert sorted(os.listdir(os.path.join(tmp_path, "k2"))) == [".zarray"]


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["v0.4/0", "v0.4/1", "v0.4/labels/nuclei/0",
                                  "v0.4_hcs/A/1/0/0"])
def test_ome_v04_blosc_lz4_fixture_read(name):
    """The reference's OME-Zarr v0.4 arrays (v2, blosc LZ4 + byte shuffle, '.'-separated keys):
    host blosc (zh_blosc_decompress) then the device bytes + scatter stages; equal to the
    chunks decoded by liblz4 (pyarrow) with the shuffle undone and assembled in numpy
    (test_blosc.independent_blosc_lz4), whole and for an interior region."""
    import json
    from test_blosc import independent_blosc_lz4
    root = os.path.join(GOLDEN, "ome_blosc", *name.split("/"))
    za = json.load(open(os.path.join(root, ".zarray")))
    shape, cs, dt = za["shape"], za["chunks"], np.dtype(za["dtype"])
    want = np.zeros(shape, dt)
    for idx in np.ndindex(*[-(-s // c) for s, c in zip(shape, cs)]):
        path = os.path.join(root, ".".join(map(str, idx)))
        if not os.path.exists(path):
            continue
        blk = np.frombuffer(independent_blosc_lz4(open(path, "rb").read()), dt).reshape(cs)
        sl = tuple(slice(i * c, min((i + 1) * c, s)) for i, c, s in zip(idx, cs, shape))
        want[sl] = blk[tuple(slice(0, x.stop - x.start) for x in sl)]
    a = v2.Array.open(z.FilesystemStore(os.path.join(GOLDEN, "ome_blosc")).resolve(
        *name.split("/")))
    np.testing.assert_array_equal(a.read(), want)
    off = [s // 3 for s in shape]
    shp = [max(1, s - o - 1) for s, o in zip(shape, off)]
    np.testing.assert_array_equal(a.read(off, shp),
                                  want[tuple(slice(o, o + n) for o, n in zip(off, shp))])
