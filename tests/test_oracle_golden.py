"""Pins the CPU oracle to the reference's own fixtures and known-answer tests.

  - testdata/sharding_index_location/{start,end} (copied to tests/golden/): decode to
    arange(4096) int32 16x16x16, index CRCs 0xB756D1D4 / 0x56F05363.
  - TestUtils.java:15-93 (permutations, computeChunkCoords, computeProjection, overflow).
  - ZarrV3Test.java:248-264 transpose known-answer test.
  - CRC-32C check value "123456789" -> 0xE3069283 (CRC32C.java table, tbl[1]=0xF26B8303).
"""
import os
import struct

import numpy as np
import pytest

import oracle as O
from helpers import GOLDEN, encode_oracle, load_reference_fixture, rand_array
from zarrhip import _abi as A


def test_crc32c_check_value():
    assert O.crc32c(b"123456789") == 0xE3069283
    assert O.crc32c(b"") == 0
    # incremental update == one shot (CRC32C.update contract)
    assert O.crc32c(b"56789", O.crc32c(b"1234")) == 0xE3069283


@pytest.mark.parametrize("loc,crc", [("end", 0xB756D1D4), ("start", 0x56F05363)])
def test_fixture_index_crc(loc, crc):
    base = os.path.join(GOLDEN, "sharding_index_location", loc, "c", "0", "0", "0")
    b = open(base, "rb").read()
    assert len(b) == 4228
    idx = b[:68] if loc == "start" else b[-68:]
    assert struct.unpack("<I", idx[-4:])[0] == crc
    assert O.crc32c(idx[:-4]) == crc
    ents = [struct.unpack("<QQ", idx[16 * i:16 * i + 16]) for i in range(4)]
    first = 68 if loc == "start" else 0
    assert ents == [(first + 1040 * i, 1040) for i in range(4)]


@pytest.mark.parametrize("loc", ["start", "end"])
def test_fixture_decodes_to_arange(loc):
    _, meta, srcs = load_reference_fixture(loc)
    out = np.frombuffer(O.array_read(meta, srcs, [0, 0, 0], [16, 16, 16]), dtype="<i4")
    np.testing.assert_array_equal(out, np.arange(4096))
    # sub-region (partial decode path) and the single-full-chunk shortcut region
    sub = np.frombuffer(O.array_read(meta, [srcs[1]], [0, 0, 8], [16, 8, 8]), "<i4")
    np.testing.assert_array_equal(sub.reshape(16, 8, 8),
                                  np.arange(4096).reshape(16, 16, 16)[:, :8, 8:])


@pytest.mark.parametrize("loc", ["start", "end"])
def test_fixture_reencode_roundtrip(loc):
    """testShardingReadWrite (ZarrV3Test.java:309-323): read → write → read equality."""
    _, meta, srcs = load_reference_fixture(loc)
    arr = np.frombuffer(O.array_read(meta, srcs, [0, 0, 0], [16, 16, 16]), "<u4").reshape(16, 16, 16)
    shards = encode_oracle(meta, arr)
    back = np.frombuffer(O.array_read(meta, shards, [0, 0, 0], [16, 16, 16]), "<u4")
    np.testing.assert_array_equal(back, arr.ravel())
    # with blosc unwrapped the payload layout is C-order, so the bytes match exactly
    assert shards == srcs


def test_is_permutation_kat():
    import ctypes as C

    def isp(v):
        return O.lib().zo_is_permutation(len(v), (C.c_int32 * max(1, len(v)))(*v)) == 1
    assert isp([2, 1, 0]) and isp([4, 2, 1, 3, 0])
    assert not isp([0, 1, 2, 0]) and not isp([0, 1, 2, 3, 5]) and not isp([])


def test_inverse_permutation_kat():
    import ctypes as C

    def inv(v):
        out = (C.c_int32 * len(v))()
        assert O.lib().zo_inverse_permutation(len(v), (C.c_int32 * len(v))(*v), out) == 0
        return list(out)
    assert inv([1, 0, 2]) == [1, 0, 2]
    assert inv([1, 2, 0]) == [2, 0, 1]
    assert inv([0, 4, 2, 1, 3]) == [0, 3, 2, 4, 1]
    assert inv([2, 0, 1]) != [2, 0, 1]


def test_compute_chunk_coords_kat():
    assert O.compute_chunk_coords([100, 100], [30, 30], [50, 20], [20, 1]) == [(1, 0), (2, 0)]
    assert O.compute_chunk_coords([1, 52], [1, 17], [0, 32], [1, 20]) == [(0, 1), (0, 2), (0, 3)]


def test_compute_projection_kat():
    co, oo, ps = O.compute_projection([0, 2], [1, 52], [1, 17], [0, 32], [1, 20])
    assert (co, oo, ps) == ([0, 0], [0, 2], [1, 17])


def test_compute_chunk_coords_overflow():
    with pytest.raises(ArithmeticError):
        O.compute_chunk_coords([100000, 100000], [1, 1], [0, 0], [100000, 100000])


def test_transpose_kat():
    """ZarrV3Test.testTransposeCodec: 2x3x3 order [1,2,0] encodes to 0,9,1,10,2,11,..."""
    data = np.arange(18, dtype=np.uint32).reshape(2, 3, 3)
    meta = A.make_meta([2, 3, 3], [2, 3, 3], 4, transpose_order=[1, 2, 0])
    (enc,) = encode_oracle(meta, data)
    assert list(np.frombuffer(enc, "<u4")) == [0, 9, 1, 10, 2, 11, 3, 12, 4, 13, 5, 14, 6, 15,
                                                7, 16, 8, 17]
    dec = np.frombuffer(O.array_read(meta, [enc], [0, 0, 0], [2, 3, 3]), "<u4").reshape(2, 3, 3)
    np.testing.assert_array_equal(dec, data)


def test_endianness_bytes():
    """testEndianness: big-endian bytes codec stores swapped elements."""
    data = np.array([[0x01020304, 0x0A0B0C0D]], dtype=np.uint32)
    meta = A.make_meta([1, 2], [1, 2], 4, endian=A.ZH_ENDIAN_BIG)
    (enc,) = encode_oracle(meta, data)
    assert enc == bytes([1, 2, 3, 4, 0xA, 0xB, 0xC, 0xD])
    assert np.frombuffer(O.array_read(meta, [enc], [0, 0], [1, 2]), "<u4").tolist() == \
        data.ravel().tolist()


def test_missing_inner_chunk_q1():
    """Q1: missing inner chunk → 0 despite fill 7; missing shard → 7."""
    meta = A.make_meta([8, 8], [4, 8], 4, fill=(7).to_bytes(4, "little"), sharded=True,
                       inner_chunk_shape=[2, 4])
    arr = np.full((8, 8), 7, np.uint32)
    arr[0, 5] = 1
    shards = encode_oracle(meta, arr)
    assert shards[1] is None
    out = np.frombuffer(O.array_read(meta, shards, [0, 0], [8, 8]), "<u4").reshape(8, 8)
    assert out[0, 5] == 1 and (out[0:2, 0:4] == 0).all() and (out[4:, :] == 7).all()


def test_crc_error_message():
    meta = A.make_meta([4, 4], [4, 4], 4, sharded=True, inner_chunk_shape=[2, 2])
    (s,) = encode_oracle(meta, rand_array([4, 4], 4, seed=1))
    bad = bytearray(s)
    bad[-1] ^= 1
    with pytest.raises(O.OracleError) as e:
        O.array_read(meta, [bytes(bad)], [0, 0], [4, 4])
    stored = struct.unpack("<i", bytes(bad[-4:]))[0]
    computed = struct.unpack("<i", s[-4:])[0]
    assert str(e.value) == ("The checksum of the sharding index is invalid. Stored: %d Computed: %d"
                            % (stored, computed))
