"""Nested sharding in the C oracle, pinned against the independent numpy restatement of the
v3 sharding byte format (tests/spec_sharding.py).  The reference holds no nested fixture:
its nested case (ZarrPythonTests.java:177-179, parse_codecs.py:46-48) round-trips through
zarr-python, which is not installed here — so this parity is "pinned to the spec
restatement", not to reference output."""
import numpy as np
import pytest

import oracle as O
import spec_sharding as spec
from zarrhip import _abi as A


def nested_meta(shape, chunk, l1, l2, dsize=4, big=False, start1=False, start2=False,
                be1=False, be2=False, crc1=True, crc2=True):
    return A.make_meta(shape, chunk, dsize, sharded=True, inner_chunk_shape=l1,
                       endian=A.ZH_ENDIAN_BIG if big else A.ZH_ENDIAN_LITTLE,
                       index_endian=A.ZH_ENDIAN_BIG if be1 else A.ZH_ENDIAN_LITTLE,
                       index_crc32c=crc1,
                       index_location=A.ZH_INDEX_START if start1 else A.ZH_INDEX_END,
                       nested_chunk_shape=l2,
                       nested_index_endian=A.ZH_ENDIAN_BIG if be2 else A.ZH_ENDIAN_LITTLE,
                       nested_index_crc32c=crc2,
                       nested_index_location=A.ZH_INDEX_START if start2 else A.ZH_INDEX_END)


def levels(l1, l2, start1=False, start2=False, be1=False, be2=False, crc1=True, crc2=True):
    return [dict(chunk=l1, index_be=be1, crc=crc1, start=start1),
            dict(chunk=l2, index_be=be2, crc=crc2, start=start2)]


CASES = [
    # ZarrPythonTests "sharding_nested": 16^3, chunk [2,4,8], sharding [2,2,4] → [2,1,2]
    dict(shape=[16, 16, 16], chunk=[2, 4, 8], l1=[2, 2, 4], l2=[2, 1, 2]),
    dict(shape=[16, 16, 16], chunk=[8, 8, 8], l1=[4, 4, 4], l2=[2, 2, 2], start1=True),
    dict(shape=[12, 20], chunk=[8, 8], l1=[4, 8], l2=[2, 4], start2=True, be2=True),
    dict(shape=[8, 8], chunk=[8, 8], l1=[4, 4], l2=[4, 2], be1=True, crc2=False, big=True),
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"{c['chunk']}-{c['l1']}-{c['l2']}")
def test_oracle_nested_matches_spec(case):
    c = dict(case)
    shape, chunk, l1, l2 = c.pop("shape"), c.pop("chunk"), c.pop("l1"), c.pop("l2")
    big = c.pop("big", False)
    m = nested_meta(shape, chunk, l1, l2, big=big, **c)
    lv = levels(l1, l2, **c)
    data = np.arange(int(np.prod(shape)), dtype=np.uint32).reshape(shape)
    data[tuple(slice(0, s // 2) for s in shape)] = 0  # elided cells/leaves at both levels
    enc = O.array_write(m, data.tobytes(), [0] * len(shape), shape)
    coords = O.compute_chunk_coords(shape, chunk, [0] * len(shape), shape)
    for cc, b in zip(coords, enc):
        # boundary chunks are padded with fill (0) like allocateFillValueChunk
        full = np.zeros(chunk, np.uint32)
        sl = tuple(slice(ci * cs, min((ci + 1) * cs, s)) for ci, cs, s in zip(cc, chunk, shape))
        part = data[sl]
        full[tuple(slice(0, p) for p in part.shape)] = part
        want = None if not full.any() else spec.encode(full, lv, leaf_be=big)
        assert b == want, f"chunk {cc}: oracle bytes differ from the spec layout"
        if b is not None:
            np.testing.assert_array_equal(spec.decode(b, chunk, lv, np.uint32, leaf_be=big), full)
    got = np.frombuffer(O.array_read(m, enc, [0] * len(shape), shape), np.uint32).reshape(shape)
    np.testing.assert_array_equal(got, data)
    # a sub-region through the partial path
    off = [1] * len(shape)
    shp = [s - 3 for s in shape]
    srcs = [enc[coords.index(cc)] for cc in O.compute_chunk_coords(shape, chunk, off, shp)]
    got = np.frombuffer(O.array_read(m, srcs, off, shp), np.uint32).reshape(shp)
    np.testing.assert_array_equal(got, data[tuple(slice(o, o + s) for o, s in zip(off, shp))])


def test_oracle_nested_sub_index_crc_error():
    m = nested_meta([8, 8], [8, 8], [4, 4], [2, 2])
    data = np.arange(64, dtype=np.uint32).reshape(8, 8) + 1
    shard = bytearray(spec.encode(data, levels([4, 4], [2, 2])))
    # first sub-shard: 4 leaves of 16 B then its 64+4 B index; flip a bit of its index
    shard[4 * 16 + 3] ^= 0x40
    with pytest.raises(O.OracleError, match="The checksum of the sharding index is invalid"):
        O.array_read(m, [bytes(shard)], [0, 0], [8, 8])


def test_oracle_nested_missing_levels_read_zero():
    """Q1 at both levels: a missing sub-shard and a missing leaf read as 0, not fill."""
    m = nested_meta([8, 8], [8, 8], [4, 4], [2, 2])
    m.fill_value[0] = 7
    data = np.arange(64, dtype=np.uint32).reshape(8, 8) + 100
    lv = levels([4, 4], [2, 2])
    shard = spec.encode(data, lv)
    import struct
    body = bytearray(shard)
    isz = 16 * 4 + 4
    idx = body[-isz:-4]
    idx[16 * 3:16 * 4] = struct.pack("<QQ", spec.MISSING, spec.MISSING)  # drop cell (1,1)
    body[-isz:] = bytes(idx) + struct.pack("<I", spec.crc32c(bytes(idx)))
    got = np.frombuffer(O.array_read(m, [bytes(body)], [0, 0], [8, 8]), np.uint32).reshape(8, 8)
    want = data.copy()
    want[4:, 4:] = 0
    np.testing.assert_array_equal(got, want)
