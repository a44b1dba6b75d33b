"""Nested sharding on the HIP path (nested_index_kernel flattening + the single-level
resolve/scatter kernels) vs the CPU oracle, bit-exact, through the C-ABI; the write path's
two-level layout vs the oracle's bytes.  Configurations follow ZarrPythonTests
"sharding_nested" (ZarrPythonTests.java:177-179) plus index location/endianness/crc
variants and transpose at the leaf level."""
import struct

import numpy as np
import pytest

import oracle as O
import spec_sharding as spec
from helpers import chunk_coords, device_read, device_write, encode_oracle, rand_array, shape_of
from test_oracle_nested import levels, nested_meta
from zarrhip import _abi as A
from zarrhip._lib import ZhError

pytestmark = pytest.mark.gpu

CASES = [
    dict(shape=[16, 16, 16], chunk=[2, 4, 8], l1=[2, 2, 4], l2=[2, 1, 2]),
    dict(shape=[16, 16, 16], chunk=[8, 8, 8], l1=[4, 4, 4], l2=[2, 2, 2], start1=True),
    dict(shape=[12, 20], chunk=[8, 8], l1=[4, 8], l2=[2, 4], start2=True, be2=True, big=True),
    dict(shape=[8, 8], chunk=[8, 8], l1=[4, 4], l2=[4, 2], be1=True, crc2=False),
    dict(shape=[40, 72, 96], chunk=[32, 64, 64], l1=[16, 32, 32], l2=[8, 16, 16]),
]


def _meta(case, order=None, dsize=4):
    c = dict(case)
    shape, chunk, l1, l2 = c.pop("shape"), c.pop("chunk"), c.pop("l1"), c.pop("l2")
    m = nested_meta(shape, chunk, l1, l2, dsize=dsize, **c)
    if order is not None:
        m.chain.has_transpose = 1
        for d, o in enumerate(order):
            m.chain.transpose_order[d] = o
    return m


def _regions(shape):
    n = len(shape)
    return [([0] * n, list(shape)),
            ([1] * n, [s - 2 for s in shape]),
            ([s // 3 for s in shape], [max(1, s // 4) for s in shape])]


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"{c['chunk']}-{c['l1']}-{c['l2']}")
def test_nested_decode_matches_oracle(dev, case):
    m = _meta(case)
    shape = shape_of(m)
    arr = rand_array(shape, 4, seed=5, fill_frac=0.0)
    arr[tuple(slice(0, s // 2) for s in shape)] = 0   # elided cells and leaves
    shards = encode_oracle(m, arr)
    coords_all = chunk_coords(m, [0] * len(shape), shape)
    pos = {c: i for i, c in enumerate(coords_all)}
    for off, shp in _regions(shape):
        srcs = [shards[pos[c]] for c in chunk_coords(m, off, shp)]
        want = np.frombuffer(O.array_read(m, srcs, off, shp), np.uint32).reshape(shp)
        got = device_read(dev, m, srcs, off, shp)
        np.testing.assert_array_equal(got, want)
        np.testing.assert_array_equal(got, arr[tuple(slice(o, o + s) for o, s in zip(off, shp))])


@pytest.mark.parametrize("order", [[2, 1, 0], [1, 0, 2]])
@pytest.mark.parametrize("dsize", [1, 2, 8])
def test_nested_transpose_leaf(dev, order, dsize):
    case = dict(shape=[16, 24, 32], chunk=[16, 24, 32], l1=[8, 12, 16], l2=[4, 6, 8])
    m = _meta(case, order=order, dsize=dsize)
    m.chain.endian = A.ZH_ENDIAN_BIG
    shape = shape_of(m)
    arr = rand_array(shape, dsize, seed=9)
    shards = encode_oracle(m, arr)
    for off, shp in _regions(shape):
        srcs = [shards[0]]
        want = O.array_read(m, srcs, off, shp)
        got = device_read(dev, m, srcs, off, shp)
        assert got.tobytes() == want


@pytest.mark.parametrize("case", CASES[:3], ids=lambda c: f"{c['chunk']}-{c['l1']}-{c['l2']}")
def test_nested_encode_matches_oracle_bytes(dev, case):
    m = _meta(case)
    shape = shape_of(m)
    arr = rand_array(shape, 4, seed=11)
    arr[tuple(slice(0, s // 2) for s in shape)] = 0
    want = encode_oracle(m, arr)
    got = device_write(dev, m, arr)
    assert got == want


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"{c['chunk']}-{c['l1']}-{c['l2']}")
@pytest.mark.parametrize("variant", ["plain", "transpose", "crc32c"])
def test_nested_encode_one_pass(dev, monkeypatch, case, variant):
    """The one-pass write on nested chains (no leaf is all fill_value, so the speculative
    layout holds): cell table, outer index and its crc32c on the host; leaf offsets, sub-index
    entries and sub-index crc32c on the device.  Boundary shards elide padding-only cells and
    leaves.  Bytes equal the oracle's."""
    m = _meta(case, order=[1, 0] + list(range(2, len(case["shape"])))
              if variant == "transpose" else None)
    if variant == "crc32c":
        m.chain.inner_crc32c = 1
    shape = shape_of(m)
    arr = rand_array(shape, 4, seed=13)
    arr[arr == 0] = 1
    want = encode_oracle(m, arr)
    assert device_write(dev, m, arr) == want


def test_nested_sub_index_crc_message(dev):
    m = nested_meta([8, 8], [8, 8], [4, 4], [2, 2])
    data = np.arange(64, dtype=np.uint32).reshape(8, 8) + 1
    shard = bytearray(spec.encode(data, levels([4, 4], [2, 2])))
    shard[4 * 16 + 3] ^= 0x40  # first sub-shard's index
    with pytest.raises(O.OracleError) as eo:
        O.array_read(m, [bytes(shard)], [0, 0], [8, 8])
    with pytest.raises(ZhError) as ed:
        device_read(dev, m, [bytes(shard)], [0, 0], [8, 8])
    assert str(ed.value) == str(eo.value)


def test_nested_leaf_out_of_range_message(dev):
    m = nested_meta([8, 8], [8, 8], [4, 4], [2, 2], crc2=False)
    data = np.arange(64, dtype=np.uint32).reshape(8, 8) + 1
    shard = bytearray(spec.encode(data, levels([4, 4], [2, 2], crc2=False)))
    # first sub-shard = 4 leaves (64 B) + 64 B index; leaf (0,1) offset far out of range
    shard[64 + 16:64 + 24] = struct.pack("<Q", 10 ** 6)
    with pytest.raises(O.OracleError) as eo:
        O.array_read(m, [bytes(shard)], [0, 0], [8, 8])
    with pytest.raises(ZhError) as ed:
        device_read(dev, m, [bytes(shard)], [0, 0], [8, 8])
    assert str(ed.value) == str(eo.value) == "Could not load byte data for chunk [0, 1]"


def test_nested_missing_levels_read_zero(dev):
    m = nested_meta([8, 8], [8, 8], [4, 4], [2, 2])
    m.fill_value[0] = 7
    data = np.arange(64, dtype=np.uint32).reshape(8, 8) + 100
    shard = bytearray(spec.encode(data, levels([4, 4], [2, 2])))
    isz = 16 * 4 + 4
    idx = shard[-isz:-4]
    idx[16 * 3:16 * 4] = struct.pack("<QQ", spec.MISSING, spec.MISSING)
    shard[-isz:] = bytes(idx) + struct.pack("<I", spec.crc32c(bytes(idx)))
    want = np.frombuffer(O.array_read(m, [bytes(shard)], [0, 0], [8, 8]), np.uint32)
    got = device_read(dev, m, [bytes(shard)], [0, 0], [8, 8])
    np.testing.assert_array_equal(got.ravel(), want)
    assert (got[4:, 4:] == 0).all() and (got[:4, :4] == data[:4, :4]).all()
    # a missing shard → fill_value
    got = device_read(dev, m, [None], [0, 0], [8, 8])
    assert (got == 7).all()
