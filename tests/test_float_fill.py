"""The write path's all-fill test on float arrays (MultiArrayUtils.allValuesEqual with
ValueAccessor.isEqual: Java's == on float / double, M/utils/MultiArrayUtils.java:69-80,
104-150), used where the reference elides a chunk (Array.writeChunk, core/Array.java:148-151)
and an inner chunk of a shard (ShardingIndexedCodec.encode :129-133).

- fill ±0.0: a chunk of zeros of either sign is all fill (+0.0 == -0.0): elided, so it reads
  back as the fill's zero — the oracle and the device agree byte for byte;
- fill NaN: NaN == NaN is false, so nothing is elided — every chunk and inner chunk is
  written, boundary padding included (an elided inner chunk would read back as 0, Q1)."""
import numpy as np
import pytest

import oracle as O
from helpers import device_read, device_write, encode_oracle
from zarrhip import _abi as A

SHAPE = [12, 16]


def _meta(dt, fill, sharded):
    ds = np.dtype(dt).itemsize
    kw = dict(sharded=True, inner_chunk_shape=[4, 8]) if sharded else {}
    return A.make_meta(SHAPE, [8, 16] if sharded else [4, 8], ds,
                       fill=np.array([fill], dt).tobytes(), is_float=True, **kw)


def _array(dt, fill):
    a = np.random.default_rng(5).standard_normal(SHAPE).astype(dt)
    a[0:4, 0:8] = -0.0                       # all negative zeros
    a[4:8, 0:8] = 0.0
    a[4:8, 0:4] = -0.0                       # mixed signs
    a[8:12, 8:16] = fill                     # the fill itself (NaN: the same bits)
    return a


def _decode(meta, chunks, dt):
    return np.frombuffer(O.array_read(meta, chunks, [0, 0], SHAPE), dt).reshape(SHAPE)


@pytest.mark.parametrize("sharded", [False, True])
@pytest.mark.parametrize("dt", ["<f4", "<f8"])
def test_oracle_zero_fill_elides_either_sign(dt, sharded):
    meta = _meta(dt, 0.0, sharded)
    a = _array(dt, 0.0)
    chunks = encode_oracle(meta, a)
    got = _decode(meta, chunks, dt)
    want = a.copy()
    if sharded:  # inner chunks [0:4, 0:8], [4:8, 0:8], [8:12, 8:16] elided → read as +0.0
        want[0:4, 0:8] = 0.0
        want[4:8, 0:8] = 0.0
    else:        # chunks [0:4, 0:8] and [4:8, 0:8] elided (their keys deleted)
        assert chunks[0] is None and chunks[2] is None
        want[0:8, 0:8] = 0.0
    np.testing.assert_array_equal(got.view(np.uint8), want.view(np.uint8))
    assert not np.signbit(got[0:8, 0:8]).any()


@pytest.mark.parametrize("sharded", [False, True])
def test_oracle_nan_fill_never_elides(sharded):
    meta = _meta("<f4", np.nan, sharded)
    a = _array("<f4", np.nan)
    a[:] = np.nan
    chunks = encode_oracle(meta, a)
    assert all(c is not None for c in chunks)  # NaN == NaN is false: every chunk written
    np.testing.assert_array_equal(_decode(meta, chunks, "<f4").view(np.uint32), a.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("sharded", [False, True])
@pytest.mark.parametrize("dt", ["<f4", "<f8"])
def test_device_zero_fill_matches_oracle_bytes(dev, dt, sharded):
    meta = _meta(dt, -0.0 if sharded else 0.0, sharded)
    a = _array(dt, 0.0)
    assert device_write(dev, meta, a) == encode_oracle(meta, a)


@pytest.mark.gpu
@pytest.mark.parametrize("sharded", [False, True])
@pytest.mark.parametrize("dt", ["<f4", "<f8"])
def test_device_nan_fill_matches_oracle_bytes(dev, dt, sharded):
    """A NaN fill equals nothing: every chunk and inner chunk is written, the boundary shard's
    pure-padding inner chunks included (rows 12-15 of the second shard), byte for byte as the
    oracle; an elided inner chunk would read back as 0, not NaN (Q1)."""
    meta = _meta(dt, np.nan, sharded)
    a = _array(dt, np.nan)
    got = device_write(dev, meta, a)
    assert got == encode_oracle(meta, a)
    assert all(c is not None for c in got)
    np.testing.assert_array_equal(device_read(dev, meta, got, [0, 0], SHAPE).view(np.uint8),
                                  a.view(np.uint8))
