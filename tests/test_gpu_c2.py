"""BASELINE configs[1] (c2) at its own geometry, scaled down: unsharded [bytes(big)] chunks
whose rows are 1024 uint32 (4 KiB), so the row kernel moves 2 MiB work items of 512 rows, and
the chunks of the last column hold 512 of their 1024 elements in bounds (the row-clipped items
the row kernel takes itself since round 2).  The bench checks the full-size array only as an
encode → decode round trip; here the device decode is compared with the oracle's
`core.Array.read` (M/core/Array.java:427-433 → BytesCodec.decode, M/core/codec/core/
BytesCodec.java:15-35) and the device encode with the oracle's shard bytes
(BytesCodec.encode :38-78), on regions that cut both chunk columns."""
import numpy as np
import pytest

import oracle as O
from helpers import chunk_coords, device_read, device_write, encode_oracle, rand_array
from zarrhip import _abi as A
from zarrhip._lib import lib

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _multi_launch(monkeypatch):
    """These tests assert which fast kernel ran (zh_debug_last_fast_path): keep small plans on
    the multi-launch kernels whatever the environment says (ZH_SMALL_ONE, conftest)."""
    monkeypatch.setenv("ZH_SMALL_ONE", "0")

SHAPE = [1, 32, 64, 1536]
CHUNK = [1, 16, 32, 1024]


def _meta():
    return A.make_meta(SHAPE, CHUNK, 4, endian=A.ZH_ENDIAN_BIG)


def _fast_path():
    """(fast_mode, row_group, pieces split) of the last decode scatter launch."""
    fp = lib().zh_debug_last_fast_path(0)
    return (fp // 10**6) % 1000, (fp % 1000) // 4, fp % 2


@pytest.mark.parametrize("small_split", ["0", None])
def test_c2_geometry_decode_and_encode(dev, monkeypatch, small_split):
    """small_split "0": whole 2 MiB chunks are the work items, as at full size (32 chunks ×
    2048 pieces there, so the small-read split never applies); None: the default knobs at
    this size, which split the 8 chunks further for the launch width."""
    for k in ("ZH_PIECE_KB", "ZH_PIPE"):
        monkeypatch.delenv(k, raising=False)
    if small_split is None:
        monkeypatch.delenv("ZH_SMALL_SPLIT", raising=False)
    else:
        monkeypatch.setenv("ZH_SMALL_SPLIT", small_split)
    meta = _meta()
    arr = rand_array(SHAPE, 4, seed=2024)
    arr[arr == 0] = 1  # no all-fill chunk: every chunk is stored
    shards = encode_oracle(meta, arr)
    assert len(shards) == 8 and all(s is not None for s in shards)
    # boundary chunks (x-index 1): 512 of 1024 elements per row in bounds, stored padded
    assert all(len(s) == 16 * 32 * 1024 * 4 for s in shards)
    assert device_write(dev, meta, arr) == shards
    pos = {c: i for i, c in enumerate(chunk_coords(meta, [0, 0, 0, 0], SHAPE))}
    regions = [([0, 0, 0, 0], SHAPE),                 # the whole array
               ([0, 3, 5, 700], [1, 27, 50, 820]),    # cuts both chunk columns
               ([0, 16, 32, 1024], [1, 16, 32, 512]),  # exactly the clipped chunk
               ([0, 0, 0, 1000], [1, 32, 64, 536])]   # the column boundary to the array end
    for off, shp in regions:
        sel = chunk_coords(meta, off, shp)
        src = [shards[pos[c]] for c in sel]
        want = np.frombuffer(O.array_read(meta, src, off, shp), np.uint32).reshape(shp)
        got = device_read(dev, meta, src, off, shp)
        np.testing.assert_array_equal(got, want)
        np.testing.assert_array_equal(
            got, arr[:, off[1]:off[1] + shp[1], off[2]:off[2] + shp[2], off[3]:off[3] + shp[3]])
        if off == [0, 0, 0, 0]:
            mode, group, split = _fast_path()
            # decode_rows_kernel (rows along the unit-stride dim, no chunk groups); whole
            # chunks as the work items unless the small-read split is on
            assert mode in (1, 2) and group == 0
            if small_split == "0":
                assert split == 0
