"""Chunk crc32c fused into the transpose tile kernel (decode_tiles_kernel<..., CRC=true>):
[transpose, bytes(big), crc32c] inner chains whose unclipped uint32 chunks take the 32x32
LDS-tile fast path.  Bit-exact against the oracle (decoded values, mismatch message) across
piece splits and transpose orders, with an elided inner chunk, a missing shard and a clipped
region (slow items keep the standalone CRC pass)."""
import numpy as np
import pytest

import oracle as O
from helpers import chunk_coords, device_read, device_write, encode_oracle, rand_array
from zarrhip import _abi as A
from zarrhip._lib import ZhError, lib

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _multi_launch(monkeypatch):
    """These tests assert which fast kernel ran (zh_debug_last_fast_path): keep small plans on
    the multi-launch kernels whatever the environment says (ZH_SMALL_ONE, conftest)."""
    monkeypatch.setenv("ZH_SMALL_ONE", "0")

SHAPE = [64, 64, 96]
CHUNK = 32 * 32 * 32 * 4 + 4  # stored inner chunk: payload + crc32c


def _meta(order):
    return A.make_meta(SHAPE, [32, 64, 64], 4, endian=A.ZH_ENDIAN_BIG, sharded=True,
                       inner_chunk_shape=[32, 32, 32], transpose_order=order, inner_crc32c=True)


def _read_both(dev, meta, shards, off, shp):
    sel = chunk_coords(meta, off, shp)
    pos = {c: i for i, c in enumerate(chunk_coords(meta, [0, 0, 0], SHAPE))}
    srcs = [shards[pos[c]] for c in sel]
    want = np.frombuffer(O.array_read(meta, srcs, off, shp), np.uint32).reshape(shp)
    return device_read(dev, meta, srcs, off, shp), want


def _variant():
    """Kernel variant of the last decode scatter launch (zh_debug_last_fast_path)."""
    return (lib().zh_debug_last_fast_path(0) // 1000) % 1000


def _corrupt_matches_oracle(dev, meta, shards, k, pos):
    bad = bytearray(shards[k])
    bad[pos] ^= 0x20
    srcs = list(shards)
    srcs[k] = bytes(bad)
    with pytest.raises(O.OracleError) as eo:
        O.array_read(meta, srcs, [0, 0, 0], SHAPE)
    with pytest.raises(ZhError) as ed:
        device_read(dev, meta, srcs, [0, 0, 0], SHAPE)
    assert str(ed.value) == str(eo.value)


@pytest.mark.parametrize("order", [[0, 2, 1], [2, 0, 1], [1, 2, 0], [2, 1, 0]])
@pytest.mark.parametrize("piece_kb", [128, 16, 4])
@pytest.mark.parametrize("fuse", ["1", "0"])
def test_chunk_crc32c_fused_tile_kernel(dev, monkeypatch, order, piece_kb, fuse):
    monkeypatch.setenv("ZH_PIECE_KB", str(piece_kb))
    monkeypatch.setenv("ZH_CRC_FUSE", fuse)
    meta = _meta(order)
    arr = rand_array(SHAPE, 4, seed=41)
    arr[0:32, 0:32, 0:32] = 0     # an elided inner chunk (Q1 zeros)
    shards = encode_oracle(meta, arr)
    shards[3] = None              # a missing shard (fill)
    for off, shp in [([0, 0, 0], SHAPE), ([5, 3, 7], [50, 60, 80])]:
        got, want = _read_both(dev, meta, shards, off, shp)
        np.testing.assert_array_equal(got, want)
    _corrupt_matches_oracle(dev, meta, shards, 0, 70000)  # first stored chunk: a fast item


@pytest.mark.parametrize("order", [[0, 2, 1], [2, 0, 1], [2, 1, 0]])
def test_row_crc_tile_kernel_is_the_default(dev, monkeypatch, order):
    """Without switches a whole-chunk [transpose, bytes(big), crc32c] read runs
    tiles_rowcrc_kernel at G = 1 (variant 51) and matches the oracle; a flipped payload byte
    in the middle of a chunk is reported with the oracle's message."""
    monkeypatch.setenv("ZH_SMALL_SPLIT", "0")
    meta = _meta(order)
    arr = rand_array(SHAPE, 4, seed=57)
    shards = encode_oracle(meta, arr)
    got, want = _read_both(dev, meta, shards, [0, 0, 0], SHAPE)
    np.testing.assert_array_equal(got, want)
    assert _variant() == 51
    _corrupt_matches_oracle(dev, meta, shards, 0, CHUNK + 65536 + 77)


@pytest.mark.parametrize("split", ["0", "1"])
def test_tile_crc_pieces_item_order(dev, monkeypatch, split):
    """Chunks cut into 32 KiB pieces (the per-chunk row-interleaved tile kernel with the chunk
    CRC fused, walked in the golden-ratio item order) give the same bytes, with and without the
    small-plan split; corruption of the last payload byte of a shard's last inner chunk is
    caught."""
    monkeypatch.setenv("ZH_SMALL_SPLIT", split)
    monkeypatch.setenv("ZH_PIECE_KB", "32")
    meta = _meta([2, 1, 0])
    arr = rand_array(SHAPE, 4, seed=43)
    shards = encode_oracle(meta, arr)
    got, want = _read_both(dev, meta, shards, [0, 0, 0], SHAPE)
    np.testing.assert_array_equal(got, want)
    np.testing.assert_array_equal(got, arr)
    # shard (1,0,0) holds 4 inner chunks; flip a bit of the 4th one's last payload byte
    _corrupt_matches_oracle(dev, meta, shards, 2, 3 * CHUNK + CHUNK - 5)


@pytest.mark.parametrize("order", [[0, 2, 1], [2, 1, 0], [1, 2, 0]])
@pytest.mark.parametrize("split", ["0", "1"])
@pytest.mark.parametrize("crc", [True, False])
def test_grouped_tile_decode(dev, monkeypatch, order, split, crc):
    """tiles_group_kernel in the decode direction (4 chunks per work item, 2 tiles of each per
    step, the next step's loads before this step's stores); with the chunk CRC the row-CRC tile
    kernel at one chunk per work item.  With the small-plan split (ZH_SMALL_SPLIT=1: this
    8-chunk read is cut into pieces) the per-chunk row-interleaved kernels run instead, CRC
    fused.  An elided inner chunk, a missing shard, a clipped region; a corrupt byte of a fast
    chunk is caught."""
    monkeypatch.setenv("ZH_SMALL_SPLIT", split)
    meta = A.make_meta(SHAPE, [32, 64, 64], 4, endian=A.ZH_ENDIAN_BIG, sharded=True,
                       inner_chunk_shape=[32, 32, 32], transpose_order=order, inner_crc32c=crc)
    arr = rand_array(SHAPE, 4, seed=47)
    arr[32:64, 0:32, 32:64] = 0
    shards = encode_oracle(meta, arr)
    shards[2] = None
    want_variant = 1 if split == "1" else 51 if crc else 24
    for off, shp in [([0, 0, 0], SHAPE), ([5, 3, 7], [50, 60, 80])]:
        got, want = _read_both(dev, meta, shards, off, shp)
        np.testing.assert_array_equal(got, want)
        if off == [0, 0, 0]:
            assert _variant() == want_variant
    if crc:
        _corrupt_matches_oracle(dev, meta, shards, 1, CHUNK + 1000)


@pytest.mark.parametrize("order", [[0, 2, 1], [2, 1, 0], [1, 2, 0], [2, 0, 1]])
@pytest.mark.parametrize("endian", [A.ZH_ENDIAN_BIG, A.ZH_ENDIAN_LITTLE])
def test_row_crc_tile_decode_endian(dev, monkeypatch, order, endian):
    """tiles_rowcrc_kernel over both byte orders (big endian: byte-swapped tables, the register
    carried swapped): same bytes as the oracle with an elided chunk, a missing shard and a
    clipped region; corruption in a chunk's first payload row, in a middle row and in its last
    byte is reported with the oracle's message."""
    monkeypatch.setenv("ZH_SMALL_SPLIT", "0")
    meta = A.make_meta(SHAPE, [32, 64, 64], 4, endian=endian, sharded=True,
                       inner_chunk_shape=[32, 32, 32], transpose_order=order, inner_crc32c=True)
    arr = rand_array(SHAPE, 4, seed=53)
    arr[32:64, 0:32, 32:64] = 0
    shards = encode_oracle(meta, arr)
    shards[2] = None
    for off, shp in [([0, 0, 0], SHAPE), ([5, 3, 7], [50, 60, 80])]:
        got, want = _read_both(dev, meta, shards, off, shp)
        np.testing.assert_array_equal(got, want)
        if off == [0, 0, 0]:
            assert _variant() == 51
    full = encode_oracle(meta, arr)  # shard 0: four in-bounds chunks of random data
    for pos in (3, CHUNK + 1000, 2 * CHUNK + 70001, CHUNK - 5):
        _corrupt_matches_oracle(dev, meta, full, 0, pos)


def test_row_crc_tile_kernel_many_groups(dev, monkeypatch):
    """The c4crc chain ([transpose [0,3,2,1], bytes(big), crc32c], 32³ uint32 inner chunks) at
    64 MiB: 512 inner chunks over 8 shards, the golden-ratio group order and the default
    row-CRC tile kernel; equals the oracle, and a flipped byte deep inside the last shard is
    reported with the oracle's message."""
    monkeypatch.delenv("ZH_SMALL_SPLIT", raising=False)
    shape = [1, 256, 256, 256]
    meta = A.make_meta(shape, [1, 128, 128, 128], 4, endian=A.ZH_ENDIAN_BIG, sharded=True,
                       inner_chunk_shape=[1, 32, 32, 32], transpose_order=[0, 3, 2, 1],
                       inner_crc32c=True)
    arr = rand_array(shape, 4, seed=59)
    arr[arr == 0] = 1
    shards = encode_oracle(meta, arr)
    # the tile encode with the fused chunk CRC (2 chunks per work item) at this size
    assert device_write(dev, meta, arr) == shards
    assert (lib().zh_debug_last_fast_path(1) % 1000000) // 1000 == 2
    want = np.frombuffer(O.array_read(meta, shards, [0, 0, 0, 0], shape), np.uint32).reshape(shape)
    got = device_read(dev, meta, shards, [0, 0, 0, 0], shape)  # pipelined (128 MiB host side)
    np.testing.assert_array_equal(got, want)
    np.testing.assert_array_equal(got, arr)
    monkeypatch.setenv("ZH_PIPE", "0")  # one plan over the whole array: the kernel it selects
    np.testing.assert_array_equal(device_read(dev, meta, shards, [0, 0, 0, 0], shape), arr)
    assert _variant() == 51
    bad = list(shards)
    k = len(bad) - 1
    b = bytearray(bad[k])
    b[37 * CHUNK + 99999] ^= 0x01
    bad[k] = bytes(b)
    with pytest.raises(O.OracleError) as eo:
        O.array_read(meta, bad, [0, 0, 0, 0], shape)
    with pytest.raises(ZhError) as ed:
        device_read(dev, meta, bad, [0, 0, 0, 0], shape)
    assert str(ed.value) == str(eo.value)


@pytest.mark.parametrize("units,order", [(5, [0, 2, 1]), (3, [0, 2, 1]), (12, [0, 2, 1])])
def test_row_crc_tile_kernel_unit_layouts(dev, monkeypatch, units, order):
    """Row-CRC tile kernel over inner chunks of `units` 32x32 tiles: at most 8 units take the
    per-unit K multiply (no regular fold step: crc_tile_step 0), 12 units the regular fold
    over a partly filled last step.  Equals the oracle; a flipped byte in the last unit of a
    chunk is caught with the oracle's message."""
    monkeypatch.setenv("ZH_SMALL_SPLIT", "0")
    shape = [units * 2, 64, 96]
    meta = A.make_meta(shape, [units * 2, 64, 64], 4, endian=A.ZH_ENDIAN_BIG, sharded=True,
                       inner_chunk_shape=[units, 32, 32], transpose_order=order,
                       inner_crc32c=True)
    arr = rand_array(shape, 4, seed=61 + units)
    arr[arr == 0] = 1
    shards = encode_oracle(meta, arr)
    got, want = _read_both_shape(dev, meta, shards, shape)
    np.testing.assert_array_equal(got, want)
    np.testing.assert_array_equal(got, arr)
    assert _variant() == 51
    chunk = units * 32 * 32 * 4 + 4
    bad = list(shards)
    b = bytearray(bad[0])
    b[chunk + chunk - 4 - 700] ^= 0x40  # second chunk, inside its last unit
    bad[0] = bytes(b)
    with pytest.raises(O.OracleError) as eo:
        O.array_read(meta, bad, [0, 0, 0], shape)
    with pytest.raises(ZhError) as ed:
        device_read(dev, meta, bad, [0, 0, 0], shape)
    assert str(ed.value) == str(eo.value)


def _read_both_shape(dev, meta, shards, shape):
    want = np.frombuffer(O.array_read(meta, shards, [0, 0, 0], shape), np.uint32).reshape(shape)
    return device_read(dev, meta, shards, [0, 0, 0], shape), want


def _aligned():
    """Whether the last decode scatter launch took the aligned-window row-CRC kernel."""
    return lib().zh_debug_last_fast_path(0) // 10**9


@pytest.mark.parametrize("nb", [16, 24, 32])
@pytest.mark.parametrize("endian", [A.ZH_ENDIAN_BIG, A.ZH_ENDIAN_LITTLE])
def test_row_crc_aligned_windows(dev, monkeypatch, nb, endian):
    """tiles_rowcrc_aln_kernel: inner chunks [32, nb, 32] under transpose [2, 1, 0] store
    [32 rows][nb units][32 words] (c4's layout), so the movers load 128-B aligned lines and
    carry each step's last line into the next step's tile through a ring of 9 LDS slots.  One
    shard of 36 inner chunks puts the payloads at every offset 4i mod 128 (the head lines, the
    carried line ends and the row tails of every δ, and δ = 0; 2, 3 and 4 steps per chunk).  Equals the oracle over the
    whole array and a ragged region, with an elided chunk (the unaligned row-CRC kernel keeps
    the layouts this one does not take: test_row_crc_tile_kernel_unit_layouts and the other
    transpose orders); flipped bytes in a row tail (read at the last step from the box), in a
    carried line end and in a head line are reported with the oracle's message."""
    monkeypatch.setenv("ZH_SMALL_SPLIT", "0")
    shape = [64, 6 * nb, 96]
    meta = A.make_meta(shape, shape, 4, endian=endian, sharded=True,
                       inner_chunk_shape=[32, nb, 32], transpose_order=[2, 1, 0],
                       inner_crc32c=True)
    arr = rand_array(shape, 4, seed=67 + nb)
    arr[arr == 0] = 1
    arr[32:64, 0:nb, 0:32] = 0  # one elided inner chunk (shifts the later payloads by a chunk)
    shards = encode_oracle(meta, arr)
    got, want = _read_both_shape(dev, meta, shards, shape)
    np.testing.assert_array_equal(got, want)
    np.testing.assert_array_equal(got, arr)
    assert _variant() == 51 and _aligned() == 1
    off, shp = [3, 5, 7], [58, 6 * nb - 9, 80]
    sel = np.frombuffer(O.array_read(meta, shards, off, shp), np.uint32).reshape(shp)
    np.testing.assert_array_equal(device_read(dev, meta, shards, off, shp), sel)
    chunk = 32 * nb * 32 * 4 + 4
    row = nb * 128  # bytes of one payload row (all units)
    for i in (5, 31):  # δ = 20 and 124
        p = i * chunk
        for pos in (p + 11 * row - 3,            # row 10's tail (the box, last step)
                    p + 4 * row + 1024 + 2,      # row 4, step 1: a carried line end
                    p + 7 * row + 1):            # row 7's head line
            _corrupt_matches_oracle_shape(dev, meta, shards, 0, pos, shape)


def _corrupt_matches_oracle_shape(dev, meta, shards, k, pos, shape):
    bad = bytearray(shards[k])
    bad[pos] ^= 0x08
    srcs = list(shards)
    srcs[k] = bytes(bad)
    with pytest.raises(O.OracleError) as eo:
        O.array_read(meta, srcs, [0] * len(shape), shape)
    with pytest.raises(ZhError) as ed:
        device_read(dev, meta, srcs, [0] * len(shape), shape)
    assert str(ed.value) == str(eo.value)


def test_row_crc_chain_64mib_defaults(dev, monkeypatch):
    """The c3crc chain ([bytes(big), crc32c], 32³ uint32 inner chunks, no transpose) at 64 MiB
    with the default kernels of both directions: the grouped row-CRC encode (2 chunks per work
    item, payloads stored through the cache since round 3) gives the oracle's shard bytes, and
    the grouped row-CRC decode (cached payload loads) gives the array back; a flipped byte deep
    inside the last shard is reported with the oracle's message."""
    for k in ("ZH_SMALL_SPLIT", "ZH_PIPE"):
        monkeypatch.delenv(k, raising=False)
    shape = [1, 256, 256, 256]
    meta = A.make_meta(shape, [1, 128, 128, 128], 4, endian=A.ZH_ENDIAN_BIG, sharded=True,
                       inner_chunk_shape=[1, 32, 32, 32], inner_crc32c=True)
    arr = rand_array(shape, 4, seed=61)
    arr[arr == 0] = 1
    want = encode_oracle(meta, arr)
    got = device_write(dev, meta, arr)
    assert (lib().zh_debug_last_fast_path(1) % 1000000) // 1000 == 2  # row groups of 2
    assert got == want
    monkeypatch.setenv("ZH_PIPE", "0")  # one plan over the whole array
    np.testing.assert_array_equal(device_read(dev, meta, want, [0, 0, 0, 0], shape), arr)
    assert (lib().zh_debug_last_fast_path(0) % 1000) // 4 == 2  # decode row groups of 2
    bad = list(want)
    k = len(bad) - 1
    b = bytearray(bad[k])
    b[45 * CHUNK + 77777] ^= 0x10
    bad[k] = bytes(b)
    with pytest.raises(O.OracleError) as eo:
        O.array_read(meta, bad, [0, 0, 0, 0], shape)
    with pytest.raises(ZhError) as ed:
        device_read(dev, meta, bad, [0, 0, 0, 0], shape)
    assert str(ed.value) == str(eo.value)


@pytest.mark.parametrize("order", [None, [0, 3, 2, 1]])
def test_plain_chains_64mib_defaults(dev, monkeypatch, order):
    """c3 / c4 chains without the chunk CRC ([(transpose [0,3,2,1],) bytes(big)], 32³ uint32
    inner chunks) at 64 MiB through the default kernels: the grouped encodes give the oracle's
    shard bytes, and the decode (lane exchange for c3, tile groups for c4) gives the array
    back, also for a region that cuts every shard."""
    for k in ("ZH_SMALL_SPLIT", "ZH_PIPE"):
        monkeypatch.delenv(k, raising=False)
    shape = [1, 256, 256, 256]
    meta = A.make_meta(shape, [1, 128, 128, 128], 4, endian=A.ZH_ENDIAN_BIG, sharded=True,
                       inner_chunk_shape=[1, 32, 32, 32], transpose_order=order)
    arr = rand_array(shape, 4, seed=67)
    arr[arr == 0] = 1
    want = encode_oracle(meta, arr)
    assert device_write(dev, meta, arr) == want
    monkeypatch.setenv("ZH_PIPE", "0")
    np.testing.assert_array_equal(device_read(dev, meta, want, [0, 0, 0, 0], shape), arr)
    off, shp = [0, 40, 8, 100], [1, 200, 240, 140]
    sel = chunk_coords(meta, off, shp)
    pos = {c: i for i, c in enumerate(chunk_coords(meta, [0, 0, 0, 0], shape))}
    got = device_read(dev, meta, [want[pos[c]] for c in sel], off, shp)
    np.testing.assert_array_equal(got, arr[0:1, 40:240, 8:248, 100:240])


@pytest.mark.parametrize("order", [[0, 2, 1], [2, 1, 0], [1, 2, 0]])
def test_tile_crc_encode_groups(dev, monkeypatch, order):
    """The tile encode with the fused chunk CRC over 2 chunks per work item: byte-identical to
    the oracle's shards (an all-fill chunk elided, so the later payloads shift), and the kernel
    that ran is that group size."""
    meta = _meta(order)
    arr = rand_array(SHAPE, 4, seed=97)
    arr[0:32, 32:64, 0:32] = 0
    want = encode_oracle(meta, arr)
    got = device_write(dev, meta, arr)
    assert got == want
    assert (lib().zh_debug_last_fast_path(1) % 1000000) // 1000 == 2


@pytest.mark.parametrize("row,group", [(64, 1), (32, 2), (16, 4)])
def test_row_crc_encode_groups(dev, monkeypatch, row, group):
    """The row encode with the fused chunk CRC ([bytes(big), crc32c], no transpose) groups
    256 B of region row per wave: 1, 2 and 4 chunks per work item for 256-, 128- and 64-B
    inner chunk rows, payloads stored through the cache: byte-identical to the oracle's
    shards (an all-fill chunk elided, so later payloads shift)."""
    meta = A.make_meta(SHAPE, [32, 64, 64], 4, endian=A.ZH_ENDIAN_BIG, sharded=True,
                       inner_chunk_shape=[32, 32, row], inner_crc32c=True)
    arr = rand_array(SHAPE, 4, seed=101)
    arr[32:64, 0:32, 0:64] = 0  # whole inner chunks for every row length
    want = encode_oracle(meta, arr)
    assert device_write(dev, meta, arr) == want
    assert (lib().zh_debug_last_fast_path(1) % 1000000) // 1000 == group


@pytest.mark.parametrize("start", [False, True])
def test_index_crc_span_combine(dev, monkeypatch, start):
    """The index crc32c with the span partials combined by the last workgroup: reads equal the
    oracle, a flipped index byte gives the oracle's message, and the write path stores the
    same index checksums (index at the end or at the start, an index of 4 KiB spans plus a
    tail)."""
    shape = [1, 96, 200, 160]
    meta = A.make_meta(shape, [1, 96, 100, 160], 4, endian=A.ZH_ENDIAN_BIG, sharded=True,
                       inner_chunk_shape=[1, 4, 4, 160], index_crc32c=True,
                       index_location=A.ZH_INDEX_START if start else A.ZH_INDEX_END)
    arr = rand_array(shape, 4, seed=103)
    shards = encode_oracle(meta, arr)
    assert device_write(dev, meta, arr) == shards
    np.testing.assert_array_equal(device_read(dev, meta, shards, [0, 0, 0, 0], shape), arr)
    isz = 16 * (96 // 4) * (100 // 4) + 4
    for k, pos in ((0, 5 if start else len(shards[0]) - isz + 4099), (1, isz // 2 if start else len(shards[1]) - 7)):
        bad = list(shards)
        b = bytearray(bad[k])
        b[pos] ^= 0x40
        bad[k] = bytes(b)
        with pytest.raises(O.OracleError) as eo:
            O.array_read(meta, bad, [0, 0, 0, 0], shape)
        with pytest.raises(ZhError) as ed:
            device_read(dev, meta, bad, [0, 0, 0, 0], shape)
        assert str(ed.value) == str(eo.value)


@pytest.mark.parametrize("loc", [A.ZH_INDEX_END, A.ZH_INDEX_START])
@pytest.mark.parametrize("elide", [False, True])
def test_crc_tile_encode_every_word_offset(dev, loc, elide):
    """The chunk-CRC tile encode at every payload word offset: c4crc's payload layout ([32
    rows][32 units][32 words] under transpose [2, 1, 0]) with 9 inner chunks per shard, so the
    payloads after each 4-byte crc32c start at every word offset mod 8 (index at the end; at
    the start the index shifts them again); an elided all-fill chunk sends its shard through
    the second pass with the host's layout.  Every byte of every shard (the buffers are
    poisoned first) equals the oracle's and the shards decode back (round 6 ran it against the
    sector-aligned store variant too before removing it, profiles/r06/aln/)."""
    shape = [64, 32 * 9, 32]
    meta = A.make_meta(shape, [32, 32 * 9, 32], 4, endian=A.ZH_ENDIAN_BIG, sharded=True,
                       inner_chunk_shape=[32, 32, 32], transpose_order=[2, 1, 0],
                       inner_crc32c=True, index_location=loc)
    arr = rand_array(shape, 4, seed=211)
    arr[arr == 0] = 1
    if elide:
        arr[32:64, 96:128, :] = 0  # one all-fill inner chunk of the second shard
    want = encode_oracle(meta, arr)
    got = device_write(dev, meta, arr)
    assert [len(g) if g else 0 for g in got] == [len(w) if w else 0 for w in want]
    assert got == want
    assert (lib().zh_debug_last_fast_path(1) % 1000000) // 1000 == 2  # the CRC tile encode
    np.testing.assert_array_equal(
        device_read(dev, meta, got, [0, 0, 0], shape), arr)
