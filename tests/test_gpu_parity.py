"""HIP path vs the CPU oracle (bit-exact), through the C-ABI.  Mirrors the reference's
own tests: ZarrV3Test testEndianness / testTransposeCodec / testShardingReadWrite /
testUnalignedArrayAccess / testLargerChunkSizeThanArraySize, ParallelWriteTest shapes,
and the ZarrPythonTests codec configurations (parse_codecs.py:104-116)."""
import itertools

import numpy as np
import pytest

import oracle as O
from helpers import (chunk_coords, device_read, device_write, encode_oracle, load_reference_fixture,
                     rand_array, shape_of)
from zarrhip import _abi as A
from zarrhip._lib import lib, ZhError

pytestmark = pytest.mark.gpu


def roundtrip(dev, meta, arr, regions):
    shards = encode_oracle(meta, arr)
    n = meta.ndim
    for off, shp in regions:
        srcs = [shards[i] for i in range(len(shards))]
        coords_all = chunk_coords(meta, [0] * n, shape_of(meta))
        sel = chunk_coords(meta, off, shp)
        pos = {c: i for i, c in enumerate(coords_all)}
        src_sel = [srcs[pos[c]] for c in sel]
        want = np.frombuffer(O.array_read(meta, src_sel, off, shp),
                             dtype=arr.dtype).reshape(shp)
        got = device_read(dev, meta, src_sel, off, shp)
        np.testing.assert_array_equal(got, want)
        sl = tuple(slice(o, o + s) for o, s in zip(off, shp))
        np.testing.assert_array_equal(got, arr[sl])
    return shards


def test_reference_fixtures_decode_to_arange(dev):
    for loc in ("start", "end"):
        _, meta, srcs = load_reference_fixture(loc)
        got = device_read(dev, meta, srcs, [0, 0, 0], [16, 16, 16])
        np.testing.assert_array_equal(got.astype(np.int64).ravel(), np.arange(4096))
        got2 = device_read(dev, meta, srcs, [3, 5, 1], [9, 7, 14])
        np.testing.assert_array_equal(got2.astype(np.int64),
                                      np.arange(4096).reshape(16, 16, 16)[3:12, 5:12, 1:15])


@pytest.mark.parametrize("fuse", ["1", "0"])
@pytest.mark.parametrize("loc,stored_crc", [("end", 0xB756D1D4), ("start", 0x56F05363)])
def test_device_crc_on_reference_index_bytes(dev, monkeypatch, loc, stored_crc, fuse):
    """The device index-CRC kernel on the reference fixture's own, untouched 68-byte index
    (testdata/sharding_index_location, Crc32cCodec.decode, Crc32cCodec.java:24-48).  With
    only the stored crc zeroed, the device must report Computed = the crc the reference
    stored; with the index intact the CRC passes and the read stops at the next stage (the
    blosc-framed inner chunks are not raw `bytes`), exactly as the oracle does.  Both forms
    of the index check: inside the slow kernel's launch (ZH_IDX_CRC_FUSE=1, the default) and
    its own launch ahead of the resolve kernel (0)."""
    monkeypatch.setenv("ZH_IDX_CRC_FUSE", fuse)
    import os
    import struct
    from helpers import GOLDEN
    _, meta, _ = load_reference_fixture(loc)
    raw = open(os.path.join(GOLDEN, "sharding_index_location", loc, "c", "0", "0", "0"),
               "rb").read()
    cpos = 64 if loc == "start" else len(raw) - 4
    assert struct.unpack("<I", raw[cpos:cpos + 4])[0] == stored_crc
    zeroed = raw[:cpos] + b"\0\0\0\0" + raw[cpos + 4:]
    signed = struct.unpack("<i", struct.pack("<I", stored_crc))[0]
    with pytest.raises(ZhError) as ed:
        device_read(dev, meta, [zeroed], [0, 0, 0], [16, 8, 8])
    assert str(ed.value) == ("The checksum of the sharding index is invalid. Stored: 0 "
                             f"Computed: {signed}")
    with pytest.raises(O.OracleError) as eo:
        O.array_read(meta, [zeroed], [0, 0, 0], [16, 8, 8])
    assert str(eo.value) == str(ed.value)
    with pytest.raises(ZhError) as ed2:
        device_read(dev, meta, [raw], [0, 0, 0], [16, 8, 8])
    with pytest.raises(O.OracleError) as eo2:
        O.array_read(meta, [raw], [0, 0, 0], [16, 8, 8])
    # Q12: both reject the 1040-byte framed chunk (the texts differ in detail)
    for e in (ed2.value, eo2.value):
        assert str(e).startswith("unexpected inner chunk byte length")


@pytest.mark.parametrize("fuse", ["1", "0"])
@pytest.mark.parametrize("loc", ["end", "start"])
def test_index_crc_multi_span_jobs(dev, monkeypatch, loc, fuse):
    """Index crc32c over jobs of several spans each (64 KiB indexes: 16 workgroups of 4 KiB per
    shard, combined by the job's last workgroup), in both launch forms (ZH_IDX_CRC_FUSE):
    intact indexes read equal to the data for an aligned region (no slow items: the fused
    launch is CRC workgroups only) and a clipped one (CRC beside the slow list); one shard's
    stored crc flipped fails with the oracle's message, whichever region touches it, and a
    region that avoids that shard reads."""
    monkeypatch.setenv("ZH_IDX_CRC_FUSE", fuse)
    meta = A.make_meta([128, 64, 64], [64, 64, 64], 4, sharded=True, inner_chunk_shape=[4, 4, 4],
                       index_location=A.ZH_INDEX_START if loc == "start" else A.ZH_INDEX_END)
    data = np.arange(128 * 64 * 64, dtype=np.uint32).reshape(128, 64, 64) * np.uint32(2654435761)
    shards = device_write(dev, meta, data)
    assert [bytes(x) for x in shards] == [bytes(x) for x in encode_oracle(meta, data)]
    regions = [([0, 0, 0], [128, 64, 64]), ([3, 5, 1], [67, 55, 62]), ([70, 0, 0], [10, 64, 64])]

    def pick(srcs, off, shp):  # the shards a region references, in chunk-coordinate order
        return [srcs[c[0]] for c in chunk_coords(meta, off, shp)]
    for off, shp in regions:
        want = data[tuple(slice(o, o + n) for o, n in zip(off, shp))]
        np.testing.assert_array_equal(device_read(dev, meta, pick(shards, off, shp), off, shp),
                                      want)
    cpos = 64 * 1024 if loc == "start" else len(shards[1]) - 4
    bad = bytearray(shards[1])
    bad[cpos] ^= 0x5A
    srcs = [shards[0], bytes(bad)]
    for off, shp in regions:
        with pytest.raises(ZhError) as ed:
            device_read(dev, meta, pick(srcs, off, shp), off, shp)
        with pytest.raises(O.OracleError) as eo:
            O.array_read(meta, pick(srcs, off, shp), off, shp)
        assert str(ed.value) == str(eo.value)
        assert str(ed.value).startswith("The checksum of the sharding index is invalid. Stored: ")
    np.testing.assert_array_equal(device_read(dev, meta, srcs[:1], [0, 0, 0], [64, 64, 64]),
                                  data[:64])


@pytest.mark.parametrize("fuse", ["1", "0"])
@pytest.mark.parametrize("dsize", [1, 2, 4, 8])
def test_small_read_one_launch(dev, monkeypatch, dsize, fuse):
    """BASELINE configs[0]'s call shape in the library's default small-plan form
    (ZH_SMALL_ONE=1: resolve + decode of every item in one launch, the index CRC in the same
    launch or, ZH_IDX_CRC_FUSE=0, its own): c4's chain (transpose [0,3,2,1], bytes(big), 32³
    inner chunks) at 64³ regions of 27 inner chunks, 26 of them clipped, one aligned region,
    a missing inner chunk (Q1: zero) and the plan size at the one-launch limit (64 chunks)."""
    monkeypatch.setenv("ZH_SMALL_ONE", "1")
    monkeypatch.setenv("ZH_IDX_CRC_FUSE", fuse)
    shape = [1, 128, 128, 128]
    meta = A.make_meta(shape, [1, 64, 128, 64], dsize, endian=A.ZH_ENDIAN_BIG, sharded=True,
                       inner_chunk_shape=[1, 32, 32, 32], transpose_order=[0, 3, 2, 1])
    arr = rand_array(shape, dsize, seed=31 + dsize)
    arr[0, 32:64, 32:64, 64:96] = 0  # an all-fill inner chunk: elided, read back as 0 (Q1)
    roundtrip(dev, meta, arr, [([0, 3, 17, 21], [1, 64, 64, 64]), ([0, 0, 0, 0], shape),
                               ([0, 33, 1, 40], [1, 64, 64, 64]), ([0, 0, 0, 0], [1, 128, 64, 128]),
                               ([0, 5, 5, 5], [1, 1, 1, 1])])
    assert lib().zh_debug_last_fast_path(0) == -1  # the one-launch kernel ran


def test_small_one_byte_bound(dev, monkeypatch):
    """Few but large chunks stay on the fast kernels (kSmallOneBytes = 16 MiB): 3 unsharded
    chunks of 8 MiB take the row kernel, 2 of them (16 MiB) the one launch."""
    monkeypatch.setenv("ZH_SMALL_ONE", "1")
    shape = [3, 1024, 2048]
    meta = A.make_meta(shape, [1, 1024, 2048], 4, endian=A.ZH_ENDIAN_BIG)
    arr = rand_array(shape, 4, seed=5)
    roundtrip(dev, meta, arr, [([0, 0, 0], shape)])
    assert lib().zh_debug_last_fast_path(0) != -1
    roundtrip(dev, meta, arr, [([1, 0, 0], [2, 1024, 2048])])
    assert lib().zh_debug_last_fast_path(0) == -1


@pytest.mark.parametrize("loc,stored_crc", [("end", 0xB756D1D4), ("start", 0x56F05363)])
def test_device_chunk_crc_on_reference_bytes(dev, loc, stored_crc):
    """The inner-chunk crc32c path (Crc32cCodec.encode/decode, Crc32cCodec.java:24-60, run as
    an inner codec) pinned to reference-produced bytes: an inner chunk whose 64-byte payload
    is the reference fixture's index body must carry the crc the reference stored for it;
    that chunk decodes, and with the crc flipped the read reports the reference message."""
    import os
    import struct
    from helpers import GOLDEN
    raw = open(os.path.join(GOLDEN, "sharding_index_location", loc, "c", "0", "0", "0"),
               "rb").read()
    body = raw[:64] if loc == "start" else raw[len(raw) - 68:len(raw) - 4]
    data = np.frombuffer(body, "<u4").reshape(4, 4)
    meta = A.make_meta([4, 4], [4, 4], 4, endian=A.ZH_ENDIAN_LITTLE, sharded=True,
                       inner_chunk_shape=[4, 4], inner_crc32c=True)
    shard = device_write(dev, meta, data)[0]
    assert shard[:64] == body
    assert struct.unpack("<I", shard[64:68])[0] == stored_crc
    assert shard == encode_oracle(meta, data)[0]
    np.testing.assert_array_equal(device_read(dev, meta, [shard], [0, 0], [4, 4]), data)
    bad = shard[:64] + struct.pack("<I", stored_crc ^ 1) + shard[68:]
    signed = struct.unpack("<i", struct.pack("<I", stored_crc))[0]
    with pytest.raises(ZhError) as ed:
        device_read(dev, meta, [bad], [0, 0], [4, 4])
    assert str(ed.value) == ("The checksum of the sharding index is invalid. Stored: "
                             f"{signed ^ 1} Computed: {signed}")


@pytest.mark.parametrize("zext", [24, 20, 22, 17, 32])
@pytest.mark.parametrize("dsize", [2, 4, 8])
@pytest.mark.parametrize("sharded", [False, True])
def test_row_clipped_items(dev, zext, dsize, sharded):
    """Items cut only along the unit-stride dim (c2's boundary chunks: 512 of 1024 z in
    bounds) go through the row kernel with narrower rows when the in-bounds prefix is a
    power-of-two number of 16-B vectors (z 24 / 20 with 16-wide chunks), else the generic
    kernel (22, 17); regions that end inside the last chunk along z only, too."""
    shape = [1, 8, 12, zext]
    if sharded:
        meta = A.make_meta(shape, [1, 8, 12, 32], dsize, endian=A.ZH_ENDIAN_BIG, sharded=True,
                           inner_chunk_shape=[1, 4, 4, 16])
    else:
        meta = A.make_meta(shape, [1, 4, 4, 16], dsize, endian=A.ZH_ENDIAN_BIG)
    arr = rand_array(shape, dsize, seed=zext + dsize)
    roundtrip(dev, meta, arr, [([0, 0, 0, 0], shape), ([0, 0, 0, 0], [1, 8, 12, 8]),
                               ([0, 4, 0, 0], [1, 4, 12, min(zext, 20)]),
                               ([0, 1, 0, 0], [1, 7, 12, zext])])


@pytest.mark.parametrize("dsize", [1, 2, 4, 8])
@pytest.mark.parametrize("endian", [A.ZH_ENDIAN_LITTLE, A.ZH_ENDIAN_BIG])
def test_unsharded_bytes(dev, dsize, endian):
    shape = [16, 16, 16]
    meta = A.make_meta(shape, [2, 4, 8], dsize, endian=endian)
    arr = rand_array(shape, dsize, seed=dsize + endian)
    roundtrip(dev, meta, arr, [([0, 0, 0], shape), ([1, 3, 5], [10, 9, 11])])


@pytest.mark.parametrize("dsize", [1, 2, 4, 8])
@pytest.mark.parametrize("endian", [A.ZH_ENDIAN_LITTLE, A.ZH_ENDIAN_BIG])
@pytest.mark.parametrize("loc", [A.ZH_INDEX_END, A.ZH_INDEX_START])
def test_sharded(dev, dsize, endian, loc):
    shape = [16, 16, 16]
    meta = A.make_meta(shape, [8, 8, 8], dsize, endian=endian, sharded=True,
                       inner_chunk_shape=[2, 4, 8], index_location=loc)
    arr = rand_array(shape, dsize, seed=3 * dsize + endian, fill_frac=0.0)
    roundtrip(dev, meta, arr, [([0, 0, 0], shape), ([1, 3, 5], [10, 9, 11]), ([8, 8, 8], [8, 8, 8])])


@pytest.mark.parametrize("order", list(itertools.permutations(range(4))))
def test_sharded_transpose_all_orders(dev, order):
    shape = [2, 24, 20, 36]
    meta = A.make_meta(shape, [2, 16, 8, 32], 4, endian=A.ZH_ENDIAN_BIG, sharded=True,
                       inner_chunk_shape=[1, 8, 4, 16], transpose_order=list(order))
    arr = rand_array(shape, 4, seed=sum(o * 10 ** i for i, o in enumerate(order)))
    roundtrip(dev, meta, arr, [([0, 0, 0, 0], shape), ([1, 3, 2, 5], [1, 17, 15, 30])])


@pytest.mark.parametrize("order", [[2, 1, 0], [1, 2, 0], [0, 2, 1], [1, 0, 2]])
@pytest.mark.parametrize("dsize", [1, 2, 8])
def test_unsharded_transpose(dev, order, dsize):
    shape = [40, 33, 70]
    meta = A.make_meta(shape, [32, 32, 64], dsize, endian=A.ZH_ENDIAN_BIG,
                       transpose_order=order)
    arr = rand_array(shape, dsize, seed=7)
    roundtrip(dev, meta, arr, [([0, 0, 0], shape), ([5, 1, 9], [30, 31, 60])])


def test_large_tiles_transpose_c4_shape(dev):
    """BASELINE config 4 shapes at reduced extent: inner 1x32x32x32, order [0,3,2,1]."""
    shape = [1, 128, 96, 80]
    meta = A.make_meta(shape, [1, 64, 64, 64], 4, endian=A.ZH_ENDIAN_BIG, sharded=True,
                       inner_chunk_shape=[1, 32, 32, 32], transpose_order=[0, 3, 2, 1])
    arr = rand_array(shape, 4, seed=11)
    roundtrip(dev, meta, arr, [([0, 0, 0, 0], shape), ([0, 7, 33, 5], [1, 100, 60, 70])])


def test_missing_inner_chunks_are_zero_and_missing_shards_fill(dev):
    """Q1: a missing inner chunk reads 0 even with a non-zero fill; a missing shard reads
    fill_value (ShardingIndexedCodec.java:189,219-221; Array.java:400-402,419-421)."""
    shape = [16, 16]
    fill = np.uint32(7)
    meta = A.make_meta(shape, [8, 8], 4, fill=int(fill).to_bytes(4, "little"), sharded=True,
                       inner_chunk_shape=[4, 4])
    arr = rand_array(shape, 4, seed=5)
    arr[0:4, 0:4] = fill      # all-fill inner chunk → (-1,-1) in the index
    arr[8:16, 8:16] = fill    # all-fill shard → deleted
    shards = encode_oracle(meta, arr)
    assert shards[3] is None
    got = device_read(dev, meta, shards, [0, 0], shape)
    want = np.frombuffer(O.array_read(meta, shards, [0, 0], shape), dtype=np.uint32).reshape(shape)
    np.testing.assert_array_equal(got, want)
    assert (got[0:4, 0:4] == 0).all()          # Q1
    assert (got[8:16, 8:16] == fill).all()


def test_boundary_chunks_larger_than_array(dev):
    """testLargerChunkSizeThanArraySize / boundary shards with padding."""
    shape = [10, 21, 13]
    meta = A.make_meta(shape, [16, 16, 16], 2, endian=A.ZH_ENDIAN_BIG, sharded=True,
                       inner_chunk_shape=[4, 8, 4], transpose_order=[1, 2, 0])
    arr = rand_array(shape, 2, seed=13)
    roundtrip(dev, meta, arr, [([0, 0, 0], shape), ([9, 20, 12], [1, 1, 1]), ([2, 3, 4], [8, 18, 9])])


def test_bool(dev):
    shape = [9, 17]
    meta = A.make_meta(shape, [4, 8], 1, is_bool=True, sharded=True, inner_chunk_shape=[2, 4])
    arr = (rand_array(shape, 1, seed=3) % 2).astype(np.uint8)
    roundtrip(dev, meta, arr, [([0, 0], shape)])


def test_crc_mismatch_message(dev):
    shape = [8, 8]
    meta = A.make_meta(shape, [8, 8], 4, sharded=True, inner_chunk_shape=[4, 4])
    arr = rand_array(shape, 4, seed=1)
    shards = encode_oracle(meta, arr)
    bad = bytearray(shards[0])
    bad[-10] ^= 0x40  # flip an index byte (inside the crc'd range)
    with pytest.raises(O.OracleError) as eo:
        O.array_read(meta, [bytes(bad)], [0, 0], shape)
    with pytest.raises(ZhError) as ed:
        device_read(dev, meta, [bytes(bad)], [0, 0], shape)
    assert str(ed.value) == str(eo.value)
    assert str(ed.value).startswith("The checksum of the sharding index is invalid. Stored: ")


@pytest.mark.parametrize("loc", [A.ZH_INDEX_END, A.ZH_INDEX_START])
def test_index_crc_multi_span_unaligned(dev, loc):
    """Index CRC over several 4 KiB spans, the index at a byte offset that is not a multiple
    of 4 (3-byte inner chunks, index at the end) or at 0 (start): decode equals the oracle,
    and a flipped byte in the third span gives the reference's checksum message."""
    shape = [41, 63]
    meta = A.make_meta(shape, [41, 63], 1, sharded=True, inner_chunk_shape=[1, 3],
                       index_location=loc)
    arr = rand_array(shape, 1, seed=8)
    arr[arr == 0] = 1
    shards = encode_oracle(meta, arr)
    got = device_read(dev, meta, shards, [0, 0], shape)
    np.testing.assert_array_equal(got, arr)
    isz = 16 * 41 * 21
    bad = bytearray(shards[0])
    ib = 0 if loc == A.ZH_INDEX_START else len(bad) - isz - 4
    bad[ib + 2 * 4096 + 77] ^= 0x10
    with pytest.raises(O.OracleError) as eo:
        O.array_read(meta, [bytes(bad)], [0, 0], shape)
    with pytest.raises(ZhError) as ed:
        device_read(dev, meta, [bytes(bad)], [0, 0], shape)
    assert str(ed.value) == str(eo.value)


def test_corrupt_offset_rejected(dev):
    shape = [8, 8]
    meta = A.make_meta(shape, [8, 8], 4, sharded=True, inner_chunk_shape=[4, 4],
                       index_crc32c=False)
    arr = rand_array(shape, 4, seed=1)
    shards = encode_oracle(meta, arr)
    bad = bytearray(shards[0])
    isz = 16 * 4
    ib = len(bad) - isz
    bad[ib + 16: ib + 24] = (10 ** 9).to_bytes(8, "little")  # entry 1 offset far out of range
    with pytest.raises(ZhError) as ed:
        device_read(dev, meta, [bytes(bad)], [0, 0], shape)
    with pytest.raises(O.OracleError) as eo:
        O.array_read(meta, [bytes(bad)], [0, 0], shape)
    assert str(ed.value) == str(eo.value) == "Could not load byte data for chunk [0, 1]"


def _shuffle_shard(meta, shard, rng, gap=True, dup=True):
    """Rewrite one shard with its inner chunks in a random order (Q7: the reference appends
    them in a nondeterministic order, ShardingIndexedCodec.java:116-147), random gaps between
    them, and (dup) two index entries sharing one payload; index rewritten with its crc32c."""
    import struct
    n = meta.ndim
    ch = meta.chain
    cps = 1
    for d in range(n):
        cps *= meta.chunk_shape[d] // ch.inner_chunk_shape[d]
    crc = bool(ch.index_has_crc32c)
    isz = 16 * cps + (4 if crc else 0)
    start = ch.index_location == A.ZH_INDEX_START
    fmt = ">QQ" if ch.index_endian == A.ZH_ENDIAN_BIG else "<QQ"
    ib = shard[:isz] if start else shard[len(shard) - isz:]
    ents = [struct.unpack(fmt, ib[16 * k:16 * k + 16]) for k in range(cps)]
    order = rng.permutation(cps)
    body, new = bytearray(), [None] * cps
    base = isz if start else 0
    for k in order:
        off, nb = ents[k]
        if off == 2 ** 64 - 1:
            new[k] = (off, nb)
            continue
        if gap:
            body += bytes(rng.integers(0, 256, int(rng.integers(0, 40)), dtype=np.uint8))
        new[k] = (base + len(body), nb)
        body += shard[off:off + nb]
    if dup:  # a later entry reuses an earlier payload: same bytes, read twice
        live = [k for k in range(cps) if new[k][0] != 2 ** 64 - 1]
        if len(live) >= 2:
            a, b = live[0], live[1]
            if shard[ents[a][0]:ents[a][0] + ents[a][1]] == shard[ents[b][0]:ents[b][0] + ents[b][1]]:
                new[b] = new[a]
    idx = b"".join(struct.pack(fmt, *e) for e in new)
    if crc:
        idx += struct.pack("<I", O.crc32c(idx))
    return (idx + bytes(body)) if start else (bytes(body) + idx)


@pytest.mark.parametrize("loc", [A.ZH_INDEX_END, A.ZH_INDEX_START])
@pytest.mark.parametrize("order", [None, [0, 3, 2, 1]])
def test_shuffled_inner_order_is_index_driven(dev, loc, order):
    """shards whose inner chunks sit in a random order with gaps decode
    exactly as the C-order shards do — the device follows the index, never the layout."""
    rng = np.random.default_rng(17)
    shape = [1, 24, 20, 40]
    meta = A.make_meta(shape, [1, 16, 16, 32], 4, endian=A.ZH_ENDIAN_BIG, sharded=True,
                       inner_chunk_shape=[1, 4, 4, 8], transpose_order=order,
                       index_location=loc)
    arr = rand_array(shape, 4, seed=23)
    arr[0, :4, :4, :8] = 0                    # one all-fill inner chunk: missing entry
    shards = encode_oracle(meta, arr)
    mixed = [None if s is None else _shuffle_shard(meta, s, rng) for s in shards]
    for off, shp in [([0, 0, 0, 0], shape), ([0, 3, 5, 7], [1, 18, 13, 30])]:
        sel = chunk_coords(meta, off, shp)
        pos = {c: i for i, c in enumerate(chunk_coords(meta, [0] * 4, shape))}
        src = [mixed[pos[c]] for c in sel]
        got = device_read(dev, meta, src, off, shp)
        want = np.frombuffer(O.array_read(meta, src, off, shp), np.uint32).reshape(shp)
        np.testing.assert_array_equal(got, want)
        np.testing.assert_array_equal(got, arr[tuple(slice(o, o + s) for o, s in zip(off, shp))])


def test_domain_error(dev):
    meta = A.make_meta([8, 8], [4, 4], 4)
    with pytest.raises(ZhError) as ed:
        device_read(dev, meta, [None], [6, 6], [4, 4])
    assert str(ed.value) == "Requested data is outside of the array's domain."


@pytest.mark.parametrize("sharded", [False, True])
@pytest.mark.parametrize("order", [None, [2, 0, 1]])
@pytest.mark.parametrize("loc", [A.ZH_INDEX_END, A.ZH_INDEX_START])
def test_device_encode_matches_oracle_bytes(dev, sharded, order, loc):
    shape = [20, 24, 40]
    meta = A.make_meta(shape, [8, 16, 32], 4, endian=A.ZH_ENDIAN_BIG, sharded=sharded,
                       inner_chunk_shape=[4, 8, 16] if sharded else None, transpose_order=order,
                       index_location=loc, fill=(3).to_bytes(4, "little"))
    arr = rand_array(shape, 4, seed=17, fill_frac=0.0)
    arr[0:8, 0:16, 0:32] = 3     # a whole chunk of fill → deleted
    arr[8:12, 0:8, 0:16] = 3     # an inner chunk of fill → (-1,-1)
    want = encode_oracle(meta, arr)
    got = device_write(dev, meta, arr)
    assert len(got) == len(want)
    for g, w in zip(got, want):
        assert g == w


@pytest.mark.parametrize("dsize", [1, 2, 4, 8])
@pytest.mark.parametrize("mode", ["unsharded", "sharded", "transpose_rows", "transpose_tiles",
                                  "crc32c"])
@pytest.mark.parametrize("loc", [A.ZH_INDEX_END, A.ZH_INDEX_START])
def test_device_encode_one_pass(dev, monkeypatch, dsize, mode, loc):
    """The one-pass write path (no all-fill chunk, so the speculative C-order layout holds):
    fast kernels on the encode view + the generic kernel for clipped chunks + device index and
    index crc32c.  Bytes equal the oracle's."""
    if mode == "unsharded" and loc == A.ZH_INDEX_START:
        pytest.skip("no index")
    shape = [40, 48, 72]          # boundary chunks on every axis
    kw = dict(endian=A.ZH_ENDIAN_BIG, index_location=loc,
              index_endian=A.ZH_ENDIAN_BIG if loc == A.ZH_INDEX_START else A.ZH_ENDIAN_LITTLE)
    if mode != "unsharded":
        kw.update(sharded=True, inner_chunk_shape=[8, 16, 32])
    if mode == "transpose_rows":
        kw.update(transpose_order=[1, 0, 2])      # keeps the last axis: row kernel
    if mode == "transpose_tiles":
        kw.update(transpose_order=[0, 2, 1])      # moves the last axis: tile kernel (u32)
    if mode == "crc32c":
        kw.update(inner_crc32c=True)
    meta = A.make_meta(shape, [16, 32, 64], dsize, fill=(7).to_bytes(dsize, "little"), **kw)
    arr = rand_array(shape, dsize, seed=31 + dsize)
    arr[arr == 7] = 8              # no element equals fill_value: nothing is elided
    want = encode_oracle(meta, arr)
    got = device_write(dev, meta, arr)
    assert [len(g) if g else 0 for g in got] == [len(w) if w else 0 for w in want]
    assert got == want


@pytest.mark.parametrize("dsize", [1, 2, 4, 8])
@pytest.mark.parametrize("order", [None, [1, 0, 2]])
def test_device_encode_grouped_rows(dev, dsize, order):
    """One-pass write with chunk rows of 1 KiB along the last axis split into inner chunks of
    64-128 B rows (many inner chunks adjacent along the region's unit-stride axis); boundary
    shards exercise the slow list beside the fast kernel."""
    last = 1024 // dsize
    inner_last = (64 if dsize <= 2 else 128) // dsize
    shape = [20, 24, last + last // 2 + inner_last // 2]
    meta = A.make_meta(shape, [8, 16, last], dsize, endian=A.ZH_ENDIAN_BIG, sharded=True,
                       inner_chunk_shape=[4, 8, inner_last], transpose_order=order)
    arr = rand_array(shape, dsize, seed=41 + dsize)
    arr[arr == 0] = 1
    want = encode_oracle(meta, arr)
    assert device_write(dev, meta, arr) == want


@pytest.mark.parametrize("crc", [False, True])
@pytest.mark.parametrize("dsize", [1, 4, 8])
@pytest.mark.parametrize("row", [32, 64, 128, 256])
def test_device_encode_chunk_groups(dev, monkeypatch, dsize, row, crc):
    """rows_group_kernel on the encode view (G consecutive inner chunks per work item so a wave
    covers 256 B of a region row: G = 8, 4, 2, 1 for 32-, 64-, 128- and 256-B inner chunk rows,
    at most 4 with the chunk CRC; 4 rows in flight per lane): an odd number of inner chunks along
    each shard row (groups straddle shard rows and the item list's end), all-fill chunks beside
    data chunks in one group (per-chunk flags from one ballot), clipped boundary chunks on the
    slow list.  crc: inner [bytes(big), crc32c], the chunk CRC fused into the grouped kernel
    where whole 4 KiB rounds allow (256/G lanes per chunk), else the CRC pass."""
    inner_last = row // dsize
    shape = [13, 24, inner_last * 7 + inner_last // 2]
    meta = A.make_meta(shape, [8, 8, inner_last * 5], dsize, endian=A.ZH_ENDIAN_BIG,
                       sharded=True, inner_chunk_shape=[4, 8, inner_last],
                       fill=(5).to_bytes(dsize, "little"), inner_crc32c=crc)
    arr = rand_array(shape, dsize, seed=53 + dsize)
    arr[arr == 5] = 6
    arr[0:4, 0:8, inner_last:2 * inner_last] = 5          # all-fill chunk next to data
    arr[4:8, 8:16, 0:3 * inner_last] = 5                  # a run of three
    arr[8:12, 0:8, 2 * inner_last:3 * inner_last] = 5
    arr[8:12, 0:8, 2 * inner_last + 1] = 9                # one element differs: kept
    want = encode_oracle(meta, arr)
    got = device_write(dev, meta, arr)
    assert [len(g) if g else 0 for g in got] == [len(w) if w else 0 for w in want]
    assert got == want


@pytest.mark.parametrize("loc", [A.ZH_INDEX_END, A.ZH_INDEX_START])
def test_device_encode_tile_groups(dev, monkeypatch, loc):
    """The grouped tile encode (tiles_group_kernel, 2 chunks per work item, 4 tiles of each per
    step): uint32 inner chunks transposed through 32x32 tiles, an odd number of chunks along
    each shard row, all-fill chunks inside groups, clipped boundary chunks."""
    shape = [40, 7, 32 * 7 + 16]
    meta = A.make_meta(shape, [32, 4, 32 * 5], 4, endian=A.ZH_ENDIAN_BIG, sharded=True,
                       inner_chunk_shape=[32, 2, 32], transpose_order=[2, 1, 0],
                       index_location=loc, fill=(5).to_bytes(4, "little"))
    arr = rand_array(shape, 4, seed=61)
    arr[arr == 5] = 6
    arr[0:32, 0:2, 32:64] = 5
    arr[0:32, 2:4, 0:96] = 5
    arr[0:32, 4:6, 64:96] = 5
    arr[7, 5, 70] = 9
    want = encode_oracle(meta, arr)
    got = device_write(dev, meta, arr)
    assert [len(g) if g else 0 for g in got] == [len(w) if w else 0 for w in want]
    assert got == want


@pytest.mark.parametrize("crc", [False, True])
@pytest.mark.parametrize("dsize", [1, 4, 8])
@pytest.mark.parametrize("row", [64, 128, 256])
def test_grouped_row_decode(dev, monkeypatch, crc, dsize, row):
    """The row decode kernels: with the chunk CRC rows_group_kernel (G = 4, 2, 1 consecutive
    inner chunks per work item for 64-, 128- and 256-B rows, per-lane-group descriptors, the
    fused chunk CRC over 256/G lanes per chunk), without it the lane exchange for 128-B rows and
    the per-chunk row kernel otherwise — copies beside Q1 zero-fill items (elided chunks) and a
    missing shard's fill, an odd chunk count per shard row, row-clipped boundary chunks sent to
    the generic kernel, a corrupt payload byte caught with the oracle's message."""
    inner_last = row // dsize
    shape = [13, 24, inner_last * 7 + inner_last // 2]
    meta = A.make_meta(shape, [8, 8, inner_last * 5], dsize, endian=A.ZH_ENDIAN_BIG,
                       sharded=True, inner_chunk_shape=[4, 8, inner_last],
                       fill=(5).to_bytes(dsize, "little"), inner_crc32c=crc)
    arr = rand_array(shape, dsize, seed=71 + dsize)
    arr[arr == 5] = 6
    arr[0:4, 0:8, inner_last:2 * inner_last] = 5          # elided → Q1 zeros on read
    shards = encode_oracle(meta, arr)
    pos = {c: i for i, c in enumerate(chunk_coords(meta, [0, 0, 0], shape))}
    shards[pos[(1, 1, 0)]] = None                          # missing shard → fill
    for off, shp in [([0, 0, 0], shape), ([1, 3, 5], [11, 20, shape[2] - 9])]:
        sel = chunk_coords(meta, off, shp)
        src = [shards[pos[c]] for c in sel]
        got = device_read(dev, meta, src, off, shp)
        want = np.frombuffer(O.array_read(meta, src, off, shp), arr.dtype).reshape(shp)
        np.testing.assert_array_equal(got, want)
    if crc:
        bad = bytearray(shards[0])
        bad[100] ^= 0x10
        src = [bytes(bad)] + shards[1:]
        with pytest.raises(O.OracleError) as eo:
            O.array_read(meta, src, [0, 0, 0], shape)
        with pytest.raises(ZhError) as ed:
            device_read(dev, meta, src, [0, 0, 0], shape)
        assert str(ed.value) == str(eo.value)


@pytest.mark.parametrize("inner_rows", [(4, 8), (2, 4), (3, 5)])
@pytest.mark.parametrize("dsize", [1, 4, 8])
@pytest.mark.parametrize("crc", [False, True])
def test_lane_exchange_row_decode(dev, monkeypatch, dsize, inner_rows, crc):
    """rows_xpose_kernel in the decode direction (128-B rows without the chunk CRC): copies
    beside Q1 zero-fill items and a missing shard's fill inside one group of 8 chunks,
    row-clipped boundary chunks on the generic kernel, partial regions; the fused-CRC and
    15-row chains fall back."""
    L = 128 // dsize
    a, b = inner_rows
    shape = [a * 3 + 1, b * 3, L * 9 + L // 2]
    meta = A.make_meta(shape, [a * 2, b * 2, L * 5], dsize, endian=A.ZH_ENDIAN_BIG,
                       sharded=True, inner_chunk_shape=[a, b, L],
                       fill=(5).to_bytes(dsize, "little"), inner_crc32c=crc)
    arr = rand_array(shape, dsize, seed=91 + dsize + a)
    arr[arr == 5] = 6
    arr[0:a, 0:b, L:2 * L] = 5                    # elided → Q1 zeros on read
    shards = encode_oracle(meta, arr)
    pos = {c: i for i, c in enumerate(chunk_coords(meta, [0, 0, 0], shape))}
    shards[pos[(1, 0, 1)]] = None                 # missing shard → fill
    for off, shp in [([0, 0, 0], shape), ([1, 1, 3], [shape[0] - 1, shape[1] - 2, shape[2] - 7])]:
        sel = chunk_coords(meta, off, shp)
        src = [shards[pos[c]] for c in sel]
        got = device_read(dev, meta, src, off, shp)
        want = np.frombuffer(O.array_read(meta, src, off, shp), arr.dtype).reshape(shp)
        np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("order", [[0, 3, 2, 1], [0, 1, 3, 2]])
def test_tile_encode_chunk_crc_fused(dev, monkeypatch, order):
    """c4crc-shaped chain at small extent: [transpose, bytes(big), crc32c] with 32x32 tiles,
    the chunk CRC fused into the tile encode (stored vectors, per-unit end shifts from the
    payload side of the table), boundary chunks through the slow list + CRC pass; equals the
    oracle and the unfused pass, and decodes back (the grouped tile encode: the unit fold step
    for 4 units)."""
    shape = [1, 64, 80, 96]
    meta = A.make_meta(shape, [1, 64, 64, 64], 4, endian=A.ZH_ENDIAN_BIG, sharded=True,
                       inner_chunk_shape=[1, 32, 32, 32], transpose_order=order,
                       inner_crc32c=True)
    arr = rand_array(shape, 4, seed=51)
    arr[arr == 0] = 1
    want = encode_oracle(meta, arr)
    assert device_write(dev, meta, arr) == want
    monkeypatch.setenv("ZH_CRC_FUSE", "0")
    assert device_write(dev, meta, arr) == want
    monkeypatch.delenv("ZH_CRC_FUSE")
    roundtrip(dev, meta, arr, [([0, 0, 0, 0], shape), ([0, 5, 7, 9], [1, 50, 60, 80])])


def test_device_encode_one_pass_fallback(dev):
    """A late all-fill inner chunk (seen only after the one-pass kernels ran) sends the write
    back through flags → layout → encode; the bytes still equal the oracle's."""
    shape = [32, 64]
    meta = A.make_meta(shape, [32, 64], 4, sharded=True, inner_chunk_shape=[8, 16],
                       endian=A.ZH_ENDIAN_BIG)
    arr = rand_array(shape, 4, seed=5)
    arr[arr == 0] = 1
    arr[24:32, 48:64] = 0          # the last inner chunk is all fill → (-1, -1)
    want = encode_oracle(meta, arr)
    assert device_write(dev, meta, arr) == want


def test_single_full_chunk_and_partial_decode_api(dev):
    """Array.java:392-395 single-full-chunk shortcut and ShardingIndexedCodec.decode /
    decodePartial through their own C-ABI entry points."""
    import ctypes as C
    shape = [32, 32]
    meta = A.make_meta(shape, [16, 16], 4, sharded=True, inner_chunk_shape=[4, 8],
                       endian=A.ZH_ENDIAN_BIG)
    arr = rand_array(shape, 4, seed=21)
    shards = encode_oracle(meta, arr)
    got = device_read(dev, meta, [shards[3]], [16, 16], [16, 16])
    np.testing.assert_array_equal(got, arr[16:, 16:])
    from zarrhip._lib import lib, i64arr, i32arr
    L = lib()
    sb = (C.c_char * len(shards[1])).from_buffer_copy(shards[1])
    out = (C.c_char * (16 * 16 * 4))()
    err = C.create_string_buffer(512)
    assert L.zh_sharding_decode(dev.h, C.byref(meta), sb, len(shards[1]), out, 0, None, err, 512) == 0
    np.testing.assert_array_equal(np.frombuffer(bytes(out), np.uint32).reshape(16, 16), arr[:16, 16:])
    out2 = (C.c_char * (5 * 7 * 4))()
    assert L.zh_sharding_decode_partial(dev.h, C.byref(meta), sb, len(shards[1]), i64arr([3, 4]),
                                        i32arr([5, 7]), out2, 0, None, err, 512) == 0
    np.testing.assert_array_equal(np.frombuffer(bytes(out2), np.uint32).reshape(5, 7),
                                  arr[3:8, 20:27])


@pytest.mark.parametrize("mode", ["unsharded", "sharded", "sharded_transpose", "nested"])
@pytest.mark.parametrize("dsize", [1, 4, 8])
def test_chunk_crc32c_decode_encode(dev, mode, dsize):
    """[transpose?, bytes, crc32c] chunk codecs on the device (data-CRC pass after resolve,
    CRC store pass after encode) vs the oracle: decoded values, encoded bytes, and regions."""
    shape = [24, 40, 36]
    kw = dict(endian=A.ZH_ENDIAN_BIG, inner_crc32c=True)
    if mode != "unsharded":
        kw.update(sharded=True, inner_chunk_shape=[8, 8, 12])
    if mode == "sharded_transpose":
        kw.update(transpose_order=[2, 0, 1])
    if mode == "nested":
        kw.update(nested_chunk_shape=[4, 8, 6])
    meta = A.make_meta(shape, [16, 16, 24], dsize, **kw)
    arr = rand_array(shape, dsize, seed=23)
    arr[0:8, 0:8, 0:12] = 0
    want = encode_oracle(meta, arr)
    got = device_write(dev, meta, arr)
    assert got == want
    roundtrip(dev, meta, arr, [([0, 0, 0], shape), ([3, 5, 7], [17, 30, 20]), ([20, 1, 30], [4, 9, 6])])


@pytest.mark.parametrize("sharded", [False, True])
def test_chunk_crc32c_mismatch_message(dev, sharded):
    shape = [16, 16]
    meta = A.make_meta(shape, [16, 16], 4, sharded=sharded,
                       inner_chunk_shape=[8, 8] if sharded else None, inner_crc32c=True)
    arr = rand_array(shape, 4, seed=2)
    b = bytearray(encode_oracle(meta, arr)[0])
    b[100] ^= 0x08
    with pytest.raises(O.OracleError) as eo:
        O.array_read(meta, [bytes(b)], [0, 0], shape)
    with pytest.raises(ZhError) as ed:
        device_read(dev, meta, [bytes(b)], [0, 0], shape)
    assert str(ed.value) == str(eo.value)


def test_chunk_crc32c_missing_and_clipped(dev):
    """Missing shards/inner chunks under a clipped region carry no source: the data-CRC pass
    must skip them (Q1 zeros, fill for a missing shard)."""
    shape = [20, 20]
    meta = A.make_meta(shape, [16, 16], 4, sharded=True, inner_chunk_shape=[8, 8],
                       inner_crc32c=True, fill=(9).to_bytes(4, "little"))
    arr = rand_array(shape, 4, seed=4)
    arr[0:8, 8:16] = 9            # an elided inner chunk
    shards = encode_oracle(meta, arr)
    shards[1] = None              # a missing shard
    off, shp = [3, 3], [15, 16]
    sel = chunk_coords(meta, off, shp)
    pos = {c: i for i, c in enumerate(chunk_coords(meta, [0, 0], shape))}
    srcs = [shards[pos[c]] for c in sel]
    want = np.frombuffer(O.array_read(meta, srcs, off, shp), np.uint32).reshape(shp)
    np.testing.assert_array_equal(device_read(dev, meta, srcs, off, shp), want)


@pytest.mark.parametrize("piece_kb", [128, 16, 4])
@pytest.mark.parametrize("fuse", ["1", "0"])
def test_chunk_crc32c_fused_row_kernel(dev, monkeypatch, piece_kb, fuse):
    """Chunk CRC fused into decode_rows_kernel (rows sequential in the payload, pieces of
    whole 4 KiB rounds): 64 KiB inner chunks in 1, 4 or 16 pieces, with elided chunks,
    a missing shard, a clipped region (slow items keep the standalone CRC pass), and a
    corrupted payload caught inside a fused item — vs the oracle and its message."""
    monkeypatch.setenv("ZH_PIECE_KB", str(piece_kb))
    monkeypatch.setenv("ZH_CRC_FUSE", fuse)
    shape = [64, 64, 96]
    meta = A.make_meta(shape, [32, 64, 64], 4, endian=A.ZH_ENDIAN_BIG, sharded=True,
                       inner_chunk_shape=[16, 32, 32], inner_crc32c=True)
    arr = rand_array(shape, 4, seed=29)
    arr[0:16, 0:32, 0:32] = 0
    shards = encode_oracle(meta, arr)
    shards[3] = None
    roundtrip_srcs = shards
    for off, shp in [([0, 0, 0], shape), ([5, 3, 7], [50, 60, 80])]:
        sel = chunk_coords(meta, off, shp)
        pos = {c: i for i, c in enumerate(chunk_coords(meta, [0, 0, 0], shape))}
        srcs = [roundtrip_srcs[pos[c]] for c in sel]
        want = np.frombuffer(O.array_read(meta, srcs, off, shp), np.uint32).reshape(shp)
        np.testing.assert_array_equal(device_read(dev, meta, srcs, off, shp), want)
    bad = bytearray(shards[0])
    bad[70000] ^= 0x20    # inside the second inner chunk's payload (a full, fast item)
    srcs = [bytes(bad)] + shards[1:]
    with pytest.raises(O.OracleError) as eo:
        O.array_read(meta, srcs, [0, 0, 0], shape)
    with pytest.raises(ZhError) as ed:
        device_read(dev, meta, srcs, [0, 0, 0], shape)
    assert str(ed.value) == str(eo.value)


@pytest.mark.parametrize("mode", ["rows", "tiles", "rows_crc"])
def test_item_permutation_order(dev, monkeypatch, mode):
    """Chunks cut into 16 KiB pieces, walked in the golden-ratio item order by the fast
    kernels: same bytes."""
    monkeypatch.setenv("ZH_PIECE_KB", "16")
    shape = [64, 64, 96]
    kw = dict(endian=A.ZH_ENDIAN_BIG, sharded=True, inner_chunk_shape=[16, 32, 32])
    if mode == "tiles":
        kw["transpose_order"] = [2, 1, 0]
    if mode == "rows_crc":
        kw["inner_crc32c"] = True
    meta = A.make_meta(shape, [32, 64, 64], 4, **kw)
    arr = rand_array(shape, 4, seed=31)
    roundtrip(dev, meta, arr, [([0, 0, 0], shape), ([3, 2, 1], [60, 61, 90])])


def _plan_read_host(dev, meta, srcs, off, shp):
    """zh_plan over HOST shard buffers (the mmap-style C-ABI use) → (array, staged bytes)."""
    import ctypes as C
    keep = [(C.c_char * max(1, len(s))).from_buffer_copy(s) if s is not None else None for s in srcs]
    plan = dev.plan(meta, [(C.addressof(k), len(s)) if s is not None else (None, 0)
                           for k, s in zip(keep, srcs)], off, shp, 0)
    try:
        staged = plan.staged_bytes()
        out = (C.c_char * (int(np.prod(shp)) * meta.dtype_size))()
        plan.execute(C.addressof(out))
        plan.wait()
        return np.frombuffer(bytes(out), np.uint32).reshape(shp), staged
    finally:
        plan.close()


def _shard_meta(**kw):
    return A.make_meta([64, 64, 64], [64, 64, 64], 4, endian=A.ZH_ENDIAN_BIG, sharded=True,
                       inner_chunk_shape=[8, 8, 8], **kw)


@pytest.mark.parametrize("loc", [A.ZH_INDEX_END, A.ZH_INDEX_START])
@pytest.mark.parametrize("ibe", [False, True])
def test_compact_staging_of_host_shards(dev, loc, ibe):
    """Host sources, sub-shard part: the planner stages the index + referenced inner chunks
    only (coalesced), rewriting the index; results equal the oracle's."""
    meta = _shard_meta(index_location=loc, index_endian=A.ZH_ENDIAN_BIG if ibe else A.ZH_ENDIAN_LITTLE)
    arr = rand_array([64, 64, 64], 4, seed=41)
    arr[8:16, 8:16, 8:16] = 0   # one elided inner chunk inside the part
    shard = encode_oracle(meta, arr)[0]
    for off, shp in [([5, 5, 5], [10, 10, 10]), ([0, 0, 0], [8, 64, 64]), ([60, 3, 0], [4, 9, 64]),
                     ([0, 0, 0], [64, 64, 32])]:
        want = np.frombuffer(O.array_read(meta, [shard], off, shp), np.uint32).reshape(shp)
        got, staged = _plan_read_host(dev, meta, [shard], off, shp)
        np.testing.assert_array_equal(got, want)
        assert staged < 0.6 * len(shard)
    got, staged = _plan_read_host(dev, meta, [shard], [0, 0, 0], [64, 64, 64])
    assert staged == len(shard)          # whole-shard reads keep one copy
    np.testing.assert_array_equal(got, arr)


def _reorder_shard(shard, meta, perm_seed):
    """Same shard, inner chunks stored in a shuffled order (index-driven decode, Q7)."""
    import struct
    n_in = 512
    isz = 16 * n_in + 4
    idx = shard[-isz:-4]
    ents = [struct.unpack("<QQ", idx[16 * k:16 * k + 16]) for k in range(n_in)]
    order = np.random.default_rng(perm_seed).permutation(n_in)
    payload, new = b"", [None] * n_in
    for k in order:
        off, nb = ents[k]
        if off == 2 ** 64 - 1:
            new[k] = (off, nb)
            continue
        new[k] = (len(payload), nb)
        payload += shard[off:off + nb]
    ib = b"".join(struct.pack("<QQ", *e) for e in new)
    return payload + ib + struct.pack("<I", O.crc32c(ib))


def test_compact_staging_shuffled_layout(dev):
    meta = _shard_meta()
    arr = rand_array([64, 64, 64], 4, seed=43)
    shard = _reorder_shard(encode_oracle(meta, arr)[0], meta, 5)
    for off, shp in [([9, 17, 33], [20, 30, 11]), ([0, 0, 0], [64, 8, 8])]:
        want = np.frombuffer(O.array_read(meta, [shard], off, shp), np.uint32).reshape(shp)
        got, staged = _plan_read_host(dev, meta, [shard], off, shp)
        np.testing.assert_array_equal(got, want)
        np.testing.assert_array_equal(got, arr[tuple(slice(o, o + s) for o, s in zip(off, shp))])
        assert staged < len(shard) / 2


def test_compact_staging_errors_match_oracle(dev):
    meta = _shard_meta()
    arr = rand_array([64, 64, 64], 4, seed=47)
    shard = encode_oracle(meta, arr)[0]
    off, shp = [1, 1, 1], [6, 6, 6]
    bad = bytearray(shard)
    bad[-20] ^= 0x01                      # index CRC
    bad_off = bytearray(shard)            # entry (0,0,0) offset beyond the shard
    bad_off[-(16 * 512 + 4):-(16 * 512 + 4) + 8] = (10 ** 9).to_bytes(8, "little")
    bad_off[-4:] = O.crc32c(bytes(bad_off[-(16 * 512 + 4):-4])).to_bytes(4, "little")
    for b in (bad, bad_off):
        with pytest.raises(O.OracleError) as eo:
            O.array_read(meta, [bytes(b)], off, shp)
        with pytest.raises(ZhError) as ed:
            _plan_read_host(dev, meta, [bytes(b)], off, shp)
        assert str(ed.value) == str(eo.value)


def test_plan_block_cache_reuse_and_release(dev):
    """Finished plans hand their device blocks to the context, later plans reuse them (no
    stale data leaks into results: every read below is checked), and zh_ctx_release_cache
    returns them to the runtime."""
    shape = [24, 40, 36]
    meta = A.make_meta(shape, [16, 16, 24], 4, endian=A.ZH_ENDIAN_BIG, sharded=True,
                       inner_chunk_shape=[8, 8, 12])
    arr = rand_array(shape, 4, seed=61)
    shards = encode_oracle(meta, arr)
    for off, shp in [([0, 0, 0], shape), ([3, 5, 7], [17, 30, 20]), ([0, 0, 0], shape)]:
        got = device_read(dev, meta, shards, off, shp)
        np.testing.assert_array_equal(got, arr[tuple(slice(o, o + s) for o, s in zip(off, shp))])
    assert dev.release_cache() > 0
    assert dev.release_cache() == 0
    got = device_read(dev, meta, shards, [0, 0, 0], shape)
    np.testing.assert_array_equal(got, arr)


@pytest.mark.parametrize("mode", ["sharded_transpose", "unsharded", "nested_crc"])
def test_array_write_host_buffers(dev, mode):
    """zh_array_write_host (the JNI write path: Java array in, byte[] chunks out) equals the
    oracle's encode, with elided inner chunks, a deleted all-fill chunk and boundary chunks."""
    shape = [20, 24, 40]
    kw = dict(endian=A.ZH_ENDIAN_BIG)
    if mode == "sharded_transpose":
        kw.update(sharded=True, inner_chunk_shape=[4, 8, 16], transpose_order=[2, 0, 1])
    if mode == "nested_crc":
        kw.update(sharded=True, inner_chunk_shape=[4, 8, 16], nested_chunk_shape=[2, 4, 8],
                  inner_crc32c=True)
    meta = A.make_meta(shape, [8, 16, 32], 4, **kw)
    arr = rand_array(shape, 4, seed=71)
    arr[arr == 0] = 1
    arr[0:8, 0:16, 0:32] = 0      # a whole chunk of fill → deleted
    arr[8:12, 0:8, 0:16] = 0      # an inner chunk of fill → (-1, -1)
    want = encode_oracle(meta, arr)
    got = dev.array_write_host(meta, arr.tobytes(), [0, 0, 0], shape, len(want))
    assert got == want


@pytest.mark.parametrize("case", [
    dict(shape=[1000], chunk=[256], inner=[64], order=None),
    dict(shape=[5, 6, 7, 8, 9], chunk=[4, 4, 4, 8, 8], inner=[2, 2, 4, 4, 8], order=[4, 0, 3, 1, 2]),
    dict(shape=[3, 2, 5, 2, 3, 4, 2, 6], chunk=[2, 2, 4, 2, 2, 4, 2, 4],
         inner=[1, 2, 2, 1, 2, 4, 1, 4], order=[7, 6, 5, 4, 3, 2, 1, 0]),
    dict(shape=[3, 2, 5, 2, 3, 4, 2, 6], chunk=[2, 2, 4, 2, 2, 4, 2, 4],
         inner=[1, 2, 2, 1, 2, 4, 1, 4], order=None),
], ids=["1d", "5d_transpose", "8d_reverse", "8d"])
@pytest.mark.parametrize("dsize", [1, 4])
def test_rank_1_to_8(dev, case, dsize):
    """Ranks 1, 5 and 8 (ZH_MAX_DIMS): sharded chains with and without transpose, whole and
    unaligned regions decoded bit-exactly, and the device encode equal to the oracle's."""
    shape, n = case["shape"], len(case["shape"])
    meta = A.make_meta(shape, case["chunk"], dsize, endian=A.ZH_ENDIAN_BIG, sharded=True,
                       inner_chunk_shape=case["inner"], transpose_order=case["order"])
    arr = rand_array(shape, dsize, seed=81 + n)
    arr[arr == 0] = 1
    off = [min(1, s - 1) for s in shape]
    shp = [s - o - (1 if s - o > 2 else 0) for s, o in zip(shape, off)]
    roundtrip(dev, meta, arr, [([0] * n, shape), (off, shp)])
    assert device_write(dev, meta, arr) == encode_oracle(meta, arr)


@pytest.mark.parametrize("case", ["sharded_transpose", "unsharded", "nested", "missing_shard"])
def test_host_output_slab_pipeline(dev, monkeypatch, case):
    """Large host reads go through the pipelined path (C-order slabs: H2D through the pinned
    ring | decode | D2H through the ring, zh_pipeline.cpp).  The thresholds are shrunk here so
    small arrays take that path: results equal the oracle, missing shards read fill_value, and
    a CRC error reports the reference's message."""
    monkeypatch.setenv("ZH_PIPE_MIN_KB", "1")
    monkeypatch.setenv("ZH_PIPE_SLAB_KB", "4")
    monkeypatch.setenv("ZH_PIPE_CHUNK_KB", "64")
    shape = [24, 40, 36]
    kw = dict(endian=A.ZH_ENDIAN_BIG, fill=(9).to_bytes(4, "little"))
    if case != "unsharded":
        kw.update(sharded=True, inner_chunk_shape=[8, 8, 12])
    if case == "sharded_transpose":
        kw.update(transpose_order=[2, 0, 1])
    if case == "nested":
        kw.update(nested_chunk_shape=[4, 8, 6])
    meta = A.make_meta(shape, [16, 16, 24], 4, **kw)
    arr = rand_array(shape, 4, seed=91)
    shards = encode_oracle(meta, arr)
    if case == "missing_shard":
        shards[1] = None
    for off, shp in [([0, 0, 0], shape), ([3, 5, 7], [17, 30, 20]), ([1, 0, 0], [1, 40, 36])]:
        coords_all = chunk_coords(meta, [0, 0, 0], shape)
        pos = {c: i for i, c in enumerate(coords_all)}
        srcs = [shards[pos[c]] for c in chunk_coords(meta, off, shp)]
        want = np.frombuffer(O.array_read(meta, srcs, off, shp), np.uint32).reshape(shp)
        np.testing.assert_array_equal(device_read(dev, meta, srcs, off, shp), want)
    if case == "sharded_transpose":
        bad = list(shards)
        b = bytearray(bad[2])
        b[-10] ^= 0x40
        bad[2] = bytes(b)
        with pytest.raises(O.OracleError) as eo:
            O.array_read(meta, bad, [0, 0, 0], shape)
        with pytest.raises(ZhError) as ed:
            device_read(dev, meta, bad, [0, 0, 0], shape)
        assert str(ed.value) == str(eo.value)


@pytest.mark.parametrize("sharded", [False, True])
def test_device_encode_subregion_offset(dev, sharded):
    """zh_array_write of a region of whole chunks away from the origin (the one-pass path
    with a non-zero region offset, one boundary chunk row): bytes equal the oracle's."""
    import ctypes as C
    from zarrhip._lib import lib
    shape = [40, 48, 70]
    meta = A.make_meta(shape, [8, 16, 32], 4, endian=A.ZH_ENDIAN_BIG, sharded=sharded,
                       inner_chunk_shape=[4, 8, 16] if sharded else None,
                       transpose_order=[0, 2, 1] if sharded else None)
    off, shp = [8, 16, 32], [24, 32, 38]     # chunks 1..3 x 1..2 x 1..2 (x clipped at 70)
    arr = rand_array(shp, 4, seed=101)
    arr[arr == 0] = 1
    want = O.array_write(meta, arr.tobytes(), off, shp)
    n = len(want)
    src = dev.malloc(arr.nbytes)
    dev.h2d(src, arr.tobytes())
    cap = lib().zh_array_encoded_bound(C.byref(meta))
    bufs = [dev.malloc(cap) for _ in range(n)]
    for b in bufs:
        dev.memset(b, 0xA5, cap)
    sizes = dev.array_write(meta, src, off, shp, [(b, cap) for b in bufs])
    got = [dev.d2h(b, sz) if sz else None for b, sz in zip(bufs, sizes)]
    for b in bufs:
        dev.free(b)
    dev.free(src)
    assert got == want


@pytest.mark.parametrize("loc", [A.ZH_INDEX_END, A.ZH_INDEX_START])
def test_truncated_shards_raise(dev, loc):
    """Fault injection: a shard cut inside its index is rejected by both paths
    (the reference's readSuffix would throw on the short buffer; no message to match); a
    shard whose payload is cut leaves index entries past the end, which both report with
    the reference's "Could not load byte data for chunk [..]"."""
    shape = [16, 16]
    meta = A.make_meta(shape, [16, 16], 4, sharded=True, inner_chunk_shape=[8, 8],
                       index_location=loc)
    arr = rand_array(shape, 4, seed=111)
    good = encode_oracle(meta, arr)[0]
    isz = 16 * 4 + 4
    cut = good[:isz - 3] if loc == A.ZH_INDEX_START else good[-(isz - 3):]
    with pytest.raises(O.OracleError):
        O.array_read(meta, [cut], [0, 0], shape)
    with pytest.raises(ZhError):
        device_read(dev, meta, [cut], [0, 0], shape)
    if loc == A.ZH_INDEX_END:
        short = good[:100] + good[-isz:]          # payload cut: entries point past the end
        with pytest.raises(O.OracleError) as eo:
            O.array_read(meta, [short], [0, 0], shape)
        with pytest.raises(ZhError) as ed:
            device_read(dev, meta, [short], [0, 0], shape)
        assert str(ed.value) == str(eo.value)
        assert str(ed.value).startswith("Could not load byte data for chunk")


def test_grouped_row_crc_decode_misaligned(dev, monkeypatch):
    """The grouped row-CRC decode (rows_group_kernel, G = 2, cached payload loads): misaligned
    payloads after each 4-byte crc32c, the same bytes as the oracle and a corrupt payload byte
    reported alike."""
    monkeypatch.setenv("ZH_SMALL_SPLIT", "0")  # whole chunks: the grouped kernel needs them
    shape = [64, 64, 96]
    meta = A.make_meta(shape, [32, 64, 64], 4, endian=A.ZH_ENDIAN_BIG, sharded=True,
                       inner_chunk_shape=[32, 32, 32], inner_crc32c=True)
    arr = rand_array(shape, 4, seed=83)
    shards = encode_oracle(meta, arr)
    got = device_read(dev, meta, shards, [0, 0, 0], shape)
    np.testing.assert_array_equal(got, arr)
    assert (lib().zh_debug_last_fast_path(0) % 1000) // 4 == 2  # row group 2
    k = max(range(len(shards)), key=lambda i: len(shards[i] or b""))  # a shard of 4 chunks
    bad = bytearray(shards[k])
    bad[3 * (32 * 32 * 32 * 4 + 4) + 4097] ^= 0x02  # chunk 3's payload: 4 mod 16 after 3 CRCs
    src = list(shards)
    src[k] = bytes(bad)
    with pytest.raises(O.OracleError) as eo:
        O.array_read(meta, src, [0, 0, 0], shape)
    with pytest.raises(ZhError) as ed:
        device_read(dev, meta, src, [0, 0, 0], shape)
    assert str(ed.value) == str(eo.value)


@pytest.mark.parametrize("order", [None, [2, 1, 0]])
def test_grouped_crc_encode_misaligned(dev, monkeypatch, order):
    """The grouped encodes with the fused chunk CRC (row kernel for [bytes, crc32c], payloads
    stored through the cache; tile kernel for [transpose, bytes, crc32c], non-temporal):
    byte-identical to the oracle's shards."""
    shape = [64, 64, 96]
    meta = A.make_meta(shape, [32, 64, 64], 4, endian=A.ZH_ENDIAN_BIG, sharded=True,
                       inner_chunk_shape=[32, 32, 32], transpose_order=order,
                       inner_crc32c=True)
    arr = rand_array(shape, 4, seed=89)
    arr[0:32, 0:32, 32:64] = 0  # an all-fill chunk: elided, the layout shifts
    want = encode_oracle(meta, arr)
    got = device_write(dev, meta, arr)
    assert got == want
